# Round 3: the raw integrator's RPM prefetch depth (substeps in flight ahead of use): 2 (default,
# libgpd.so) vs 4 / 6 (libgpd_ahead4/6.so), bench.py's raw-integrator leg alternated; then the
# integrate parity tests on the default build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zq}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2 3; do
  for lib in libgpd.so libgpd_ahead4.so libgpd_ahead6.so; do
    GPD_LIB=$P/$lib timeout -k 10 300 python -c "
import json, torch, bench
r = bench.raw_integrator(torch.device('cuda:0'), 'f64')
print('$lib', round(r['kernel_us'], 1), round(r['frac'], 3))" >> $OUT/raw.log 2>> $OUT/raw.err || exit $?
  done
done
echo ALLDONE
