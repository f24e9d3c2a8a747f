# A/B of library builds on bench.py's raw-integrator line (1M drones x 32 substeps), alternating.
#   AB_RAW_LIBS="libgpd_old.so libgpd.so ..." bash scripts/ab_raw.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab_raw
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
i=0
for lib in ${AB_RAW_LIBS:-libgpd_old.so libgpd.so libgpd_old.so libgpd.so}; do
  i=$((i+1))
  GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$P/$lib timeout -k 10 300 python -c "
import json, torch, bench
print(json.dumps(bench.raw_integrator(torch.device('cuda:0'), 'f64')))" > $OUT/run${i}_$lib.json 2> $OUT/run${i}_$lib.err || exit $?
done
echo done
