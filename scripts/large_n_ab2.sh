# Large-N step A/B, round 3 second pass: sc1|nt write-through stores, + nt history DMA, + nt state
# loads, against the base build, from 4096 to 4M envs (graph replay, U[-1,1] actions).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3f}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in $LN_VARIANTS; do
    GPD_LIB=$P/libgpd_$v.so PROBE_ENVS=4096,65536,262144,1048576,4194304 PROBE_SCALES=1.0 timeout -k 10 240 python -u scripts/large_n_probe.py 2>&1 | grep -v amdgpu >> $OUT/large_n.log || exit $?
  done
done
echo ALLDONE
