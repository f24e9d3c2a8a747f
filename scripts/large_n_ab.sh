# Large-N step A/B (round 3): cache-policy bits of the write-through stores, DMA issue point,
# store policies; graph-replayed 1M / 4M envs, variants alternated twice on one box.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3e}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in $LN_VARIANTS; do
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/large_n_probe.py 2>&1 | grep -v amdgpu >> $OUT/large_n.log || exit $?
  done
  PROBE_POLICIES=1 timeout -k 10 200 python -u scripts/large_n_probe.py 2>&1 | grep -v amdgpu >> $OUT/large_n.log || exit $?
  # the 4096-env store policy (PMC: write-through obs rows cost +0.29 MB per launch in the io kernel)
  PROBE_ENVS=4096 PROBE_POLICIES=2,3,1,4,0 PROBE_SCALES=1.0 timeout -k 10 200 python -u scripts/large_n_probe.py 2>&1 | grep -v amdgpu >> $OUT/policy_4096.log || exit $?
done
echo ALLDONE
