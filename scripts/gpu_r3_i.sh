# Round 3: store policy 2 vs 3 at 4096 envs (io kernel), 6 alternations; contact iteration
# histograms of the world-frame solve (GPD_CONTACT_STATS build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3i}
mkdir -p $OUT
for rep in 1 2 3; do
  PROBE_ENVS=4096 PROBE_POLICIES=2,3,2,3 PROBE_SCALES=1.0 timeout -k 10 200 python -u scripts/large_n_probe.py 2>&1 | grep -v amdgpu >> $OUT/policy_4096.log || exit $?
done
GPD_LIB=gym_pybullet_drones_routing_amd/libgpd_stats.so timeout -k 10 300 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " > $OUT/contact_stats.log || exit $?
echo ALLDONE
