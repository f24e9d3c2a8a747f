cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6g
for rep in 1 2; do for v in ${POLICY_VARIANTS:-""}; do
  if [ -z "$v" ]; then L=gym_pybullet_drones_routing_amd/libgpd_policy.so; else L=gym_pybullet_drones_routing_amd/libgpd_policy_$v.so; fi
  GPD_POLICY_LIB=$L timeout -k 10 120 python -u scripts/policy_probe.py graph >> gpurun_out/r6g/polab.log 2>&1 || exit 1
done; done
GPD_POLICY_LIB=gym_pybullet_drones_routing_amd/libgpd_policy_tanh.so timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r6g/tanh_tests.log 2>&1
echo ALLDONE
