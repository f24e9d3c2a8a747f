# Round 3: contact parity gates with the world-frame register solve, then the contact A/B
# (old = round-2 LDS solve, new = base-frame register solve, world = world-frame register solve).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3c}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_bullet.py tests/test_golden.py tests/test_env_api.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for v in old new world; do
    echo "== $v rep $rep" >> $OUT/ab_contact.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/contact_probe.py 2>&1 | grep -v amdgpu | grep -v "sim = \|UserWarning" >> $OUT/ab_contact.log || exit $?
  done
done
echo ALLDONE
