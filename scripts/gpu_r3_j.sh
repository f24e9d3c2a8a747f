# Round 3: contact tests + contact probe (timing and iteration histograms) with parked idle lanes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bullet.py tests/test_golden.py tests/test_gpu_wide.py tests/test_gpu_pid.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/contact_probe.py 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/contact.log || exit $?
done
GPD_LIB=gym_pybullet_drones_routing_amd/libgpd_stats.so timeout -k 10 300 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " > $OUT/contact_stats.log || exit $?
echo ALLDONE
