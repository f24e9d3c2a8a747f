# Round 3: targeted GPU tests (new boundary / reward / hand-off tests, Bullet contact parity with
# the register-resident solve), the contact A/B (old = HEAD solver, new = register solver) and the
# HBM ceiling sweep.  Each GPU step has its own timeout.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3b}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py tests/test_env_api.py tests/test_gpu_dist.py tests/test_gpu_bullet.py tests/test_golden.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for v in old new; do
    echo "== $v rep $rep" >> $OUT/ab_contact.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/contact_probe.py 2>&1 | grep -v amdgpu >> $OUT/ab_contact.log || exit $?
  done
done
timeout -k 10 300 ./scripts/ubench/hbm_ceiling > $OUT/hbm_ceiling.txt 2>&1 || exit $?
echo ALLDONE
