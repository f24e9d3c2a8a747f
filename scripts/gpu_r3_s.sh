# Round 3: contact solve v2 (exec-masked friction pairs, clamp as new - old, one-op residual max):
# bullet parity tests on the default library, then step-time A/B against v1 and a noinline
# solve, then the cycle counters (stats builds; f* = every solve forced to 50 iterations).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3s}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_bullet.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for v in gpd gpd_cv1 gpd_cv2ni; do
    echo "== $v rep $rep" >> $OUT/ab.log
    GPD_LIB=$P/lib$v.so timeout -k 10 200 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/ab.log || exit $?
  done
done
for v in sv1 sv2; do
  echo "== $v" >> $OUT/stats.log
  GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/stats.log || exit $?
done
for v in fv1 fv2 fv2ni; do
  echo "== $v" >> $OUT/stats.log
  GPD_LIB=$P/libgpd_$v.so timeout -k 10 200 python -u scripts/contact_probe.py rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/stats.log || exit $?
done
echo ALLDONE
