# Round 3: the PYB flag-set step kernels for MultiHoverAviary's default Physics.PYB and the
# single-drone PYB_GND_DRAG_DW: bullet GPU tests (incl. the resynced contact step test of every
# PYB flag-set step kernel), then the contact probe against the previous library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zc}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_bullet.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread -s > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for v in gpd gpd_prev; do
    echo "== $v rep $rep" >> $OUT/ab.log
    GPD_LIB=$P/lib$v.so timeout -k 10 200 python -u scripts/contact_probe.py crash multi multi2pyb 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/ab.log || exit $?
  done
done
echo ALLDONE
