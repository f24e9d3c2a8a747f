# Round 3: the downwash kernels' friction g vectors in LDS (GPD_CONTACT_FGL, libgpd.so) vs in
# VGPRs (libgpd_nofgl.so): bullet GPU tests, then the contact probe alternated.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zj}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_bullet.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2 3; do
  for v in gpd gpd_nofgl; do
    echo "== $v rep $rep" >> $OUT/ab.log
    GPD_LIB=$P/lib$v.so timeout -k 10 200 python -u scripts/contact_probe.py multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/ab.log || exit $?
  done
done
echo ALLDONE
