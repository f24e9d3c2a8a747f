# Round 3: idle lanes on the block's first drone (blk) vs on drone 0 (nopark), contact probe
# alternated; then the GPU tests that cover thin blocks, wide envs and contact.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3l}
mkdir -p $OUT
P=gym_pybullet_drones_routing_amd
for rep in 1 2; do
  for v in nopark blk; do
    echo "== $v rep $rep" >> $OUT/contact.log
    GPD_LIB=$P/libgpd_$v.so timeout -k 10 300 python -u scripts/contact_probe.py crash rest multi 2>&1 | grep -v "amdgpu\|UserWarning\|sim = " >> $OUT/contact.log || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bullet.py tests/test_golden.py tests/test_gpu_wide.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
echo ALLDONE
