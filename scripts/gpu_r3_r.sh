# Round 3: the full-size GPU tests incl. the STREAM integrate bit-identity test.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3r}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
echo ALLDONE
exit $rc
