# Round 3: GPU tests + smoke + default bench line, one box.  Each GPU step has its own timeout.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo ALLDONE
