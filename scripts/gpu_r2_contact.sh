# GPU tests (one pytest process) + a bench pass without the CPU legs; logs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo ALLDONE
