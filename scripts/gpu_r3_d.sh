# Round 3: full GPU suite on the current code, then the 4096-env PMC itemization sweep.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3d}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 ./scripts/ubench/step_stream > $OUT/step_stream.txt 2>&1 || exit $?
RUN_TAG=r3d/pmc bash scripts/pmc_itemize.sh || exit $?
echo ALLDONE
