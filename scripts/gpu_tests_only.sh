# GPU parity tests only (one pytest process), log under gpurun_out/tests/.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tests
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf ${PYTEST_ARGS} > gpurun_out/tests/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests/gpu_tests.log
exit $rc
