# Quick GPU iteration: parity tests + latency probe + phase stamps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/quick/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/latency_probe.py > gpurun_out/quick/latency.log 2>&1 || exit $?
timeout -k 10 300 python scripts/stamp_probe.py > gpurun_out/quick/stamps.log 2>&1 || exit $?
echo done
