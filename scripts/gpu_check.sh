cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/precision_study.py > gpurun_out/precision.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
