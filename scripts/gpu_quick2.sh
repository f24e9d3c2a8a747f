# Quick kernel iteration: variant parity tests + geometry probe (+ optional bench).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-q}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "step_parity_hover or duo_kernel" > $OUT/kern_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.log 2>&1 || exit $?
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-sweep --no-cpu-baseline > $OUT/bench_300.json 2> $OUT/bench_300.err || exit $?
fi
echo ALLDONE
