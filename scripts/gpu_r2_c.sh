# Round-2: kernel-variant tests first (three-wave io kernel), then the geometry probe and a bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "step_parity_hover or duo_kernel" > $OUT/kern_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-sweep --no-cpu-baseline > $OUT/bench_300.json 2> $OUT/bench_300.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > $OUT/bench_20.json 2> $OUT/bench_20.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
echo "pytest rc=$?" >> $OUT/gpu_tests.log
echo ALLDONE
