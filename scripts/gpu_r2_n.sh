cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2n}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GEOM_CASES="2048,16,2 2048,16,3 4096,16,2 4096,16,3 8192,32,2 8192,32,3 16384,64,2 16384,64,3" timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > $OUT/bench_20.json 2> $OUT/bench_20.err || exit $?
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-sweep --no-cpu-baseline > $OUT/bench_300.json 2> $OUT/bench_300.err || exit $?
echo ALLDONE
