# Round-3 full run on the final code: GPU tests, smoke, bench, rocprofv3 kernel traces (bench config,
# then the large-N sweep) and PMC passes (FETCH_SIZE / WRITE_SIZE separately, kernel trace only).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3h}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --no-sweep --no-latency-model > $OUT/prof_bench_stdout.json 2> $OUT/prof_bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_sweep -o sweep --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof_sweep_stdout.json 2> $OUT/prof_sweep.err || exit $?
for E in 4096 65536 1048576 4194304; do
  S=50; [ $E -ge 1048576 ] && S=10
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$E -o fetch --output-format csv -- python3 scripts/prof_step.py --envs $E --steps $S > /dev/null 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$E -o write --output-format csv -- python3 scripts/prof_step.py --envs $E --steps $S > /dev/null 2>&1 || exit $?
done
echo ALLDONE
