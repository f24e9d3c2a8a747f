# Round-2 first GPU pass: GPU tests, smoke, bench at the driver's shape and at 300 steps,
# the self-launched 2-rank rehearsal (gloo, one GPU), and the job's CPU share.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2a}
mkdir -p $OUT
python - > $OUT/cpus.txt 2>&1 <<'PY'
import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), "OMP", os.environ.get("OMP_NUM_THREADS"))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > $OUT/bench_20.json 2> $OUT/bench_20.err || exit $?
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-sweep --no-cpu-baseline > $OUT/bench_300.json 2> $OUT/bench_300.err || exit $?
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-sweep > $OUT/bench_g2.json 2> $OUT/bench_g2.err || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err || exit $?
echo ALLDONE
