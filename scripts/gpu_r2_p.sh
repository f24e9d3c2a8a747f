cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2p}
mkdir -p $OUT
timeout -k 10 300 python scripts/timing_probe.py > $OUT/timing.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > $OUT/bench_20.json 2> $OUT/bench_20.err || exit $?
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-sweep --no-cpu-baseline > $OUT/bench_300.json 2> $OUT/bench_300.err || exit $?
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-sweep > $OUT/bench_g2.json 2> $OUT/bench_g2.err || exit $?
timeout -k 10 300 python examples/learn.py --gpus 2 --dist-backend gloo --n_envs 512 --total_timesteps 40000 > $OUT/learn_g2.log 2>&1 || exit $?
echo ALLDONE
