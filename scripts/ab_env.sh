# A/B timing of one environment knob on one box: GPU tests first, then bench.py (no sweep, no
# CPU baseline) alternating AB_VAR=<value> over AB_VALS, at AB_ENVS envs per run.
#   AB_VAR=GPD_HIST_EARLY AB_VALS="0 1 0 1" AB_ENVS="4096 16384" bash scripts/ab_env.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab_${AB_VAR:-knob}
mkdir -p $OUT
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for E in ${AB_ENVS:-4096}; do
  for val in ${AB_VALS:-"0 1 0 1"}; do
    i=$((i+1))
    env ${AB_VAR:-GPD_NOTHING}=$val timeout -k 10 300 python bench.py --no-cpu-baseline --no-sweep --envs $E --steps ${AB_STEPS:-2000} --warmup 100 \
      > $OUT/run${i}_${E}_${val}.json 2> $OUT/run${i}_${E}_${val}.err || exit $?
  done
done
echo done
