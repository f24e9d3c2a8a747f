# One parameterised GPU-box runner (replaces the per-call scripts/gpu_r*_*.sh of rounds 1-3).
#   gpurun -- 'RUN_TAG=r4a bash scripts/gpu_job.sh <job> [job ...]'
# Jobs (each GPU step under its own timeout; the first failure ends the call):
#   tests          pytest -m gpu in one process (TEST_PATHS / PYTEST_ARGS narrow it)
#   smoke          __graft_entry__.smoke()
#   bench          bench.py (the driver's default line) -> bench.json
#   traces         rocprofv3 --kernel-trace --stats of the bench command and of the sweep
#   pmc_bytes      FETCH_SIZE / WRITE_SIZE passes (separate runs) over the 4096 .. 4M env steps
#   probe          scripts/contact_probe.py $PROBE_CASES with every library of $LIBS, alternated
#                  $REPS times (LIBS: names of libgpd_<name>.so, "main" = libgpd.so)
#   probe_trace    rocprofv3 --kernel-trace --stats of contact_probe.py $PROBE_CASES for each library of $LIBS
#   pmc_icache     SQC I-cache and FETCH_SIZE / WRITE_SIZE passes (separate runs) over the 4096-env
#                  headline step for each library of $LIBS
#   pmc_probe      one PMC pass per counter group of $PMC_GROUPS (';'-separated) and library of $LIBS
#                  over contact_probe.py $PROBE_CASES (PROBE_STEPS / PROBE_WARM shorten it)
#   ab             bench.py --no-cpu-baseline --steps 300 with every library of $LIBS, alternated
#   rollout        scripts/prof_rollout.py (bench.py's RL-rollout leg) for each store policy of
#                  $POLICIES (gpd_config::store_policy, 0 = library default), alternated $REPS times
#   rollout_trace  rocprofv3 --kernel-trace --stats of prof_rollout.py for each policy of $POLICIES
#   py             python -u $PY_ARGS (a probe script), output to py.log
#   full           tests smoke bench traces pmc_bytes
# Output: gpurun_out/$RUN_TAG/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${RUN_TAG:-job}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
P=gym_pybullet_drones_routing_amd
REPS=${REPS:-2}
libpath() { if [ "$1" = main ]; then echo $P/libgpd.so; else echo $P/libgpd_$1.so; fi; }
quiet() { grep -v "amdgpu.ids\|UserWarning\|sim = \|warnings.warn" || true; }

job_tests() {
  timeout -k 10 900 python -u -m pytest ${TEST_PATHS:-tests} -m gpu -q -p no:cacheprovider -rf --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
  local rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; return $rc
}
job_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; }
job_bench() { timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; }
job_traces() {
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-sweep --no-latency-model --no-rollout > $OUT/prof_bench_stdout.json 2> $OUT/prof_bench.err || return $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_sweep -o sweep --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $OUT/prof_sweep_stdout.json 2> $OUT/prof_sweep.err
}
job_pmc_bytes() {
  for E in 4096 65536 1048576 4194304; do
    local S=50; [ $E -ge 1048576 ] && S=10
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$E -o fetch --output-format csv -- \
      python3 scripts/prof_step.py --envs $E --steps $S > /dev/null 2>&1 || return $?
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$E -o write --output-format csv -- \
      python3 scripts/prof_step.py --envs $E --steps $S > /dev/null 2>&1 || return $?
  done
}
job_probe() {
  for rep in $(seq $REPS); do
    for v in $LIBS; do
      echo "== $v rep $rep" >> $OUT/probe.log
      GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$(libpath $v) timeout -k 10 300 python -u scripts/contact_probe.py $PROBE_CASES \
        > $OUT/probe_tmp.log 2>&1 || { cat $OUT/probe_tmp.log >> $OUT/probe.log; return 1; }
      quiet < $OUT/probe_tmp.log >> $OUT/probe.log
    done
  done
}
job_probe_trace() {
  for v in $LIBS; do
    GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$(libpath $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$v \
      -o probe --output-format csv -- python3 scripts/contact_probe.py $PROBE_CASES > $OUT/trace_$v.log 2>&1 || return $?
  done
}
job_pmc_icache() {
  for v in $LIBS; do
    local k=0
    for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" FETCH_SIZE WRITE_SIZE; do
      k=$((k + 1))
      GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$(libpath $v) timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/icache_${v}_$k \
        -o pmc --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 40 > $OUT/icache_${v}_$k.log 2>&1 || return $?
    done
  done
}
job_pmc_probe() {
  local IFS_SAVE=$IFS; IFS=';'; local groups=($PMC_GROUPS); IFS=$IFS_SAVE
  for v in $LIBS; do
    local k=0
    for grp in "${groups[@]}"; do
      k=$((k + 1))
      GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$(libpath $v) timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc_${v}_$k \
        -o pmc --output-format csv -- python3 scripts/contact_probe.py $PROBE_CASES > $OUT/pmc_${v}_$k.log 2>&1 || return $?
    done
  done
}
job_ab() {
  for rep in $(seq $REPS); do
    for v in $LIBS; do
      GPD_ALLOW_ABI_MISMATCH=1 GPD_LIB=$(libpath $v) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 \
        ${BENCH_ARGS} > $OUT/ab_${v}_r$rep.json 2> $OUT/ab_${v}_r$rep.err || return $?
    done
  done
}
job_rollout() {
  for rep in $(seq $REPS); do
    for pol in ${POLICIES:-0}; do
      echo "== policy $pol rep $rep" >> $OUT/rollout.log
      timeout -k 10 300 python -u scripts/prof_rollout.py --policy $pol 2>> $OUT/rollout.err | quiet >> $OUT/rollout.log || return $?
    done
  done
}
job_rollout_trace() {
  for pol in ${POLICIES:-0}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rollout_p$pol -o rollout --output-format csv -- \
      python3 scripts/prof_rollout.py --policy $pol > $OUT/prof_rollout_p$pol.json 2> $OUT/prof_rollout_p$pol.err || return $?
  done
}
job_py() { timeout -k 10 ${PY_TIMEOUT:-300} python -u $PY_ARGS > $OUT/py.log 2>&1; }

jobs="$@"
[ "$jobs" = full ] && jobs="tests smoke bench traces pmc_bytes"
for j in $jobs; do
  echo "[$(date +%T)] $j" >> $OUT/jobs.log
  job_$j; rc=$?
  echo "[$(date +%T)] $j rc=$rc" >> $OUT/jobs.log
  # pytest rc 1 = test failures (read the log); anything else (timeouts, aborts, faults) ends the call
  if [ $rc -ne 0 ] && ! { [ $j = tests ] && [ $rc -eq 1 ]; }; then exit $rc; fi
done
echo ALLDONE
