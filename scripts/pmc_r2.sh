# HBM byte accounting: FETCH_SIZE / WRITE_SIZE calibration probe (4/8/16 B per lane), then the
# step kernel at 4096 / 65536 / 1M / 4M envs, each counter in its own pass (TCC slots).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r2q}
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d $OUT/cal_$c -o cal --output-format csv -- ./scripts/ubench/fetch_probe > $OUT/cal_$c.log 2>&1 || exit $?
done
for E in 4096 65536 1048576 4194304; do
  S=50; [ $E -ge 1048576 ] && S=10
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_${c}_$E -o pmc --output-format csv -- python3 scripts/prof_step.py --envs $E --steps $S > /dev/null 2>&1 || exit $?
  done
done
echo ALLDONE
