# HBM bytes per step launch at 4096 envs by launch shape: step_waves 1/2/3 x
# store_policy 1..4 (1 + write-through mask: bit 0 obs rows, bit 1 state).  Kernel trace for the
# duration, FETCH_SIZE and WRITE_SIZE in separate PMC passes (kernel trace only).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3p}
mkdir -p $OUT
E=${PMC_ENVS:-4096}
for W in 3 2 1; do
  for P in 1 2 3 4; do
    D=$OUT/w${W}_p${P}
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/trace -o t --output-format csv -- python3 scripts/prof_step.py --envs $E --steps 200 --waves $W --policy $P > /dev/null 2>&1 || exit $?
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o f --output-format csv -- python3 scripts/prof_step.py --envs $E --steps 50 --waves $W --policy $P > /dev/null 2>&1 || exit $?
    timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $D/write -o w --output-format csv -- python3 scripts/prof_step.py --envs $E --steps 50 --waves $W --policy $P > /dev/null 2>&1 || exit $?
    echo "w$W p$P done" >> $OUT/progress.txt
  done
done
python3 scripts/pmc_table.py $OUT > $OUT/table.txt 2>&1
echo ALLDONE
