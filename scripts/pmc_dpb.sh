# Is the 4096-env FETCH excess a counter artefact of 16-lane blocks?  Single-wave kernel at 4096
# envs with 16 vs 64 drones per block (FETCH_SIZE / WRITE_SIZE passes, store policy 3 and 2).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3g}/pmc_dpb
mkdir -p $OUT
for DPB in 16 64; do
  for P in 3 2; do
    D=$OUT/w1_p${P}_d${DPB}
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/trace -o t --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 200 --waves 1 --policy $P --dpb $DPB > /dev/null 2>&1 || exit $?
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o f --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 50 --waves 1 --policy $P --dpb $DPB > /dev/null 2>&1 || exit $?
    timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $D/write -o w --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 50 --waves 1 --policy $P --dpb $DPB > /dev/null 2>&1 || exit $?
  done
done
python3 scripts/pmc_table.py $OUT > $OUT/table.txt 2>&1
