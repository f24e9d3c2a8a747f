# Round 3: instruction fetch in FETCH_SIZE (scripts/ubench/ifetch_probe.hip), one PMC pass each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3m}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/ifetch -o f --output-format csv -- ./scripts/ubench/ifetch_probe > $OUT/ifetch.txt 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $OUT/icache -o i --output-format csv -- ./scripts/ubench/ifetch_probe >> $OUT/ifetch.txt 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $OUT/icache_step -o s --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 50 > /dev/null 2>&1 || exit $?
echo ALLDONE
