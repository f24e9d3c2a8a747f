# Round 3: counters available on gfx950 and the wave-level instruction-fetch counters of the 4096-env
# step (one PMC group per pass).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3o}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" "SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_HITS"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $grp -d $OUT/step_$tag -o p --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 40 > /dev/null 2> $OUT/step_$tag.err || echo "pass $tag failed rc=$?" >> $OUT/fail.log
  timeout -s KILL 60 rocprofv3 --pmc $grp -d $OUT/probe_$tag -o p --output-format csv -- ./scripts/ubench/ifetch_probe > /dev/null 2> $OUT/probe_$tag.err || echo "probe $tag failed rc=$?" >> $OUT/fail.log
done
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $OUT/probe_trace -o t --output-format csv -- ./scripts/ubench/ifetch_probe > /dev/null 2>&1 || true
echo ALLDONE
