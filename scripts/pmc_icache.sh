# Instruction-cache / wait PMC passes over the 4096-env step (2 vs 3 waves), one counter group per run.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-pmc}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for w in 2 3; do
  for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 60 rocprofv3 --pmc $grp -d $OUT/pmc_${w}_$tag -o pmc --output-format csv -- python3 scripts/prof_step.py --envs 4096 --steps 40 --waves $w > /dev/null 2> $OUT/pmc_${w}_$tag.err || echo "pass $w $tag failed rc=$?" >> $OUT/fail.log
  done
done
echo ALLDONE
