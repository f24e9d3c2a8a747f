# Block geometry sweep of the PYB contact kernels (round 6): scripts/contact_probe.py per case and
# drones-per-block value (GPD_PROBE_DPB, 0 = the library's choice), alternated $REPS times.
#   gpurun -- 'RUN_TAG=r6f CASES="multi2pyb crash" DPBS="0 8 4 2" bash scripts/dpb_sweep.sh'
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-dpb}
mkdir -p "$OUT"
for rep in $(seq ${REPS:-2}); do
  for c in ${CASES:-multi2pyb}; do
    for d in ${DPBS:-0 8 4}; do
      echo "== case $c dpb $d rep $rep" >> $OUT/dpb.log
      GPD_PROBE_DPB=$d timeout -k 10 240 python -u scripts/contact_probe.py $c > $OUT/dpb_tmp.log 2>&1 || { cat $OUT/dpb_tmp.log >> $OUT/dpb.log; exit 1; }
      grep "us/step" $OUT/dpb_tmp.log >> $OUT/dpb.log
    done
  done
done
echo ALLDONE
