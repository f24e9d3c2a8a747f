cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-st}
mkdir -p $OUT
for w in 2 3; do
  STAMP_WAVES=$w STAMP_PRECS=f64 STAMP_ENVS="4096 16384" timeout -k 10 300 python scripts/stamp_probe.py >> $OUT/stamps.log 2>&1 || exit $?
done
echo ALLDONE
