# Kernel iteration: variant parity tests, stamps (2 vs 3 waves), geometry probe.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-it}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "step_parity_hover or duo_kernel" > $OUT/kern_tests.log 2>&1 || exit $?
for w in 2 3; do
  STAMP_WAVES=$w STAMP_PRECS=f64 STAMP_ENVS="${STAMP_ENVS:-4096 16384}" timeout -k 10 300 python scripts/stamp_probe.py >> $OUT/stamps.log 2>&1 || exit $?
done
timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.log 2>&1 || exit $?
echo ALLDONE
