# Launch-floor microbenchmark, step time vs substeps, launch geometry; logs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-lat}
mkdir -p $OUT
timeout -k 10 120 ./scripts/ubench/launch_floor > $OUT/launch_floor.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/latency_probe.py > $OUT/latency.log 2>&1 || exit $?
ROUNDS=2 timeout -k 10 300 python -u scripts/geom_probe.py > $OUT/geom.log 2>&1 || exit $?
echo ALLDONE
