# Round 3: 2-drone MultiHoverAviary PPO on Physics.PYB with the flag-set kernel for multi PYB.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zg}
mkdir -p $OUT
timeout -k 10 420 python -u examples/learn.py --multiagent true --max_seconds 360 --output $OUT/learn_pyb_multi.json > $OUT/learn_multi.log 2>&1 || exit $?
echo ALLDONE
