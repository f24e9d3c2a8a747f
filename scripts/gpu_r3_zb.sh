# Round 3: PPO to the reference's thresholds on the final code, Physics.PYB (the env classes'
# default, with the ground contact): HoverAviary (474.15) and 2-drone MultiHoverAviary (949.5).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zb}
mkdir -p $OUT
timeout -k 10 420 python -u examples/learn.py --max_seconds 360 --output $OUT/learn_pyb_single.json > $OUT/learn_single.log 2>&1 || exit $?
timeout -k 10 420 python -u examples/learn.py --multiagent true --max_seconds 360 --output $OUT/learn_pyb_multi.json > $OUT/learn_multi.log 2>&1 || exit $?
echo ALLDONE
