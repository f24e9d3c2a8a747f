# PPO seed sweep for SURVEY f1 (examples/learn.py, single-drone HoverAviary, Physics.PYB, ONE_D_RPM):
#   gpurun -- 'RUN_TAG=r5l MODE=eager SEEDS="0 1 2" MAXS=150 bash scripts/learn_seeds.sh'
# One run per seed, each under its own timeout; the first failure ends the call.  JSON histories
# land in gpurun_out/$RUN_TAG/ (copied to profiles/r5/learn_seeds/ afterwards).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-learn}
mkdir -p "$OUT"
EXTRA=""
[ "${MODE:-eager}" = graph ] && EXTRA="--graph"
# ROLLOUT: fused (the policy kernel, learn.py's default) or eager (torch library calls); MULTI=true:
# the 2-drone MultiHoverAviary env (learn.py --multiagent)
EXTRA="$EXTRA --rollout ${ROLLOUT:-fused} --multiagent ${MULTI:-false}"
TAGP=${MODE:-eager}_${ROLLOUT:-fused}$([ "${MULTI:-false}" = true ] && echo _multi)
for s in ${SEEDS:-0 1 2}; do
  timeout -k 10 $(( ${MAXS:-150} + 120 )) python -u examples/learn.py --seed $s --max_seconds ${MAXS:-150} $EXTRA \
    --output $OUT/${TAGP}_s$s.json > $OUT/${TAGP}_s$s.log 2>&1 || exit $?
done
echo ALLDONE
