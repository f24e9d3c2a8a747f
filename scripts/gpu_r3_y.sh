# Round 3: per-rank PPO learners (examples/learn.py --learner per-rank): the learn plumbing GPU
# tests, then a 2-rank gloo rehearsal on this GPU training HoverAviary (DYN) to the threshold.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3y}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_learn_plumbing.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u examples/learn.py --gpus 2 --dist-backend gloo --learner per-rank --n_envs 8192 --physics dyn --max_seconds 200 --output $OUT/learn_per_rank_dyn.json > $OUT/learn.log 2>&1
echo "learn rc=$?" >> $OUT/learn.log
echo ALLDONE
