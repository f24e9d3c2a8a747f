# Round 3: the hand-off tests (RCCL one-rank, gloo two-rank with HIP sims) after the gather-mode
# change, then a two-rank gloo rehearsal of bench.py's multi-rank path (both hand-off legs).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3q}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_env_api.py -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 64 --warmup 16 --dist-backend gloo > $OUT/bench2.json 2> $OUT/bench2.err
echo "rc=$?" >> $OUT/bench2.err
echo ALLDONE
