# Round 3: bench.py's strong-scaling leg (32768 envs split over the ranks): one rank, then the
# two-rank gloo rehearsal on this GPU.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3za}
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sweep --no-latency-model --steps 64 --warmup 8 > $OUT/bench1.json 2> $OUT/bench1.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 64 --warmup 16 --dist-backend gloo > $OUT/bench2.json 2> $OUT/bench2.err
echo "rc=$?" >> $OUT/bench2.err
echo ALLDONE
