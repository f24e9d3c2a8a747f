# Round 3: four-rank gloo rehearsal of bench.py's multi-rank path on this one GPU (strong leg,
# hand-off legs), the driver's N = 4 form with gloo in place of RCCL.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r3zn}
mkdir -p $OUT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 4 --steps 64 --warmup 16 --dist-backend gloo > $OUT/bench4.json 2> $OUT/bench4.err
echo "rc=$?" >> $OUT/bench4.err
echo ALLDONE
