# Two ranks on the one GPU of a gpurun box over gloo: rehearses bench.py's multi-rank path
# (torchrun env, barriers, max-over-ranks timing, obs all-gather); the RCCL run is the driver's.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dist
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 64 --warmup 16 --dist-backend gloo > gpurun_out/dist/bench2.json 2> gpurun_out/dist/bench2.err
echo "rc=$?" >> gpurun_out/dist/bench2.err
