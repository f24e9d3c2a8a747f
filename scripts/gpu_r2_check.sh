# Checkpoint run: every GPU test in one pytest process, smoke(), the two-rank gloo rehearsal of
# bench.py (torchrun form and the self-launching --gpus form); logs under gpurun_out/$TAG.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-chk}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 64 --warmup 16 --dist-backend gloo --no-cpu-baseline > $OUT/bench2_torchrun.json 2> $OUT/bench2_torchrun.err || exit $?
timeout -k 10 400 python bench.py --gpus 2 --steps 64 --warmup 16 --dist-backend gloo --no-cpu-baseline > $OUT/bench2_self.json 2> $OUT/bench2_self.err || exit $?
echo ALLDONE
