# Write-through store policy probe: latency at small N and bandwidth sweep per GPD_WT value.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/wt
for W in 0 1 3; do
  GPD_WT=$W timeout -k 10 300 python scripts/latency_probe.py > gpurun_out/wt/latency_$W.log 2>&1 || exit $?
  GPD_WT=$W timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/wt/bench_$W.json 2> gpurun_out/wt/bench_$W.err || exit $?
done
echo done
