cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 300 python scripts/stamp_probe.py > gpurun_out/quick/stamps.log 2>&1
