#!/bin/bash
# scripts/region_probe.py under HIP runtime (ROCclr) environment settings that govern how the
# host waits for a completion signal; one output file per setting in gpurun_out/short/.
set -e
mkdir -p gpurun_out/short
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python3 -u scripts/region_probe.py > gpurun_out/short/env_$tag.txt 2>&1; }
run base X=1
run awt50 ROC_ACTIVE_WAIT_TIMEOUT=50
run awt1000 ROC_ACTIVE_WAIT_TIMEOUT=1000
run sss0 ROC_SYSTEM_SCOPE_SIGNAL=0
run blk0 DEBUG_HIP_BLOCK_SYNC=0
run cpuwait0 ROC_CPU_WAIT_FOR_SIGNAL=0
