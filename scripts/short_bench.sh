#!/bin/bash
# The driver's short bench (K=20, W=5) five times in fresh processes, then K=300 once, headline
# leg only (no sweep / CPU baseline / latency model); one JSON line each into gpurun_out/short/.
set -e
mkdir -p gpurun_out/short
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-sweep --no-cpu-baseline \
    --no-latency-model > gpurun_out/short/k20_$i.json 2> gpurun_out/short/k20_$i.err
done
timeout -k 10 120 python3 bench.py --gpus 1 --steps 300 --warmup 20 --no-sweep --no-cpu-baseline \
  --no-latency-model > gpurun_out/short/k300.json 2> gpurun_out/short/k300.err
