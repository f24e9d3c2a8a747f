"""Timeline of short bench.py-style timed regions for rocprofv3 --kernel-trace --hip-runtime-trace:
12 regions of `synchronize; replay a K-step graph; synchronize` at 4096 envs (argv[1] = K,
default 20).  scripts/region_timeline.py reads the trace and splits each region into host
launch -> first kernel start, the kernels, and last kernel end -> synchronize return."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
E = 4096
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
pool = (torch.rand((64, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
g = sim.capture_graph([pool[k % 64] for k in range(K)])
g.replay()
torch.cuda.synchronize()
walls = []
for _ in range(12):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t0) * 1e6)
print("region walls us:", " ".join(f"{w:.1f}" for w in walls), flush=True)
