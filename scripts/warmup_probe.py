"""The driver's short timed region (K = 20 graph-replayed steps at 4096 envs) after two warm-up
shapes, in alternation, 15 regions each: (a) one upload replay + 5 eager steps (bench.py), (b) one
upload replay + one more replay of the same graph right before the region."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

E, K = 4096, 20
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
pool = (torch.rand((64, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
res = {"a": [], "b": []}
for it in range(15):
    for mode in ("a", "b"):
        g = sim.capture_graph([pool[k % 64] for k in range(K)])
        g.replay()
        if mode == "a":
            for k in range(5):
                sim.step(pool[k])
        else:
            g.replay()
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e6 / K)
        del g
for mode, r in res.items():
    r.sort()
    print(f"warm-up {mode}: median {r[len(r) // 2]:.3f} us/step, min {r[0]:.3f}, max {r[-1]:.3f}", flush=True)
