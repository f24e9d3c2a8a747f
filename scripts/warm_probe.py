"""Does a large-N step time depend on how long the GPU has been busy?  Times consecutive
16-step graph replays at 1M envs right after the sim is created (and again after a 1 s idle
gap), one HIP event pair per replay, to separate a warm-up of the GPU (clocks / power state)
from the kernel itself."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

E, G = 1 << 20, 16
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
acts = [(torch.rand((E, 1, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(G)]
g = sim.capture_graph(acts)
torch.cuda.synchronize()


def series(n, label):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        g.replay()
        b.record()
    torch.cuda.synchronize()
    us = [1000 * a.elapsed_time(b) / G for a, b in ev]
    print(label, " ".join(f"{u:6.1f}" for u in us), flush=True)


series(40, "cold start   ")
time.sleep(1.0)
series(40, "after 1 s idle")
series(40, "continuing   ")
