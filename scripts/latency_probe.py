"""Step-kernel time at small N vs substeps per launch (fixed cost vs per-substep chain)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

def probe(E, pyb, ctrl, prec, reps=20, G=16):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision=prec, pyb_freq=pyb, ctrl_freq=ctrl, device="cuda:0")
    acts = [((torch.rand((E, 1, 4), device="cuda:0") * 2 - 1) * 0.05).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    for _ in range(3): g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): g.replay()
    e.record(); torch.cuda.synchronize()
    sim.close()
    return 1000 * s.elapsed_time(e) / (reps * G)

for prec in ("f64", "f32"):
    for E in (64, 4096, 16384):
        row = [f"{probe(E, pyb, 30, prec):7.2f}" for pyb in (30, 240, 480)]
        print(prec, "E", E, "us/step for 1/8/16 substeps:", " ".join(row), flush=True)

# floor: a hipGraph of 16 trivial torch kernels (kernel boundary + launch inside a graph)
x = torch.zeros(4096, device="cuda:0")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(16):
        x.add_(1.0)
for _ in range(3): g.replay()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); s.record()
for _ in range(50): g.replay()
e.record(); torch.cuda.synchronize()
print("trivial kernel in graph: %.2f us/launch" % (1000 * s.elapsed_time(e) / 800))
