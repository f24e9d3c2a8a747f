"""Launch-geometry A/B: step time (hipGraph of 16 env.steps, HIP events) per
(envs, drones per block, two-wave kernel on/off).  GPD_DRONES_PER_BLOCK / GPD_DUO are read at
gpd_create, so one process covers every combination."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim


def probe(E, dpb, duo, reps=30, G=16):
    os.environ["GPD_DRONES_PER_BLOCK"] = str(dpb)
    os.environ["GPD_DUO"] = str(duo)
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
    geo = (sim.constants.drones_per_block, sim.constants.lanes_per_block)
    acts = [(torch.rand((E, 1, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    for _ in range(3):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    sim.close()
    return geo, 1000 * s.elapsed_time(e) / (reps * G)


cases = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("GEOM_CASES", "4096,16,0 4096,16,1 4096,8,1 4096,32,1 4096,64,1 16384,64,0 16384,16,1 16384,64,1 65536,64,0 65536,64,1 262144,64,0 262144,64,1").split()]
for E, dpb, duo in cases:
    geo, us = probe(E, dpb, duo)
    print(f"E {E:7d} drones/block {geo[0]:2d} lanes/block {geo[1]:3d}: {us:8.2f} us/step  "
          f"{E * 8 / us * 1e-3:7.2f} G drone*dt/s", flush=True)
