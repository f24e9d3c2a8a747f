"""Launch-geometry probe for BASELINE config 4 (MultiHoverAviary x 8 drones, downwash, staggered
init): step time per (envs, drones per block) - CASES="E,dpb ..."; GPD_DRONES_PER_BLOCK is read
at gpd_create."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

stag = [[0.15 * math.cos(2 * math.pi * i / 8), 0.15 * math.sin(2 * math.pi * i / 8), 0.5 + 0.1 * i] for i in range(8)]
for case in os.environ.get("CASES", "512,8 512,16 512,32 512,64").split():
    E, dpb = (int(x) for x in case.split(","))
    if dpb > 0:
        os.environ["GPD_DRONES_PER_BLOCK"] = str(dpb)
    else:                                   # the library's own choice
        os.environ.pop("GPD_DRONES_PER_BLOCK", None)
    sim = BatchedAviarySim(n_envs=E, drones_per_env=8, task="multihover", act=ActionType.RPM, physics=Physics.DYN,
                           aero=("dw",), initial_xyzs=stag, precision="f64", device="cuda:0")
    acts = [(torch.rand((E, 8, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(16)]
    g = sim.capture_graph(acts)
    for _ in range(3):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(30):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    us = 1000 * s.elapsed_time(e) / (30 * 16)
    print(f"{E} envs x 8 drones, drones/block {sim.constants.drones_per_block:2d}: {us:7.2f} us/step "
          f"{E * 64 / us * 1e-3:6.2f} G drone*dt/s", flush=True)
    sim.close()
