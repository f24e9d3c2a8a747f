"""Step time of envs of more than 64 drones (step_kernel_wide, one env per workgroup), ctrl_freq
30: GPD_LIB selects the library (A/B of the wide kernel's history copy)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

for D, E in ((96, 256), (300, 64), (1024, 16)):
    sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM, physics=Physics.DYN,
                           device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = [(torch.rand((E, D, 4), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous() for _ in range(16)]
    graph = sim.capture_graph(acts)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        graph.replay()
    b.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(os.environ.get('GPD_LIB', 'libgpd.so'))} D={D} E={E}: "
          f"{a.elapsed_time(b) * 1000 / 160:.1f} us per step", flush=True)
    sim.close()
