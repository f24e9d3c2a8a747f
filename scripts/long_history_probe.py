"""Step time of long-action-history envs (ctrl_freq = pyb_freq / 2): 240 Hz control runs on the
one-wave run-time-flag kernel, 480 Hz on step_kernel_wide (one env per workgroup, gpd_create's
fallback when the 64-row observation tile does not fit the LDS).  HIP events over graph replays."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

for E in (4096, 65536):
    for ctrl in (30, 240, 480):
        for phys in (Physics.DYN, Physics.PYB):
            sim = BatchedAviarySim(n_envs=E, task="hover", act=ActionType.RPM, physics=phys, pyb_freq=2 * ctrl,
                                   ctrl_freq=ctrl, device="cuda:0")
            g = torch.Generator(device="cuda:0")
            g.manual_seed(0)
            acts = [(torch.rand((E, 1, 4), generator=g, device="cuda:0") * 2 - 1).contiguous() for _ in range(16)]
            graph = sim.capture_graph(acts)
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            n = 10
            for _ in range(n):
                graph.replay()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1000 / (n * 16)
            k = sim.constants
            print(f"E={E} ctrl={ctrl} {phys.name}: obs width {sim.obs_width}, drones/block {k.drones_per_block}: "
                  f"{us:.1f} us per step", flush=True)
            sim.close()
