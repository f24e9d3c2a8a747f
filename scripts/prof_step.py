"""Profiling driver: a few env.steps of E envs (for rocprofv3 kernel-trace / PMC passes)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=1 << 20)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--precision", default="f64")
ap.add_argument("--act", default="rpm")
ap.add_argument("--waves", type=int, default=0, help="gpd_config step_waves (0 = automatic)")
ap.add_argument("--policy", type=int, default=0, help="gpd_config store_policy (0 = automatic; 1 + write-through mask)")
ap.add_argument("--dpb", type=int, default=0, help="gpd_config drones_per_block (0 = automatic)")
a = ap.parse_args()
from gym_pybullet_drones_routing_amd.enums import ActionType
A = 4 if a.act == "rpm" else 1
sim = BatchedAviarySim(n_envs=a.envs, task="hover", precision=a.precision, act=ActionType(a.act), device="cuda:0",
                       tuning={k: v for k, v in (("step_waves", a.waves), ("store_policy", a.policy),
                                                   ("drones_per_block", a.dpb)) if v} or None)
acts = (torch.rand((4, a.envs, 1, A), device="cuda:0") * 2 - 1).contiguous()
for k in range(a.steps):
    sim.step(acts[k % 4])
torch.cuda.synchronize()
print("done", a)
