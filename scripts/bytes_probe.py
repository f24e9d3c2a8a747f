"""Achieved bandwidth vs observation width at large N (one substep per step, so the step is
pure data movement): ctrl_freq sets the action-history length L = ctrl_freq//2."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

def run(E, f, G=8, reps=6):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", pyb_freq=f, ctrl_freq=f, device="cuda:0")
    acts = [((torch.rand((E, 1, 4), device="cuda:0") * 2 - 1) * 0.05).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    for _ in range(2): g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): g.replay()
    e.record(); torch.cuda.synchronize()
    us = 1000 * s.elapsed_time(e) / (reps * G)
    L = f // 2
    real = 8
    rd = 13 * real + 16 + (L - 1) * 16 + 8
    wr = 20 * real + (12 + 4 * L) * 4 + 16 + 8 + 6
    sim.close(); del acts, g; torch.cuda.empty_cache()
    return us, rd, wr

E = 1 << 20
for f in (2, 8, 30, 60):
    us, rd, wr = run(E, f)
    print(f"ctrl_freq {f:3d} (L={f//2:2d}): {us:7.1f} us  read {rd} B  write {wr} B per drone  -> {E*(rd+wr)/us/1e3:6.0f} GB/s "
          f"(read {E*rd/us/1e3:5.0f}, write {E*wr/us/1e3:5.0f})", flush=True)
