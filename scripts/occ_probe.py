"""Step time at large N for the occupancy question (GPD_LIB selects a diagnostic build that pads
the step kernel's LDS tile, GPD_TILE_MIN): a 16-step graph replayed 4 times after a warm-up
replay, HIP events; us per step for several workloads.  argv[1] = tag."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.enums import Physics  # noqa: E402
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("GPD_LIB", "libgpd.so"))
CASES = [("dyn f64", 1 << 18, 1, {}), ("dyn f64", 1 << 20, 1, {}), ("dyn f64", 1 << 22, 1, {}),
         ("dyn f32", 1 << 20, 1, {"precision": "f32"}), ("dyn f32", 1 << 22, 1, {"precision": "f32"}),
         ("gnd+drag f64", 1 << 20, 1, {"aero": ("gnd", "drag")}),
         ("multi8 dw f64", 1 << 17, 8, {"physics": Physics.DYN, "aero": ("dw",)})]
for name, E, D, kw in CASES:
    kw = dict(kw)
    prec = kw.pop("precision", "f64")
    task = "hover" if D == 1 else "multihover"
    sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task=task, precision=prec, device="cuda:0", **kw)
    pool = (torch.rand((4, E, D, 4), device="cuda:0") * 0.2 - 0.1).contiguous()
    g = sim.capture_graph([pool[k % 4] for k in range(16)])
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(4):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1000 / 64
    print(f"{tag:10s} {name:14s} N={E * D:8d} {us:8.1f} us/step", flush=True)
    sim.close()
    del pool, g
    torch.cuda.empty_cache()
