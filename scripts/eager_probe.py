"""Host cost of the eager BatchedAviarySim.step() at 4096 envs (no events, no graph): the time
per call of 3000 back-to-back calls.  Compares sim_old (a copy of an older sim.py, if present)
with sim."""
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
res = {}
mods = ("sim_old", "sim", "sim_old", "sim") if os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym_pybullet_drones_routing_amd", "sim_old.py")) else ("sim",)
for mod in mods:
    m = importlib.import_module("gym_pybullet_drones_routing_amd." + mod)
    s = m.BatchedAviarySim(n_envs=4096, task="hover", device="cuda:0")
    a = torch.zeros((4096, 1, 4), device="cuda:0")
    for _ in range(200): s.step(a)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3000): s.step(a)
    torch.cuda.synchronize()
    res.setdefault(mod, []).append(1e6 * (time.perf_counter() - t) / 3000)
    s.close()
print(json.dumps(res))
