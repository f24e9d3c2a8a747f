"""Step time of the single-wave kernel at 4096 HoverAviary envs by force-term set (plain DYN
single-wave, ground effect, drag, both): where config 3's extra time goes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gym_pybullet_drones_routing_amd.enums import ActionType  # noqa: E402
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

dev = torch.device("cuda:0")
out = []
for aero in [(), ("gnd",), ("drag",), ("gnd", "drag")]:
    os.environ["GPD_DUO"] = "0"
    sim = BatchedAviarySim(n_envs=4096, task="hover", act=ActionType.RPM, aero=aero, device=dev)
    pool = bench.make_pool(4096, 4, dev, seed=3, pool=16)
    w, n, k = bench.time_graph(sim, pool, 400, 50)
    out.append({"aero": list(aero), "kernel_us": k, "lanes_per_block": sim.constants.lanes_per_block})
    sim.close()
print(json.dumps(out))
