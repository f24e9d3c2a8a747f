"""Step time at 4096 envs (f64 HoverAviary, RPM) for A/B of diagnostic builds (GPD_LIB): K = 300
graph-replayed steps after a warm-up replay, HIP events, median of 7 regions."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
E = int(os.environ.get("GPD_PROBE_ENVS", "4096"))
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0",
                       tuning={"step_waves": int(os.environ.get("GPD_PROBE_WAVES", "0"))})
pool = (torch.rand((64, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
g = sim.capture_graph([pool[k % 64] for k in range(300)])
g.replay()
torch.cuda.synchronize()
r = []
for _ in range(7):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    r.append(s.elapsed_time(e) * 1000 / 300)
r.sort()
print(f"{tag:10s} E={E} {r[3]:.3f} us/step (min {r[0]:.3f})", flush=True)
