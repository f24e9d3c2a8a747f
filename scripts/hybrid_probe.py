"""Short timed region (K = 20 steps at 4096 envs): one 20-launch graph against m native launches
followed by a graph of the other 20 - m (does an earlier first kernel shorten the region?)."""
import os, sys, time, torch
sys.path.insert(0, "/root/repo") if os.path.exists("/root/repo") else None
sys.path.insert(0, os.getcwd())
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
E = 4096
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
pool = (torch.rand((64, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
K = 20
def region(body, reps=41):
    r = []
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter(); body(); torch.cuda.synchronize()
        r.append((time.perf_counter() - t0) * 1e6 / K)
    r.sort(); return r[reps // 2], r[0]
g20 = sim.capture_graph([pool[k % 64] for k in range(K)]); g20.replay()
for m in (1, 2, 3):
    gm = sim.capture_graph([pool[k % 64] for k in range(m, K)]); gm.replay()
    def hyb(m=m, gm=gm):
        sim.step_seq(pool, m)
        gm.replay()
    torch.cuda.synchronize()
    print(f"graph20 {region(g20.replay)}  native{m}+graph{K-m} {region(hyb)}", flush=True)
