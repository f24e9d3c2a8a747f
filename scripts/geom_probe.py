"""Launch-geometry A/B: step time (hipGraph of 16 env.steps, HIP events) per
(envs, drones per block, waves per step block), set through gpd_config's tuning fields
(BatchedAviarySim(tuning=...)), so one process covers every combination.  Each case is timed
twice in interleaved rounds (ROUNDS), so clock drift shows up as a spread, not a bias."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402


def probe(E, dpb, waves, reps=30, G=16):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0",
                           tuning={"drones_per_block": dpb, "step_waves": waves})
    geo = (sim.constants.drones_per_block, sim.constants.lanes_per_block)
    acts = [(torch.rand((E, 1, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    for _ in range(20):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    sim.close()
    return geo, 1000 * s.elapsed_time(e) / (reps * G)


default = ("4096,16,1 4096,16,2 4096,16,3 4096,8,2 4096,8,3 4096,4,3 4096,32,3 "
           "16384,64,1 16384,16,2 16384,16,3 16384,64,3 65536,64,1 65536,64,2 65536,64,3")
cases = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("GEOM_CASES", default).split()]
res = {c: [] for c in cases}
for _ in range(int(os.environ.get("ROUNDS", "2"))):
    for c in cases:
        res[c].append(probe(*c))
for (E, dpb, waves), r in res.items():
    geo = r[0][0]
    us = [x[1] for x in r]
    print(f"E {E:7d} drones/block {geo[0]:2d} lanes/block {geo[1]:3d}: "
          + " ".join(f"{u:8.2f}" for u in us) + f" us/step  {E * 8 / min(us) * 1e-3:7.2f} G drone*dt/s", flush=True)
