"""Store-policy A/B at the bandwidth-bound sizes: step time (hipGraph of 16 env.steps, HIP
events) per gpd_config::store_policy (1 = plain stores, 2 = write-through obs rows, 3 =
write-through state, 4 = both; 0 = automatic) at 1M and 4M envs, interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

ALG = 774


def probe(E, pol, reps=4, G=16):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0",
                           tuning={"store_policy": pol})
    acts = [(torch.rand((E, 1, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    for _ in range(2):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    sim.close()
    del g, acts
    torch.cuda.empty_cache()
    return 1000 * s.elapsed_time(e) / (reps * G)


cases = [(E, p) for E in (1 << 20, 1 << 22) for p in (1, 2, 3, 4)]
res = {c: [] for c in cases}
for _ in range(int(os.environ.get("ROUNDS", "2"))):
    for c in cases:
        res[c].append(probe(*c))
for (E, p), r in res.items():
    us = min(r)
    print(f"E {E:8d} store_policy {p}: " + " ".join(f"{x:8.1f}" for x in r) +
          f" us/step  best {ALG * E / us / 1e3 / 8000 * 100:5.1f} % of 8 TB/s", flush=True)
