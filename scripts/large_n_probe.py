#!/usr/bin/env python3
"""Step time of the single-wave kernel at 1M / 4M HoverAviary envs (f64, RPM), graph replay,
for the library GPD_LIB points at (A/B builds: scripts/large_n_ab.sh).  Two action sets: the
bench's U[-1,1] (episodes end, auto-reset rows) and 0.05 * U[-1,1] (hover, no resets)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402


def run(E, scale, G=16, reps=4, policy=0):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0",
                           tuning={"store_policy": policy} if policy else None)
    gen = torch.Generator(device="cuda:0").manual_seed(7)
    acts = [((torch.rand((E, 1, 4), generator=gen, device="cuda:0") * 2 - 1) * scale).contiguous() for _ in range(G)]
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
    us = 1000 * s.elapsed_time(e) / (reps * G)
    sim.close()
    del acts, g
    torch.cuda.empty_cache()
    return us


if __name__ == "__main__":
    tag = os.path.basename(os.environ.get("GPD_LIB", "libgpd.so"))
    envs = [int(x) for x in os.environ.get("PROBE_ENVS", f"{1 << 20},{1 << 22}").split(",")]
    pols = [int(x) for x in os.environ.get("PROBE_POLICIES", "0").split(",")]
    scales = [float(x) for x in os.environ.get("PROBE_SCALES", "1.0,0.05").split(",")]
    for E in envs:
        G, reps = (16, 4) if E > 100000 else (128, 20)
        for pol in pols:
            for scale in scales:
                us = run(E, scale, G=G, reps=reps, policy=pol)
                print(f"{tag:24s} policy {pol} E={E:8d} actions x{scale:<4} {us:8.2f} us  "
                      f"{774 * E / us / 1e3:6.0f} GB/s alg", flush=True)
