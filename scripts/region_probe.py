"""Fixed cost of a bench.py timed region (synchronize on both sides of K env.steps at 4096 envs,
f64 HoverAviary), split into its parts.  Each variant is timed 41 times; the median and min wall
time of the whole region are printed in us, and per step.

  empty        synchronize; t0; synchronize                      (the two syncs alone)
  graph        synchronize; t0; replay; synchronize              (K steps in one graph)
  graph+ev     as bench.py: event records around the replay
  graph+evsync replay; ev1.record; ev1.synchronize(); synchronize
  graph+ssync  replay; stream.synchronize(); synchronize
  native       one gpd_step_seq call of K launches
  host         host time of replay() alone (returns before the GPU is done)

argv[1] = default|spin|yield|block sets hipSetDeviceFlags before the context exists."""
import ctypes
import os
import sys
import time

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
import torch  # noqa: E402  (no HIP call yet)

if mode != "default":
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    flag = {"spin": 1, "yield": 2, "block": 4}[mode]
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
    print("hipSetDeviceFlags", mode, "rc", rc, flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

E = int(os.environ.get("GPD_PROBE_ENVS", "4096"))
REPS = 41
sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
pool = (torch.rand((64, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
stream = torch.cuda.current_stream()


def region(body):
    r = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        body()
        torch.cuda.synchronize()
        r.append((time.perf_counter() - t0) * 1e6)
    r.sort()
    return r[REPS // 2], r[0]


def report(name, K, med_min):
    med, mn = med_min
    print(f"{mode:7s} {name:13s} K={K:4d}: region {med:8.2f} us (min {mn:8.2f})  "
          f"per step {med / max(K, 1):6.2f} (min {mn / max(K, 1):6.2f})", flush=True)


report("empty", 0, region(lambda: None))
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for K in (1, 5, 20, 100, 300):
    g = sim.capture_graph([pool[k % 64] for k in range(K)])
    g.replay()
    sim.step_seq(pool, 8)
    torch.cuda.synchronize()
    report("graph", K, region(g.replay))

    def with_ev():
        ev0.record(stream)
        g.replay()
        ev1.record(stream)
    report("graph+ev", K, region(with_ev))

    def with_evsync():
        g.replay()
        ev1.record(stream)
        ev1.synchronize()
    report("graph+evsync", K, region(with_evsync))

    def with_ssync():
        g.replay()
        stream.synchronize()
    report("graph+ssync", K, region(with_ssync))
    report("native", K, region(lambda: sim.step_seq(pool, K)))
    h = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        h.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    h.sort()
    print(f"{mode:7s} {'host':13s} K={K:4d}: replay() returns after {h[REPS // 2]:8.2f} us", flush=True)
    del g
