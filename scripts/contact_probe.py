#!/usr/bin/env python3
"""Step time of the Physics.PYB kernels with and without ground contact (4096 HoverAviary envs, f64).

Cases ('multi' / 'multifly': bench.py's 512 x 8 PYB_GND_DRAG_DW row with U[-1,1] / hover actions):
'crash' = U[-1,1] RPM actions (many drones end up on the plane, as in bench.py's PYB row),
'rest' = zero actions of thrust 0.8 hover (every drone resting on the plane after ~0.3 s),
'fly' = hover actions (no contact), 'noplane' = U[-1,1] with the plane off.  Prints one line
per case: mean us/step over a timed region of replayed steps and the fraction of low drones.
Select the library with GPD_LIB (A/B builds), the block geometry with GPD_PROBE_DPB (drones per block)."""
import ctypes
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics  # noqa: E402
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402


STAG = [[0.15 * math.cos(2 * math.pi * i / 8), 0.15 * math.sin(2 * math.pi * i / 8), 0.5 + 0.1 * i] for i in range(8)]


# GPD_PROBE_NODC=1: the multi-drone cases without the drone <-> drone contact
NODC = ("no_drone_contact",) if os.environ.get("GPD_PROBE_NODC") == "1" else ()


def run(case, E=4096, warm=int(os.environ.get("PROBE_WARM", 60)), steps=int(os.environ.get("PROBE_STEPS", 200))):
    aero = ("no_plane",) if case == "noplane" else ()
    if case in ("multi", "multifly", "multi8pyb"):    # bench.py's PYB_GND_DRAG_DW row: 512 MultiHover envs x 8
        E, D = 512, 8                                 # drones, staggered (multi8pyb: the same on Physics.PYB)
        sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM,
                               physics=Physics.PYB if case == "multi8pyb" else Physics.PYB_GND_DRAG_DW,
                               initial_xyzs=STAG, device="cuda:0", aero=NODC)
    elif case == "multi2pyb":   # MultiHoverAviary's default: 2 drones, Physics.PYB (examples/learn.py --multiagent)
        E, D = 2048, 2
        sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM,
                               physics=Physics.PYB, device="cuda:0", aero=NODC)
    else:
        D = 1
        sim = BatchedAviarySim(n_envs=E, act=ActionType.RPM, physics=Physics.PYB, aero=aero, device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(0)
    dpb = int(os.environ.get("GPD_PROBE_DPB", "0"))      # drones per block (0: the library's choice)
    if dpb:
        sim.close()
        kw = dict(tuning={"drones_per_block": dpb}, device="cuda:0")
        if case in ("multi", "multifly"):
            sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM,
                                   physics=Physics.PYB_GND_DRAG_DW, initial_xyzs=STAG, **kw)
        elif case == "multi2pyb":
            sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM,
                                   physics=Physics.PYB, **kw)
        else:
            sim = BatchedAviarySim(n_envs=E, act=ActionType.RPM, physics=Physics.PYB, aero=aero, **kw)
    n = warm + steps
    if case in ("crash", "noplane", "multi", "multi2pyb", "multi8pyb"):
        acts = torch.rand((n, E, D, 4), generator=g, device="cuda:0", dtype=torch.float32) * 2 - 1
    elif case == "rest":
        acts = torch.full((n, E, D, 4), -1.0, device="cuda:0")      # 0.95 hover RPM: sinks and rests
    else:                  # fly / multifly: hover actions, no contact
        acts = torch.zeros((n, E, D, 4), device="cuda:0")
    for t in range(warm):
        sim.step(acts[t])
    torch.cuda.synchronize()
    NH = 256 + 4 * 4096 + 16
    if hasattr(sim._lib, "gpd_debug_contact_hist"):     # the stats below cover the timed steps only
        sim._lib.gpd_debug_contact_hist((ctypes.c_ulonglong * NH)())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for t in range(warm, n):
        sim.step(acts[t])
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / steps
    z = sim.state20()[:, 2]
    lowf = float((z < 0.02).double().mean())
    print(f"{case:8s} {us:9.2f} us/step  low drones {lowf:.3f}", flush=True)
    lib = sim._lib
    if hasattr(lib, "gpd_debug_contact_hist"):       # -DGPD_CONTACT_STATS build
        h = (ctypes.c_ulonglong * NH)()
        lib.gpd_debug_contact_hist(h)
        it = np.array(h[:51])
        la = np.array(h[51:116])
        if it.sum():
            print(f"   solves {it.sum()}  iterations: mean {np.dot(np.arange(51), it) / it.sum():.2f} "
                  f"hist {dict((i, int(v)) for i, v in enumerate(it) if v)}  active lanes mean "
                  f"{np.dot(np.arange(65), la) / la.sum():.1f}", flush=True)
            if h[122]:
                print(f"   shader cycles: setup {h[120] / it.sum():.0f} per solve, loop {h[121] / h[122]:.0f} per "
                      f"iteration ({h[121] / it.sum():.0f} per solve)", flush=True)
        tot = np.array(h[256 + 4096:256 + 8192], dtype=np.float64) / steps
        if tot.any():
            pl = np.array(h[256 + 8192:256 + 12288], dtype=np.float64) / steps
            dcb = np.array(h[256:256 + 4096], dtype=np.float64) / steps
            order = np.argsort(tot)[::-1][:4]
            print("   step-kernel cycles per step, slowest blocks: " + "; ".join(
                f"b{b}: total {tot[b]:.0f} plane {pl[b]:.0f} pair {dcb[b]:.0f}" for b in order) +
                f"; mean total {tot[tot > 0].mean():.0f} plane {pl[tot > 0].mean():.0f} pair {dcb[tot > 0].mean():.0f}",
                flush=True)
        if h[116]:
            print(f"   drone contact per solve: setup {h[117] / h[116]:.0f} cycles (pass 1 {h[123] / h[116]:.0f}), "
                  f"iterations {h[119] / h[116]:.2f} x {h[118] / max(h[119], 1):.0f} cycles, "
                  f"near pairs {h[127] / h[116]:.2f}, contacts {h[126] / h[116]:.2f}", flush=True)
            if h[248]:
                print(f"   rare path per call: columns {h[244] / h[248]:.0f}, park {h[245] / h[248]:.0f}, call "
                      f"{h[246] / h[248]:.0f} (solve {(h[117] + h[118]) / h[116]:.0f}), unpark + deltas "
                      f"{h[247] / h[248]:.0f} cycles", flush=True)
            print(f"   pass 0 narrowphases end at {h[254] / h[116]:.0f} cycles per solve; island solves {h[124]}, "
                  f"register fast path {h[125]} of {h[116]}; Gauss-Seidel rounds per phase {h[243] / h[116]:.2f}",
                  flush=True)
            print(f"   narrowphase levels: {[int(x) for x in h[249:253]]}, least-overlap fallback {h[253]}", flush=True)
            npb = 256 + 4 * 4096
            if h[npb]:
                print(f"   contacts: most in one solve {h[255]}, solves past the register rows {h[npb + 5]}, "
                      f"contact passes per solve {h[npb + 6] / h[116]:.2f}", flush=True)
                if h[npb + 12]:
                    gi = h[npb + 12]
                    print(f"   general-path iterations {gi}: per iteration island sweeps {h[npb + 7] / gi:.0f}, "
                          f"normal rounds {h[npb + 8] / gi:.0f}, friction rounds {h[npb + 9] / gi:.0f}, ends "
                          f"{h[npb + 10] / gi:.0f} cycles; rounds per phase {h[npb + 11] / gi:.2f}", flush=True)
                print(f"   narrowphase passes {h[npb]}: near pairs {h[npb + 3] / h[npb]:.2f}, rim tasks "
                      f"{h[npb + 1] / h[npb]:.0f}, selection {h[npb + 2] / h[npb]:.0f}, fallback + face points "
                      f"{h[npb + 4] / h[npb]:.0f} cycles per pass", flush=True)
            lg = np.array(h[128:192])
            print(f"   drone contact solve cycles (log2 buckets): "
                  f"{dict((f'2^{i}', int(v)) for i, v in enumerate(lg) if v)}", flush=True)
            di = np.array(h[192:243])
            print(f"   drone contact iterations hist {dict((i, int(v)) for i, v in enumerate(di) if v)}", flush=True)
            blk = np.array(h[256:256 + 4096], dtype=np.float64) / steps
            top = np.sort(blk)[::-1][:4]
            print(f"   drone contact cycles per step, by block: max {top[0]:.0f} (next {top[1:].round().tolist()}), "
                  f"mean over blocks {blk[blk > 0].mean() if (blk > 0).any() else 0:.0f}", flush=True)
        # per launch: the slowest block (what the kernel's duration follows) and where its cycles went
        nps = int(os.environ.get("PROBE_PERSTEP", "40"))
        rows = []
        g2 = torch.Generator(device="cuda:0").manual_seed(1)
        for t in range(nps):
            a = torch.rand((E, D, 4), generator=g2, device="cuda:0") * 2 - 1 if case in ("crash", "noplane", "multi", "multi2pyb", "multi8pyb") else acts[t % n]
            sim.step(a)
            lib.gpd_debug_contact_hist(h)
            tb = np.array(h[256 + 4096:256 + 8192], dtype=np.float64)
            b = int(np.argmax(tb))
            rows.append((tb[b], h[256 + 8192 + b], h[256 + b], h[256 + 12288 + b],
                         np.max(np.array(h[256:256 + 4096], dtype=np.float64)), tb.mean()))
        r = np.array(rows, dtype=np.float64)
        print(f"   per launch ({nps}): slowest block total {r[:, 0].mean():.0f} (plane {r[:, 1].mean():.0f}, pair solve "
              f"{r[:, 2].mean():.0f}, pair rare path incl. the solve {r[:, 3].mean():.0f}); mean block total "
              f"{r[:, 5].mean():.0f}; largest pair-solve cycles of any block {r[:, 4].mean():.0f} (max {r[:, 4].max():.0f})",
              flush=True)
    sim.close()


if __name__ == "__main__":
    for case in (sys.argv[1:] or ["fly", "noplane", "crash", "rest", "multi"]):
        run(case)
