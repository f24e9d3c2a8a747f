#!/usr/bin/env python3
"""Benchmark of the batched HoverAviary DYN path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E]

One "step" = one env.step() of every env (HoverAviary, cf2x, Physics.DYN, ActionType.RPM,
240 Hz physics / 30 Hz control -> 8 substeps) on synthetic uniform [-1, 1] actions that are
resident in HBM before the timed region.  Unit of work: one drone advanced one 1/240 s
substep (drone*dt).  value = drone*dt of all ranks / max-over-ranks wall time of K steps.

Multi-GPU: one process per GPU (torchrun); each rank owns E envs (weak scaling), there is no
collective inside the timed loop.  The RCCL all-gather of the observation batch to a learner
on rank 0 (config 5) is timed separately and reported under "handoff" (on one GPU: a one-rank RCCL
group with the collectives forced).

Extra JSON fields: "roofline" (step kernel, HIP events on the launch stream), "cpu_baseline"
(the oracle, rank 0 at N=1), "parity" (the metric's state-L2 leg: GPU vs the C oracle over 5 s,
beside the CPU baseline), "sweep" (large-N roofline), "kernel_us".
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
STRONG_ENVS = 32768          # config 5's global env count, the strong-scaling leg


def alg_bytes_per_drone_step(act="rpm", real_bytes=8):
    """SURVEY.md §8(d) algorithmic bytes per drone per ctrl step (obs materialised), with the
    state in the compute precision ("fp32; double for fp64"):
      read  state 13*r + action 4A + action history 14*4A
      write state 13*r + last rpm 4*r + obs (12+15A)*4 + reward/terminated/truncated 6
    fp32 RPM: 52+16+224+52+16+288+6 = 654 B (81.75 B per drone*dt), as SURVEY quotes;
    fp64 RPM: 104+16+224+104+32+288+6 = 774 B (96.75 B per drone*dt)."""
    A = 4 if act == "rpm" else 1
    return 13 * real_bytes + 4 * A + 14 * 4 * A + 13 * real_bytes + 4 * real_bytes + (12 + 15 * A) * 4 + 6


def pmc_traffic(grid, precision):
    """HBM bytes per step-kernel launch measured by rocprofv3 PMC passes (FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE, MI355X_MICROARCH.md §HBM) in the newest profiles/*_summary.json that
    covers this grid; None when no such measurement is committed."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("precision", "f64") != precision:
            continue
        for row in d.get("pmc", []):
            if row.get("grid") == grid:
                best = (row["traffic_bytes"], os.path.relpath(f, ROOT))
    return best


def instruction_fetch_bytes(kernel, grid):
    """FETCH_SIZE bytes per launch that are instruction fetch (SQC I-cache misses x the FETCH_SIZE
    per miss of scripts/ubench/ifetch_probe.hip), from the newest profiles/r*/icache/calibration.json."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "icache", "calibration.json"))):
        try:
            k = json.load(open(f))["step_kernels"][kernel]
        except Exception:
            continue
        if k.get("grid") == grid:
            best = k["instruction_fetch_size_bytes"]
    return best


def rocprof_kernel_us(kernel, grid, precision):
    """Mean duration of `kernel` at `grid` lanes in the newest committed rocprofv3 kernel trace
    (profiles/*_summary.json "kernels" rows): the rocprof figure the live event time must match."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("precision", "f64") != precision:
            continue
        for row in d.get("kernels", []):
            if row.get("kernel") == kernel and row.get("grid") == grid and "bench" in row.get("trace", ""):
                best = (row["mean_us"], os.path.relpath(f, ROOT), row.get("b2b_median_us"))
    return best


def step_kernel_name(sim, rbytes, act):
    """The step kernel a plain-DYN single-drone sim launches (rocprofv3 name)."""
    real = "double" if rbytes == 8 else "float"
    a = 0 if act == "rpm" else 1
    if sim.constants.lanes_per_block in (128, 192):
        return "gpd::step_kernel_duo<%s, %d, %s>" % (real, a, "true" if sim.constants.lanes_per_block == 192 else "false")
    return "gpd::step_kernel<%s, %d, false, 0>" % (real, a)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_info():
    model = platform.processor() or ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    return model, os.cpu_count()


def cpu_baseline(seconds=10.0, act="rpm"):
    """Reference-shaped numpy oracle (one env object, per-drone Python loop, 8 substeps per
    step) on one core: the stand-in for the reference's own env.step()."""
    from oracle.ref_aviary import RefAviary
    A = 4 if act == "rpm" else 1
    rng = np.random.default_rng(0)
    env = RefAviary(act=act, task="hover")
    env.reset()
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = rng.uniform(-1, 1, (1, A)).astype(np.float32)
        _, _, te, tr, _ = env.step(a)
        if te or tr:
            env.reset()
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    model, ncpu = cpu_info()
    return {"value": steps * env.PYB_STEPS_PER_CTRL / el, "unit": "drone*dt/s", "cores": 1, "kind": "port",
            "sample": f"{steps} HoverAviary env.step() calls (cf2x, DYN, RPM, U[-1,1] actions, auto-reset) "
                      f"in {el:.1f} s on 1 core of '{model}' ({ncpu} host CPUs); numpy fp64 restatement of "
                      "BaseAviary.step without pybullet call overhead (flatters the reference)"}


def _cpu_env_worker(args):
    seconds, act, seed = args
    from oracle.ref_aviary import RefAviary
    A = 4 if act == "rpm" else 1
    rng = np.random.default_rng(seed)
    env = RefAviary(act=act, task="hover")
    env.reset()
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        a = rng.uniform(-1, 1, (1, A)).astype(np.float32)
        _, _, te, tr, _ = env.step(a)
        if te or tr:
            env.reset()
        steps += 1
    return steps, time.perf_counter() - t0


def job_cpus():
    """CPUs this job may use: the scheduler affinity, capped by the pool's per-job share
    (OMP_NUM_THREADS is set to it on the GPU box; os.cpu_count() there is the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline_procs(procs, seconds=10.0, act="rpm"):
    """The reference's own parallelism (SubprocVecEnv / make_vec_env(n_envs=...), examples/learn.py:53-57):
    one reference-shaped numpy env per process, `procs` processes stepping concurrently; value =
    the sum of their drone*dt/s."""
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_env_worker, [(seconds, act, 100 + i) for i in range(procs)])
    steps = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res) * 8
    model, ncpu = cpu_info()
    return {"value": rate, "unit": "drone*dt/s", "cores": procs, "kind": "port",
            "per_core": rate / procs,
            "sample": f"{procs} processes x one HoverAviary env (numpy fp64 restatement, DYN, RPM, U[-1,1], "
                      f"auto-reset), {steps} env.step() calls in {seconds:.0f} s on '{model}' "
                      f"({procs} of {ncpu} host CPUs: the job's CPU share)"}


def cpu_baseline_openmp(E, seconds=5.0, act="rpm", threads=16):
    """The C oracle (oracle/gpd_oracle.c, fp64, OpenMP over envs) stepping E HoverAviary envs on
    `threads` host cores: the optimised-CPU reference point for the same batched workload."""
    from oracle.c_oracle import COracle
    A = 4 if act == "rpm" else 1
    c = COracle(n_envs=E, task="hover", act=act, threads=threads)
    rng = np.random.default_rng(0)
    pool = rng.uniform(-1, 1, (8, E, 1, A)).astype(np.float32)
    c.step(pool[0])
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        c.step(pool[steps % 8])
        steps += 1
    el = time.perf_counter() - t0
    c.close()
    model, ncpu = cpu_info()
    return {"value": E * 8 * steps / el, "unit": "drone*dt/s", "cores": threads, "kind": "port",
            "sample": f"{steps} steps of {E} HoverAviary envs (C fp64 restatement, OpenMP, {threads} threads of "
                      f"'{model}') in {el:.1f} s"}


def state_parity(device, precision, E=256, T=150, seed=0):
    """The metric's "state L2" leg, run beside the CPU baseline (the oracle as the checker only):
    E HoverAviary envs (cf2x, DYN, RPM, auto-reset) stepped T = 150 ctrl steps (5 s, 1200
    substeps) on the GPU and by the C fp64 restatement of BaseAviary.step (oracle/gpd_oracle.c)
    on the same actions; per-drone relative L2 error of pos/quat/rpy/vel/ang_v after every step
    (tests/oracle_runs.py::state_rel_err, the parity tests' metric).  PyBullet itself is not
    available anywhere in this pipeline."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    from oracle.c_oracle import COracle

    def rel_err(a, b):
        a, b = a[..., :16], b[..., :16]
        d = a - b
        dq_flip = a[..., 3:7] + b[..., 3:7]
        flip = (dq_flip ** 2).sum(-1, keepdims=True) < (d[..., 3:7] ** 2).sum(-1, keepdims=True)
        d[..., 3:7] = np.where(flip, dq_flip, d[..., 3:7])
        return np.sqrt((d ** 2).sum(-1)) / np.maximum(np.sqrt((b ** 2).sum(-1)), 1e-6)

    rng = np.random.default_rng(seed)
    acts = np.clip(rng.normal(0, 0.1, (T, E, 1, 4)), -1, 1).astype(np.float32)
    acts[:, : E // 8] = rng.uniform(-1, 1, (T, E // 8, 1, 4)).astype(np.float32)   # forces resets
    sim = BatchedAviarySim(n_envs=E, task="hover", act=ActionType.RPM, precision=precision, autoreset=True,
                           device=device)
    orc = COracle(n_envs=E, task="hover", act="rpm")
    errs, n_done = [], 0
    for t in range(T):
        _, _, te, tr = sim.step(torch.from_numpy(acts[t]).to(device))
        _, _, te_o, tr_o = orc.step(acts[t])
        n_done += int(te_o.sum() + tr_o.sum())
        errs.append(rel_err(sim.state20().cpu().numpy(), orc.state20()))
    sim.close()
    orc.close()
    e = np.stack(errs)
    return {"state_rel_l2_max": float(e.max()), "state_rel_l2_median": float(np.median(e)),
            "gate": 1e-10 if precision == "f64" else 1e-3, "envs": E, "ctrl_steps": T, "substeps": T * 8,
            "episode_ends": n_done,
            "vs": "C fp64 restatement of BaseAviary.step (oracle/gpd_oracle.c); PyBullet is unavailable"}


def _timed_region(device, body):
    """The contract's timed region: barrier + synchronize, `body()` (K env.step launches),
    synchronize, and the wall time between.  No HIP events inside it: an event record before the
    first launch holds the queue for ~3-5 us, a fixed cost that is 4-5 % of a 20-step region
    (scripts/region_probe.py, profiles/r2/latency/region_*.txt)."""
    torch.cuda.synchronize(device)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    body()
    torch.cuda.synchronize(device)
    wall = time.perf_counter() - t0
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    return wall


def _event_region_us(device, body, launches, min_launches=256):
    """The same launches again, right after the timed region, repeated to at least
    `min_launches` step launches and bracketed by one HIP event pair on the launch stream:
    returns the step kernel's average duration in us, including the in-graph kernel boundary
    (an upper bound; rocprofv3 reports the kernel alone).  The repetition keeps the region's
    own fixed cost (queue start after the first event, the first launch's cold caches: ~10 us,
    DESIGN.md §7) from inflating the per-launch figure of a short (K = 20) timed region."""
    reps = max(1, -(-int(min_launches) // max(1, int(launches))))
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    ev0.record(stream)
    for _ in range(reps):
        body()
    ev1.record(stream)
    torch.cuda.synchronize(device)
    return 1000.0 * ev0.elapsed_time(ev1) / (reps * launches)


def time_graph(sim, pool, steps, warmup, per_graph=256):
    """Timed region in hipGraph mode: one graph = `per_graph` consecutive env.step() launches
    reading distinct pre-filled action slots, plus one graph of the remaining steps % per_graph
    launches, so that exactly `steps` steps are timed.  Before the timed region every captured
    graph is replayed at least once (the first replay of a graph pays its upload to the device),
    then `warmup` further untimed steps run, whatever `warmup` is.
    The kernel duration comes from _event_region_us over the same replays right after it (for
    fewer than 256 steps: over one 256-launch graph of the same kind).
    Returns (wall seconds, steps run, kernel us)."""
    P = pool.shape[0]
    steps = max(1, int(steps))
    per_graph = min(per_graph, steps)
    reps, rem = divmod(steps, per_graph)
    graph = sim.capture_graph([pool[k % P] for k in range(per_graph)])
    tail = sim.capture_graph([pool[k % P] for k in range(rem)]) if rem else None
    # first replays (graph upload) outside the timed region, then the requested warm-up steps
    graph.replay()
    if tail is not None:
        tail.replay()
    wreps, wrem = divmod(max(0, int(warmup)), per_graph)
    for _ in range(wreps):
        graph.replay()
    for k in range(wrem):
        sim.step(pool[k % P])

    def body():
        for _ in range(reps):
            graph.replay()
        if tail is not None:
            tail.replay()
    wall = _timed_region(sim.device, body)
    if steps >= 256:
        return wall, steps, _event_region_us(sim.device, body, steps)
    # a short timed region: the kernel time from one 256-launch graph of the same steps, so that
    # neither the region's fixed cost nor per-replay graph boundaries enter the per-launch figure
    long_graph = sim.capture_graph([pool[k % P] for k in range(256)])
    long_graph.replay()
    kern = _event_region_us(sim.device, long_graph.replay, 256)
    del long_graph                      # released here, not inside whatever is timed next
    torch.cuda.synchronize(sim.device)
    return wall, steps, kern


def time_native(sim, pool, steps, warmup):
    """Timed region as ONE gpd_step_seq call: `steps` env.step() launches issued back to back from
    native code (step k reads action slot k % P), no graph.  Its per-region fixed cost is a little
    below a graph replay's, but each launch costs the host ~5-6 us (about one kernel), so at large
    K it can turn host-bound (scripts/timing_probe.py); reported beside the graph timing.  Kernel
    duration from _event_region_us over the same call right after it.  Returns (wall s, steps, kernel us)."""
    steps = max(1, int(steps))
    sim.step_seq(pool, max(1, int(warmup)))

    def body():
        sim.step_seq(pool, steps)
    wall = _timed_region(sim.device, body)
    return wall, steps, _event_region_us(sim.device, body, steps)


def time_steps(sim, pool, steps, warmup):
    """Eager launches (one BatchedAviarySim.step() call per env.step, as an SB3-style caller
    makes them): the wall time of `steps` back-to-back calls, then a second pass with a HIP event
    pair around every gpd_step on the launch stream for the per-launch kernel time.
    Returns (wall seconds, mean kernel us)."""
    P = pool.shape[0]
    for k in range(warmup):
        sim.step(pool[k % P])
    torch.cuda.synchronize(sim.device)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    torch.cuda.synchronize(sim.device)
    t0 = time.perf_counter()
    for k in range(steps):
        sim.step(pool[(warmup + k) % P])
    torch.cuda.synchronize(sim.device)
    wall = time.perf_counter() - t0
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    stream = torch.cuda.current_stream(sim.device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for k in range(steps):
        ev[k][0].record(stream)
        sim.step(pool[(warmup + k) % P])
        ev[k][1].record(stream)
    torch.cuda.synchronize(sim.device)
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    return wall, 1000.0 * float(np.mean(kern_ms))


def launch_floor_us(device, launches=64, reps=20):
    """Per-launch cost of an EMPTY kernel replayed back to back from a hipGraph (torch's spin
    kernel with a zero count): the dependent kernel-boundary cost every step launch pays."""
    sleep = getattr(torch.cuda, "_sleep", None)
    x = torch.zeros(64, device=device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(launches):
            if sleep is not None:
                sleep(0)
            else:
                x.add_(1.0)
    for _ in range(3):
        g.replay()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    ev0.record()
    for _ in range(reps):
        g.replay()
    ev1.record()
    torch.cuda.synchronize(device)
    return 1000.0 * ev0.elapsed_time(ev1) / (launches * reps)


def latency_model(device, precision, act, E, kern_us, nsub):
    """Latency roofline of the bench config (the step is latency-bound at 4096 envs, DESIGN.md
    §7): step kernel time = launch floor + fixed in-kernel work (state/action loads, final
    readback + hooks, output rows) + nsub x the substep critical path.  The substep slope comes
    from the same workload at 1 and 16 substeps per control step (pyb_freq 30 / 480 Hz, ctrl
    30 Hz); the floor from an empty kernel.  'bound_us' = floor + nsub x slope is the time with
    zero prologue / epilogue; frac = bound / achieved."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    A = 4 if act == "rpm" else 1
    k = {}
    for pyb in (30, 480):
        sim = BatchedAviarySim(n_envs=E, task="hover", act=ActionType(act), precision=precision,
                               pyb_freq=pyb, ctrl_freq=30, device=device)
        pool = make_pool(E, A, device, seed=5, pool=16)
        k[pyb] = time_graph(sim, pool, 256, 32)[2]
        sim.close()
    slope = (k[480] - k[30]) / 15.0
    floor = launch_floor_us(device)
    fixed = k[30] - slope - floor
    model = floor + fixed + nsub * slope
    bound = floor + nsub * slope
    return {"launch_floor_us": floor, "per_substep_us": slope, "fixed_in_kernel_us": fixed,
            "kernel_us_1_substep": k[30], "kernel_us_16_substeps": k[480], "model_us": model,
            "achieved_us": kern_us, "bound_us": bound, "frac": bound / kern_us,
            "note": "kernel time = launch floor + fixed in-kernel work + substeps x substep critical path; "
                    "bound = floor + substeps x critical path (no prologue / epilogue)"}


def other_configs(device, precision, act):
    """BASELINE.json configs 3 and 4 and the controller action types, each timed like the main
    line (hipGraph replays of env.step for every env) - reported beside the metric, not as it."""
    import math
    from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    stag = [[0.15 * math.cos(2 * math.pi * i / 8), 0.15 * math.sin(2 * math.pi * i / 8), 0.5 + 0.1 * i] for i in range(8)]
    cases = [
        ("config3: 4096 HoverAviary envs, ground effect + drag on the DYN integrator",
         dict(n_envs=4096, task="hover", act=ActionType(act), physics=Physics.DYN, aero=("gnd", "drag")), 4),
        ("config4: 512 MultiHoverAviary x 8 drones, downwash (staggered init, SURVEY 8(d))",
         dict(n_envs=512, drones_per_env=8, task="multihover", act=ActionType.RPM, physics=Physics.DYN, aero=("dw",),
              initial_xyzs=stag), 4),
        ("4096 HoverAviary envs, ActionType.ONE_D_PID (batched DSLPIDControl + DYN)",
         dict(n_envs=4096, task="hover", act=ActionType.ONE_D_PID, physics=Physics.DYN), 1),
        ("4096 HoverAviary envs, ActionType.PID (waypoint + DSLPIDControl, Physics.PYB)",
         dict(n_envs=4096, task="hover", act=ActionType.PID, physics=Physics.PYB), 3),
        ("4096 HoverAviary envs, Physics.PYB (HoverAviary default: restated Bullet multibody step)",
         dict(n_envs=4096, task="hover", act=ActionType(act), physics=Physics.PYB), 4),
        ("512 MultiHoverAviary x 8 drones, Physics.PYB_GND_DRAG_DW (Bullet step, staggered init)",
         dict(n_envs=512, drones_per_env=8, task="multihover", act=ActionType.RPM, physics=Physics.PYB_GND_DRAG_DW,
              initial_xyzs=stag), 4),
        ("512 MultiHoverAviary x 8 drones, Physics.PYB (the same staggered batch without the downwash, "
         "whose (r/4dz)^2 force drives the row above into piles)",
         dict(n_envs=512, drones_per_env=8, task="multihover", act=ActionType.RPM, physics=Physics.PYB,
              initial_xyzs=stag), 4),
        ("2048 MultiHoverAviary x 2 drones, Physics.PYB (MultiHoverAviary's default, examples/learn.py "
         "--multiagent's env; drone<->drone and plane contact)",
         dict(n_envs=2048, drones_per_env=2, task="multihover", act=ActionType.RPM, physics=Physics.PYB), 4),
    ]
    out = []
    for name, kw, A in cases:
        sim = BatchedAviarySim(precision=precision, autoreset=True, device=device, **kw)
        E, D = sim.n_envs, sim.drones_per_env
        g = torch.Generator(device=device)
        g.manual_seed(3)
        pool = (torch.rand((16, E, D, A), generator=g, device=device) * 2 - 1).contiguous()
        if A == 3:
            pool *= 0.5
        w, n, k = time_graph(sim, pool, 64, 16)
        out.append({"config": name, "n_drones": E * D, "kernel_us": k, "ms_per_step": 1000 * w / n,
                    "value": E * D * sim.pyb_steps_per_ctrl * n / w, "unit": "drone*dt/s"})
        sim.close()
    return out


def _policy_mlp(n_in, n_out):
    """SB3 MlpPolicy's network (examples/learn.py mlp: [64, 64] tanh), random-initialised."""
    import torch.nn as nn
    return nn.Sequential(nn.Linear(n_in, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, n_out))


def handoff_leg(sim, global_envs, hmode, cap, gpool, G, rank, device, force=False):
    """One LearnerHandoff configuration, per step.  ``ms_per_step``: a hand-off step (action
    scatter + shard step + pack + ONE collective + unpack) inside a captured graph of 32 of them,
    by HIP events - how examples/learn.py runs it (the fused rollout replays n_steps of them with
    the policy kernel between, ``rollout_with_policy_us_per_step``); ``replay_ms_per_step``: one
    ``step()`` call per step replaying the captured one-step graph (the host's launch included);
    ``eager_ms_per_step``: the same calls without a graph (G steps after 3 warm ones, wall clock,
    max over ranks).  Also the bytes that land per step, how many steps needed the second
    (overflow) exchange and the finished-env rate of the batch.  A ``terminal_capacity`` below the
    shard reads the finished count on the host every step: eager only."""
    import torch.distributed as dist

    from gym_pybullet_drones_routing_amd.shard import LearnerHandoff, max_over_ranks
    h = LearnerHandoff(sim, global_envs, mode=hmode, force_collectives=force, terminal_capacity=cap)
    fin = torch.zeros((G,), dtype=torch.int64, device=device)

    def timed():
        for k in range(3):
            h.step(gpool[k % 8] if rank == 0 else None)
        torch.cuda.synchronize(device)
        dist.barrier()
        torch.cuda.synchronize(device)
        h.terminal_bytes, h.steps, h.second_exchanges = 0, 0, 0
        t0 = time.perf_counter()
        for k in range(G):
            r = h.step(gpool[k % 8] if rank == 0 else None)
            if r is not None:
                fin[k] = (r[2] | r[3]).sum()
        torch.cuda.synchronize(device)
        return max_over_ranks(time.perf_counter() - t0, device)

    def graph_us(body, k=32, reps=4):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(k):
                body()
        g.replay()
        torch.cuda.synchronize(device)
        dist.barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(reps):
            g.replay()
        ev1.record()
        torch.cuda.synchronize(device)
        del g
        return max_over_ranks(1000.0 * ev0.elapsed_time(ev1) / (reps * k), device)

    eager = timed()
    out = dict(h.stats(), eager_ms_per_step=1000 * eager / G)
    if not h.host_sync_per_step and not h._stage:
        src = h.global_actions if h.is_learner else None
        out["ms_per_step"] = graph_us(lambda: h.step_body(src)) / 1000.0
        if hmode == "gather":
            # the config-5 RL step: the fused policy kernel on the learner's gathered batch (the
            # bench's 64-64 tanh actor + critic), then the hand-off step, as learn.py's rollout
            from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
            Eg, D, W, A = global_envs, sim.drones_per_env, sim.obs_width, sim.act_width

            class _AC(torch.nn.Module):
                def __init__(self):
                    super().__init__()
                    self.pi, self.vf = _policy_mlp(D * W, D * A), _policy_mlp(D * W, 1)
                    self.log_std = torch.nn.Parameter(torch.zeros(D * A))
            if h.is_learner:
                torch.manual_seed(0)
                kern = MlpPolicyKernel(_AC().to(device), seed=3)
                bufs = [torch.zeros((Eg, D * W), device=device), torch.zeros((Eg, D * A), device=device),
                        torch.zeros(Eg, device=device), torch.zeros(Eg, device=device),
                        torch.zeros(Eg, device=device), torch.zeros(Eg, device=device)]
                obs_v, tobs_v = h.obs.view(Eg, -1), h.terminal_rows.view(Eg, -1)

                def body():
                    kern.step(obs_v, h.global_actions.view(Eg, -1), *bufs[:4],
                              prev=(h.reward, h.terminated, h.truncated, tobs_v), buf_rew=bufs[4], buf_done=bufs[5])
                    h.step_body(h.global_actions)
            else:
                def body():
                    h.step_body(None)
            with torch.no_grad():
                out["rollout_with_policy_us_per_step"] = graph_us(body)
        h.capture()                       # step() replays one captured hand-off step from now on
        out["replay_ms_per_step"] = 1000 * timed() / G
        out["graphed"] = True
    else:
        out["ms_per_step"] = out["eager_ms_per_step"]
    if rank == 0:
        f = fin.double()
        out["finished_envs_per_step"] = {"mean": float(f.mean()), "max": int(fin.max()),
                                         "frac_mean": float(f.mean()) / global_envs}
    h.close()
    return out


def rollout_leg(device, precision, act, E, K=64, reps=8, store_policy=2):
    """What an RL caller pays per env.step (the caller: examples/learn.py's PPO rollout, the
    reference's learn.py:52-94 through SB3): ONE hipGraph of K x (policy, gpd_step) at E envs,
    against the same graph without gpd_step, by HIP events over graph replays.  The policy is the
    fused rollout kernel (``policy.MlpPolicyKernel``: actor + critic 64-64 tanh forward, Normal
    sample, clip, the rollout-buffer rows and the previous step's time-limit bootstrap in one
    launch; what examples/learn.py runs) and, beside it under ``torch_policy``, the same work as
    torch library calls (nn.Linear / tanh / randn / clamp / copies).  ``store_policy``:
    gpd_config::store_policy; 2 (write-through rows), what examples/learn.py sets (between the
    policy's kernels it measured 6.12 vs 6.40 us per step against the default 3,
    profiles/r4/rollout_policy/)."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    tuning = {"store_policy": store_policy} if store_policy else None
    sim = BatchedAviarySim(n_envs=E, task="hover", act=ActionType(act), precision=precision, autoreset=True,
                           device=device, tuning=tuning)
    W, A = sim.obs_width, sim.act_width
    torch.manual_seed(0)

    class _AC(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.pi, self.vf = _policy_mlp(W, A), _policy_mlp(W, 1)
            self.log_std = torch.nn.Parameter(torch.zeros(A))

    ac = _AC().to(device)
    pi, vf, log_std = ac.pi, ac.vf, ac.log_std.detach()
    obs = sim.obs.view(E, W)                      # sim-owned, rewritten in place by every step
    tobs = sim.terminal_obs.view(E, W)
    act_buf = torch.zeros((E, 1, A), device=device)
    buf_obs = torch.zeros((K, E, W), device=device)
    buf_act = torch.zeros((K, E, A), device=device)
    buf_val = torch.zeros((K, E), device=device)
    buf_logp = torch.zeros((K, E), device=device)
    buf_rew = torch.zeros((K, E), device=device)
    buf_done = torch.zeros((K, E), device=device)
    kern = MlpPolicyKernel(ac, seed=1)

    def seq_torch(with_step):
        for t in range(K):
            mu = pi(obs)
            v = vf(obs).squeeze(-1)
            a = mu + log_std.exp() * torch.randn_like(mu)
            act_buf.copy_(a.clamp(-1.0, 1.0).view(E, 1, A))     # SB3 clips to the Box
            buf_obs[t].copy_(obs)
            buf_act[t].copy_(a)
            buf_val[t].copy_(v)
            if with_step:
                sim.step(act_buf)
            buf_rew[t].copy_(sim.reward)
            buf_done[t].copy_(torch.logical_or(sim.terminated, sim.truncated))

    def seq_fused(with_step):
        for t in range(K):
            prev = (sim.reward, sim.terminated, sim.truncated, tobs) if t else None
            kern.step(obs, act_buf.view(E, A), buf_obs[t], buf_act[t], buf_logp[t], buf_val[t], prev=prev,
                      buf_rew=buf_rew[t - 1] if t else None, buf_done=buf_done[t - 1] if t else None)
            if with_step:
                sim.step(act_buf)

    def measure(seq):
        res = {}
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):             # warm the library kernels before capture
            seq(False)
        torch.cuda.current_stream(device).wait_stream(side)
        for name, with_step in (("policy_only", False), ("rollout", True)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                seq(with_step)
            g.replay()
            g.replay()
            res[name + "_us_per_step"] = _event_region_us(device, g.replay, K, min_launches=K * reps)
            del g
        res["step_in_rollout_us"] = res["rollout_us_per_step"] - res["policy_only_us_per_step"]
        return res

    with torch.no_grad():
        out = measure(seq_fused)
        out["torch_policy"] = measure(seq_torch)
    out.update({"n_envs": E, "steps_per_graph": K, "store_policy": store_policy or "library default",
                "what": "one hipGraph of K x (fused policy kernel: actor + critic 64-64 tanh MLP forward, Normal "
                        "sample, clip, rollout-buffer rows, previous step's bootstrap; gpd_step) vs the same without "
                        "gpd_step; step_in_rollout = the difference; torch_policy = the policy as torch library "
                        "calls"})
    sim.close()
    torch.cuda.synchronize(device)
    return out


def hbm_copy_gbps(device, n=1 << 28, reps=5):
    """torch copy_ of n float32 (1 GiB, far past the 256 MB Infinity Cache), bytes read + written
    per second: reported beside the HIP ceiling below (torch's copy keeps one load per lane in
    flight and measured ~5.0 TB/s where a deeper copy reaches ~6.1)."""
    x = torch.empty(n, device=device)
    y = torch.empty(n, device=device)
    y.copy_(x)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(reps):
        y.copy_(x)
    torch.cuda.synchronize(device)
    el = (time.perf_counter() - t0) / reps
    del x, y
    torch.cuda.empty_cache()
    return 2 * n * 4 / el / 1e9


HBM_CEILING_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scripts", "ubench", "libhbm_ceiling.so")


def hbm_ceiling(device):
    """The achievable HBM rate on this box, measured live (scripts/ubench/hbm_ceiling.hip,
    built in-tree as libhbm_ceiling.so): coalesced float4 copy / read-only streams far past the
    Infinity Cache, best over 1-8 loads in flight per lane, plain or nontemporal, 1-8 blocks of 256
    threads per CU (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy).  None when the library is
    absent (the torch copy_ figure stays beside it)."""
    if not os.path.exists(HBM_CEILING_LIB):
        return None
    import ctypes
    lib = ctypes.CDLL(HBM_CEILING_LIB)
    lib.hbm_ceiling_gbps.restype = ctypes.c_double
    lib.hbm_ceiling_gbps.argtypes = [ctypes.c_int, ctypes.c_int]
    with torch.cuda.device(device):
        copy = lib.hbm_ceiling_gbps(0, 0)
        read = lib.hbm_ceiling_gbps(1, 0)
    torch.cuda.empty_cache()
    if copy <= 0 or read <= 0:
        return None
    return {"copy_GBps": copy, "read_GBps": read,
            "source": "scripts/ubench/hbm_ceiling.hip (float4 streams, 704 MB per launch, best of the "
                      "in-flight-depth x policy x blocks-per-CU sweep)"}


def raw_integrator(device, precision, n_drones=1 << 20, n_sub=32):
    """SURVEY §8(d) raw-integrator mode: gpd_integrate with the RPMs streamed per substep
    ([n_sub][N][4] real), state in registers for all n_sub substeps, no trajectory; algorithmic
    bytes = n_sub*N*4r (RPMs) + N*17r (state + last RPM read) + N*20r (state written)."""
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    sim = BatchedAviarySim(n_envs=n_drones, task="none", precision=precision, autoreset=False, device=device)
    r = 8 if precision == "f64" else 4
    dt = torch.float64 if precision == "f64" else torch.float32
    rpm = (14468.43 * (1 + 0.05 * (torch.rand((n_sub, n_drones, 4), device=device) * 2 - 1))).to(dt).contiguous()
    for _ in range(2):
        sim.integrate(rpm)
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    torch.cuda.synchronize(device)
    ev0.record(stream)
    for _ in range(reps):
        sim.integrate(rpm)
    ev1.record(stream)
    torch.cuda.synchronize(device)
    us = 1000.0 * ev0.elapsed_time(ev1) / reps
    alg = n_sub * n_drones * 4 * r + n_drones * 17 * r + n_drones * 20 * r
    sim.close()
    del rpm
    torch.cuda.empty_cache()
    return {"mode": f"gpd_integrate, {n_sub} substeps per launch, RPMs streamed from HBM, no trajectory",
            "n_drones": n_drones, "kernel_us": us, "value": n_drones * n_sub / (us * 1e-6), "unit": "drone*dt/s",
            "achieved_GBps": alg / (us * 1e-6) / 1e9, "frac": alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS,
            "alg_bytes_per_drone_dt": (alg / (n_drones * n_sub))}


def make_pool(E, A, device, seed, pool=64):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return (torch.rand((pool, E, 1, A), generator=g, device=device) * 2 - 1).contiguous()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the env, bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--act", default="rpm", choices=["rpm", "one_d_rpm"])
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"],
                    help="f64 (default) is the parity-gated path (<=1e-10 vs the fp64 oracle)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes of the all-core CPU baseline (0 = the CPUs this job may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--no-latency-model", action="store_true",
                    help="skip the latency-model leg (its 1- and 16-substep launches share the bench kernel's "
                         "name and grid, so a rocprofv3 trace of the bench kernel leaves it out)")
    ap.add_argument("--no-handoff", action="store_true",
                    help="skip the one-GPU learner hand-off leg (a one-rank RCCL group)")
    ap.add_argument("--no-rollout", action="store_true",
                    help="skip the RL-rollout leg (its step launches share the bench kernel's name and grid)")
    ap.add_argument("--mode", default="graph", choices=["native", "graph", "eager"],
                    help="timed region: hipGraph replays (default), a native launch loop (gpd_step_seq), or "
                         "one Python step() call per env.step")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the real multi-GPU path); gloo only to rehearse several ranks on one GPU")
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, world, port, argv):
    """A self-launched rank (fresh interpreter, torch.multiprocessing spawn): the torchrun env."""
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run(parse_args(argv))


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}; launch one rank per GPU")
        run(args)
        return
    if args.gpus <= 1:
        run(args)
        return
    # --gpus N without a launcher: start N rank processes before anything touches the GPU
    # (device_count() does not initialise HIP on this image)
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and n_dev < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs for RCCL, {n_dev} visible "
                         "(--dist-backend gloo rehearses several ranks on one GPU)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, args.gpus, port, sys.argv[1:])) for r in range(args.gpus)]
    for p in procs:
        p.start()
    codes = []
    for p in procs:
        p.join()
        codes.append(p.exitcode)
    bad = [c for c in codes if c != 0]
    if bad:
        raise SystemExit(f"bench.py: rank exit codes {codes}")


_JSON_FD = None     # the process's real stdout while fd 1 points at stderr (run())


class _HandoffWatchdog:
    """N > 1: the hand-off legs run last, and theirs are the only collectives of the run that span
    GPUs (one-rank RCCL is all this pipeline can execute before the driver's multi-GPU runs).
    Should they hang, the weak-scaling line must still come out: after ``limit`` s rank 0 writes
    the line measured so far with ``handoff = {"error": ...}`` to the real stdout and every rank
    ends its process (os._exit: no collective teardown to wait for)."""

    def __init__(self, result, rank, limit):
        import threading
        self.result, self.rank, self.limit = result, rank, limit
        self.timer = threading.Timer(limit, self._fire)
        self.timer.daemon = True
        self.timer.start()

    def _fire(self):
        if self.rank == 0 and self.result is not None and _JSON_FD is not None:
            line = dict(self.result, handoff={"error": f"hand-off legs unfinished after {self.limit:.0f} s "
                                                       "(watchdog; the step line above them is complete)"})
            os.write(_JSON_FD, (json.dumps(line) + "\n").encode())
        os._exit(0)

    def cancel(self):
        self.timer.cancel()


def run(args):
    # the JSON line is the only thing this process writes to stdout: native libraries write to fd 1
    # directly (RCCL prints its version banner when it creates a communicator), so fd 1 points at
    # stderr until the line is printed; restored whatever happens
    global _JSON_FD
    sys.stdout.flush()
    json_fd = os.dup(1)
    _JSON_FD = json_fd
    os.dup2(2, 1)
    try:
        result = _run(args)
    finally:
        sys.stdout.flush()
        os.dup2(json_fd, 1)
        os.close(json_fd)
        _JSON_FD = None
    if result is not None:
        print(json.dumps(result), flush=True)


def _run(args):
    """One rank's bench; rank 0 returns the result dict (None elsewhere)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local_rank
    if args.dist_backend == "gloo":
        dev_index = local_rank % torch.cuda.device_count()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_index}"))
        else:
            torch.distributed.init_process_group("gloo")
    device = torch.device(f"cuda:{dev_index}")
    torch.cuda.set_device(device)

    from gym_pybullet_drones_routing_amd.enums import ActionType
    from gym_pybullet_drones_routing_amd.shard import LearnerHandoff, max_over_ranks, rank_seed
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim

    E = args.envs
    A = 4 if args.act == "rpm" else 1
    sim = BatchedAviarySim(n_envs=E, task="hover", act=ActionType(args.act), precision=args.precision,
                           autoreset=True, device=device)
    nsub = sim.pyb_steps_per_ctrl
    pool = make_pool(E, A, device, seed=rank_seed(1000, rank))
    # (1) eager pass (also the SB3-style per-call number); per-launch event pairs
    eager_wall, eager_kern_us = time_steps(sim, pool, args.steps, args.warmup)
    # (2) timed pass: the same steps replayed from a hipGraph (no host launch overhead); the
    #     roofline's kernel duration comes from the events around these replays
    # the other launch form beside it (same K; native loop when graphs are timed, and back), run
    # first: native launches issued after graph replays measured slower
    n_wall, n_steps, n_kern = (time_native if args.mode != "native" else time_graph)(sim, pool, args.steps, args.warmup)
    if args.mode == "eager":
        wall, steps_run, kern_us = eager_wall, args.steps, eager_kern_us
    elif args.mode == "native":
        wall, steps_run, kern_us = time_native(sim, pool, args.steps, args.warmup)
    else:
        wall, steps_run, kern_us = time_graph(sim, pool, args.steps, args.warmup)
    other_leg = {"mode": "native" if args.mode != "native" else "graph", "ms_per_step": 1000.0 * n_wall / n_steps,
                 "value": E * nsub * n_steps / n_wall, "kernel_us_per_launch_events": n_kern}
    wall = max_over_ranks(wall, device)
    eager_wall = max_over_ranks(eager_wall, device)
    drone_dt = world * E * nsub * steps_run
    value = drone_dt / wall
    ms_per_step = 1000.0 * wall / steps_run
    rbytes = 8 if args.precision == "f64" else 4
    alg = alg_bytes_per_drone_step(args.act, rbytes) * E
    achieved = alg / (kern_us * 1e-6) / 1e9
    result = {
        "metric": "env-steps/sec (drone·dt) at 4096 envs, 1/2/4/8 GPU; state L2 vs PyBullet",
        "value": value, "unit": "drone*dt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32" if args.precision == "f32" else "f64", "data": "synthetic",
        "mode": {"eager": "one Python BatchedAviarySim.step() call per env.step",
                 "graph": "hipGraph replay, up to 256 env.step launches per graph (+ one graph of the remainder)",
                 "native": "one gpd_step_seq call: K env.step launches back to back from native code"}[args.mode],
        "config": {"workload": f"{E} HoverAviary envs per GPU (cf2x, Physics.DYN, ActionType.{args.act.upper()}, "
                               f"240/30 Hz = {nsub} substeps/step, U[-1,1] actions, SB3 auto-reset)",
                   "n_envs_per_gpu": E, "global_envs": E * world, "drones_per_env": 1,
                   "parallelism": f"env-sharded x{world} (no collective in the step loop)"},
        "kernel_us": kern_us,
        "timed_region_note": ("a timed region carries a fixed ~18 us HIP round trip (graph launch -> first kernel, "
                              "completion -> synchronize return), ~0.9 us/step at K = 20; per-step cost without it "
                              "= kernel_us (DESIGN.md §7.1)") if args.steps < 100 else None,
        "eager": {"ms_per_step": 1000.0 * eager_wall / args.steps,
                  "value": world * E * nsub * args.steps / eager_wall,
                  "kernel_us_per_launch_events": eager_kern_us},
        "ctrl_steps_per_s": world * E * args.steps / wall,
        "other_launch_form": other_leg,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "traffic_unit": "bytes per launch",
                     "kernel": step_kernel_name(sim, rbytes, args.act),
                     "alg_bytes_per_launch": alg},
    }

    grid_lanes = -(-sim.n_drones // sim.constants.drones_per_block) * sim.constants.lanes_per_block  # launch geometry
    result["roofline"]["grid_lanes"] = grid_lanes
    rp = rocprof_kernel_us(result["roofline"]["kernel"], grid_lanes, args.precision)
    if rp is not None:
        result["roofline"]["kernel_us_rocprof"] = rp[0]
        result["roofline"]["kernel_us_rocprof_source"] = rp[1]
        # the same fraction from the committed rocprofv3 trace's durations, so the line follows
        # profiles/: the mean over all launches (most of them isolated by the profiler: what a
        # caller that does other work between steps pays) and the back-to-back median
        result["roofline"]["frac_rocprof_mean"] = alg / (rp[0] * 1e-6) / 1e9 / HBM_PEAK_GBPS
        if rp[2] is not None:
            # the profiler leaves most launches isolated (each waits for the host); the ones that
            # still ran back to back, as in the graph-replayed timed region, are the like-for-like
            # figure for kernel_us (scripts/prof_summary.py B2B_US)
            result["roofline"]["kernel_us_rocprof_back_to_back_median"] = rp[2]
            result["roofline"]["frac_rocprof_back_to_back"] = alg / (rp[2] * 1e-6) / 1e9 / HBM_PEAK_GBPS
    tr = pmc_traffic(grid_lanes, args.precision)
    if tr is not None:
        result["roofline"]["traffic"] = tr[0]
        result["roofline"]["traffic_source"] = tr[1] + " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes)"
        ifetch = instruction_fetch_bytes(result["roofline"]["kernel"], grid_lanes)
        if ifetch is not None:
            # FETCH_SIZE also counts the kernel's instruction fetch (calibrated on a kernel that
            # touches no data, profiles/r3/icache/): the data traffic is what remains
            result["roofline"]["traffic_instruction_fetch"] = 2 * ifetch
            result["roofline"]["traffic_data"] = tr[0] - 2 * ifetch
    # strong scaling: config 5's 32768 envs in total, split over the ranks (at N = 8
    # the weak line's 4096 per GPU); the driver's N = 1/2/4/8 runs then hold both curves
    if STRONG_ENVS % world == 0:
        Es = STRONG_ENVS // world
        ss = BatchedAviarySim(n_envs=Es, task="hover", act=ActionType(args.act), precision=args.precision,
                              autoreset=True, device=device)
        sp = make_pool(Es, A, device, seed=rank_seed(2000, rank), pool=16)
        Ks = 64
        ws, ns, ks = time_graph(ss, sp, Ks, 16)
        ws = max_over_ranks(ws, device)
        result["strong"] = {"scaling": "strong", "global_envs": STRONG_ENVS, "envs_per_gpu": Es,
                            "ms_per_step": 1000.0 * ws / ns, "value": STRONG_ENVS * nsub * ns / ws,
                            "kernel_us": ks, "steps": ns}
        ss.close()
        del sp
    if world > 1 or (rank == 0 and not args.no_handoff):
        # config 5: the learner hand-off (shard.LearnerHandoff): rank 0 scatters the global action
        # batch, every rank steps its shard and packs its record (obs, reward, terminated,
        # truncated, the finished envs' 12 state columns), ONE collective brings the records to the
        # learner ("gather") or to every rank ("all_gather"), one kernel unpacks them.  One GPU: a
        # one-rank RCCL group with the collectives forced, so the same calls run as on a node.  An
        # optional leg: a failure is recorded, never the end of the run
        one_rank = world == 1
        created = False
        dog = _HandoffWatchdog(result if rank == 0 else None, rank, 240.0) if world > 1 else None
        try:
            if one_rank and args.dist_backend == "nccl" and not torch.distributed.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ["MASTER_PORT"] = str(_free_port())
                torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=device)
                created = True
            if torch.distributed.is_initialized():
                gpool = make_pool(E * world, A, device, seed=11, pool=8) if rank == 0 else None
                G = max(30, args.steps // 3)
                coll = "RCCL" if args.dist_backend == "nccl" else "gloo (rehearsal, through host memory)"
                legs = {hmode: handoff_leg(sim, E * world, hmode, None, gpool, G, rank, device, force=one_rank)
                        for hmode in ("gather", "all_gather")}
                cap = max(1, E // 8)
                sync_legs = {f"{hmode}_cap{cap}": handoff_leg(sim, E * world, hmode, cap, gpool, G, rank, device,
                                                              force=one_rank)
                             for hmode in ("gather", "all_gather")}
                result["handoff"] = {
                    "mode": f"learner hand-off per step ({coll}{', one rank, collectives forced' if one_rank else ''}): "
                            "actions from rank 0 (grouped RCCL send / recv), shard step, pack kernel (the finished "
                            "envs' 12 state columns into the record), ONE collective of the records (gather = "
                            "grouped RCCL send / recv to the learner, all_gather = ncclAllGather; rccl.RcclComm), "
                            "unpack kernel; ms_per_step = one hand-off step inside a captured graph of 32 (HIP "
                            "events; how examples/learn.py's fused rollout runs it, rollout_with_policy_us_per_step "
                            "with its policy kernel), replay_ms_per_step = one step() call replaying the captured "
                            "one-step graph, eager_ms_per_step = the same calls without a graph",
                    "step_only_ms": 1000.0 * eager_wall / args.steps, "legs": legs,
                    "synchronising_legs": sync_legs,
                    "synchronising_legs_note": f"terminal_capacity {cap} < shard: the finished envs' columns compacted "
                                               "into a fixed block, the largest finished count read ON THE HOST every "
                                               "step (one synchronisation; not capturable), a second exchange on "
                                               "overflow"}
        except Exception as exc:
            result["handoff"] = {"error": f"{type(exc).__name__}: {exc}"}
        finally:
            if dog is not None:
                dog.cancel()
            if created:
                torch.distributed.destroy_process_group()

    if rank == 0 and world == 1 and not args.no_latency_model:
        result["roofline"]["latency_model"] = latency_model(device, args.precision, args.act, E, kern_us, nsub)
    if rank == 0 and world == 1 and not args.no_rollout:
        result["rollout"] = rollout_leg(device, args.precision, args.act, E)
    if rank == 0 and world == 1 and not args.no_sweep:
        sweep = []
        for e_large in (65536, 1 << 20, 1 << 22):
            s2 = BatchedAviarySim(n_envs=e_large, task="hover", act=ActionType(args.act),
                                  precision=args.precision, autoreset=True, device=device)
            p2 = make_pool(e_large, A, device, seed=7, pool=16)
            w2, n2, k2 = time_graph(s2, p2, 32, 16)
            ach = alg_bytes_per_drone_step(args.act, rbytes) * e_large / (k2 * 1e-6) / 1e9
            sweep.append({"n_envs": e_large, "kernel_us": k2, "ms_per_step": 1000 * w2 / n2,
                          "value": e_large * nsub * n2 / w2, "achieved_GBps": ach, "frac": ach / HBM_PEAK_GBPS})
            s2.close()
            del p2
            torch.cuda.empty_cache()
        torch_copy = hbm_copy_gbps(device)
        ceil = hbm_ceiling(device)
        copy = ceil["copy_GBps"] if ceil else torch_copy
        for row in sweep:
            row["frac_of_copy"] = row["achieved_GBps"] / copy
            if row["n_envs"] * alg_bytes_per_drone_step(args.act, rbytes) < 256 * 2 ** 20:
                # the whole working set fits the 256 MB Infinity Cache: not an HBM measurement
                row["mall_resident"] = True
                row["frac"] = None
                row["frac_of_copy"] = None
        result["sweep"] = sweep
        result["hbm_copy_GBps"] = copy
        result["hbm_copy_torch_GBps"] = torch_copy
        result["hbm_ceiling"] = ceil

    if rank == 0 and world == 1 and not args.no_sweep:
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            result["other_configs"] = other_configs(device, args.precision, args.act)
        result["raw_integrator"] = raw_integrator(device, args.precision)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the reference's parallelism: one numpy env per process on every CPU of the job's share
        # (cpu_baseline), beside the same on 1 core and the C/OpenMP restatement on those CPUs
        ncores = args.cpu_procs or job_cpus()
        one = cpu_baseline(args.cpu_seconds, args.act)
        try:
            result["cpu_baseline"] = cpu_baseline_procs(ncores, args.cpu_seconds, args.act)
        except Exception as exc:
            result["cpu_baseline"] = dict(one, error_all_cores=str(exc))
        result["cpu_baseline_1core"] = one
        result["speedup_vs_cpu_baseline"] = value / result["cpu_baseline"]["value"]
        try:
            result["cpu_baseline_openmp"] = cpu_baseline_openmp(E, args.cpu_seconds, args.act, threads=ncores)
        except Exception as exc:  # the C oracle is optional for the bench
            result["cpu_baseline_openmp"] = {"error": str(exc)}
        try:
            result["parity"] = state_parity(device, args.precision)
        except Exception as exc:
            result["parity"] = {"error": str(exc)}

    sim.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    return result if rank == 0 else None


if __name__ == "__main__":
    main()
