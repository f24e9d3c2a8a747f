"""Measured parity margins of the HIP path vs the fp64 oracle (for DESIGN.md): max / median
per-drone relative state error over 5 s of raw integration (plain DYN, with aero terms, with
downwash) and over step() rollouts, f64 and f32."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle.ref_aviary import RefAviary, rpm_from_action
from tests.oracle_runs import run_integrate, run_vec, state_rel_err
from tests.test_gpu_parity import _random_raw, HOVER
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
rng = np.random.default_rng(0)
n, T = 64, 1200
raw0 = _random_raw(rng, n)
rpms = rpm_from_action(HOVER, rng.uniform(-1, 1, (T, n, 4)).astype(np.float32))
for label, aero, z in (("DYN", (), 1.0), ("DYN + gnd + drag", ("gnd", "drag"), 0.06)):
    r0 = raw0.copy(); r0[:, 2] = z + rng.uniform(-0.01, 0.01, n)
    ref = run_integrate(rpms * (0.5 if aero else 1.0) + (HOVER * 0.5 if aero else 0.0), r0, aero=aero)
    for prec in ("f64", "f32"):
        sim = BatchedAviarySim(n_envs=n, task="none", precision=prec, aero=aero, device="cuda:0")
        sim.set_raw_state(r0)
        traj = sim.integrate(rpms * (0.5 if aero else 1.0) + (HOVER * 0.5 if aero else 0.0), record=True).cpu().numpy()
        err = state_rel_err(traj, ref)
        print(f"integrate 5 s, {label}, {prec}: max {err.max():.2e}  median {np.median(err):.2e}", flush=True)
        sim.close()
E, Tst = 16, 120
acts = np.clip(rng.normal(0, 0.15, (Tst, E, 1, 4)), -1, 1).astype(np.float32)
envs = []
run_vec(acts, E, envs=envs)
ref = np.concatenate([e.state20() for e in envs])
for prec in ("f64", "f32"):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision=prec, device="cuda:0")
    for t in range(Tst):
        sim.step(torch.from_numpy(acts[t]).cuda())
    err = state_rel_err(sim.state20().cpu().numpy(), ref)
    print(f"step() 120 ctrl steps, hover-biased actions, {prec}: max {err.max():.2e}  median {np.median(err):.2e}", flush=True)
    sim.close()
