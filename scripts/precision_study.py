"""f32 vs f64 kernel: state error growth vs the fp64 oracle, and step-kernel time."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle.ref_aviary import rpm_from_action
from tests.oracle_runs import run_integrate, state_rel_err
from tests.test_gpu_parity import _random_raw, HOVER
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
rng = np.random.default_rng(0)
n, T = 64, 1200
for label, tilt, spin, scale in (("random init, U[-1,1] rpm/substep", 0.3, 2.0, 1.0), ("hover init, U[-1,1]/ctrl step", 0.0, 0.0, 1.0)):
    raw0 = _random_raw(rng, n, tilt=tilt, spin=spin)
    if spin == 0.0:
        a = rng.uniform(-1, 1, (T // 8, n, 4)).astype(np.float32)
        rpms = np.repeat(rpm_from_action(HOVER, a), 8, axis=0)
    else:
        rpms = rpm_from_action(HOVER, rng.uniform(-1, 1, (T, n, 4)).astype(np.float32) * np.float32(scale))
    ref = run_integrate(rpms, raw0)
    for prec in ("f32", "f64"):
        sim = BatchedAviarySim(n_envs=n, task="none", precision=prec, device="cuda:0")
        sim.set_raw_state(raw0)
        traj = sim.integrate(rpms, record=True).cpu().numpy()
        err = state_rel_err(traj, ref)
        print(f"{label} {prec}: max rel err at 1s {err[:240].max():.2e} 2s {err[:480].max():.2e} 5s {err.max():.2e}; median@5s {np.median(err[-1]):.2e}")
        sim.close()
for prec in ("f32", "f64"):
    for E in (4096, 1 << 20):
        sim = BatchedAviarySim(n_envs=E, task="hover", precision=prec, device="cuda:0")
        acts = (torch.rand((8, E, 1, 4), device="cuda:0") * 2 - 1).contiguous()
        for k in range(10): sim.step(acts[k % 8])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for k in range(50): sim.step(acts[k % 8])
        e.record(); torch.cuda.synchronize()
        print(f"step {prec} E={E}: {1000*s.elapsed_time(e)/50:.1f} us/step")
        sim.close()
