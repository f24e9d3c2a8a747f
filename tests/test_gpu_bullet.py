"""GPU-vs-oracle parity of the Physics.PYB* path: the reference's link forces
handed to the restated Bullet3 multibody base step (oracle/bullet_mb.py), through the C ABI.

Same gates as tests/test_gpu_parity.py: per-drone relative L2 error of the state over every
substep, fp64 max <= 1e-10; fp32 median <= 1e-5 and max <= 1e-3.  Parity here is against the
restatement (pybullet itself is unavailable: "parity unpinned", see oracle/bullet_mb.py).
"""
import math

import numpy as np
import pytest
import torch

from oracle.ref_aviary import RefAviary
from tests.oracle_runs import assert_obs_match, run_integrate, run_vec, state_rel_err
from tests.test_gpu_parity import HOVER, TOL, TOL_MEDIAN, _random_raw, _rpms, _sim, _staggered

pytestmark = pytest.mark.gpu


def _physics(aero):
    from gym_pybullet_drones_routing_amd.enums import Physics
    return {(): Physics.PYB, ("gnd",): Physics.PYB_GND, ("drag",): Physics.PYB_DRAG, ("dw",): Physics.PYB_DW,
            ("gnd", "drag", "dw"): Physics.PYB_GND_DRAG_DW}.get(tuple(aero))


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("aero", [(), ("gnd",), ("drag",)])
def test_integrate_pyb_parity(prec, aero):
    rng = np.random.default_rng(31)
    n, T = 48, 1200
    raw0 = _random_raw(rng, n, z=0.06 if aero else 1.0, tilt=0.3, spin=3.0)
    rpms = _rpms(rng, T, n, scale=0.5)
    ref = run_integrate(rpms, raw0, aero=aero, integrator="bullet")
    sim = _sim(n_envs=n, task="none", precision=prec, physics=_physics(aero))
    sim.set_raw_state(raw0)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    err = state_rel_err(traj, ref)
    print(f"\n[parity] bullet integrate {prec} {aero}: max rel err {err.max():.3e} median {np.median(err):.3e}")
    assert np.isfinite(traj).all()
    assert err.max() <= TOL[prec]
    assert np.median(err) <= TOL_MEDIAN[prec]
    sim.close()


def test_integrate_pyb_fast_spin_clamps():
    """Large rates: the coordinate-velocity clamp (+-100) engages on the first substep, and at
    pyb_freq 120 the exponential map's angular-motion threshold (|w| dt > pi/4) engages too
    (|w| <= 100 sqrt(3) keeps it below the threshold at 240 Hz)."""
    rng = np.random.default_rng(32)
    n, T = 16, 240
    raw0 = _random_raw(rng, n, spin=0.0)
    raw0[:, 10:13] = rng.uniform(-1, 1, (n, 3)) * 180.0
    raw0[:, 7:10] = rng.uniform(-1, 1, (n, 3)) * 140.0
    rpms = _rpms(rng, T, n)
    ref = run_integrate(rpms, raw0, integrator="bullet", pyb_freq=120, ctrl_freq=30)
    assert (np.abs(ref[0, :, 13:16]) == 100.0).any() and (np.abs(ref[0, :, 10:13]) == 100.0).any()
    assert (np.linalg.norm(ref[:, :, 13:16], axis=-1) / 120 > math.pi / 4).any()
    sim = _sim(n_envs=n, task="none", precision="f64", physics=_physics(()), pyb_freq=120, ctrl_freq=30)
    sim.set_raw_state(raw0)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    assert np.abs(traj[..., 13:16]).max() <= 100.0
    assert state_rel_err(traj, ref).max() <= TOL["f64"]
    sim.close()


def test_gpu_kat_damped_free_fall():
    """rpm = 0: vz' = vz + dt (-G - 0.04 (1 + |vz|) vz), exactly as the restated damping says."""
    n, T = 4, 1200
    sim = _sim(n_envs=n, task="none", precision="f64", physics=_physics(()))
    traj = sim.integrate(np.zeros((T, n, 4)), record=True).cpu().numpy()
    vz, dt = 0.0, 1.0 / 240
    ref = []
    for _ in range(T):
        vz = vz + dt * (-9.8 - 0.04 * (1 + abs(vz)) * vz)
        ref.append(vz)
    np.testing.assert_allclose(traj[:, 0, 12], ref, rtol=1e-12)
    assert np.array_equal(traj[:, :, 3:7], np.tile([0, 0, 0, 1.0], (T, n, 1)))
    sim.close()


def test_downwash_pyb_parity():
    rng = np.random.default_rng(33)
    E, D, T = 4, 8, 600
    xyz = _staggered(D)
    rpms = _rpms(rng, T, E * D, scale=0.3)
    ref = np.concatenate([RefAviary(num_drones=D, task="none", aero=("dw",), initial_xyzs=xyz, integrator="bullet")
                          .integrate(rpms[:, e * D:(e + 1) * D]) for e in range(E)], axis=1)
    sim = _sim(n_envs=E, drones_per_env=D, task="none", precision="f64", physics=_physics(("dw",)),
               initial_xyzs=xyz)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    err = state_rel_err(traj, ref)
    print(f"\n[parity] bullet downwash: max rel err {err.max():.3e}")
    assert err.max() <= TOL["f64"]
    sim.close()


@pytest.mark.parametrize("act", ["rpm", "one_d_rpm"])
def test_step_parity_hover_pyb(act):
    """HoverAviary with its default Physics.PYB: obs / reward / done with SB3 auto-reset."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(34)
    E, T = 16, 80
    A = 4 if act == "rpm" else 1
    acts = np.clip(rng.normal(0, 0.1, (T, E, 1, A)), -1, 1).astype(np.float32)
    acts[:, :4] = rng.uniform(-1, 1, (T, 4, 1, A)).astype(np.float32)
    if A == 1:
        acts[:, 4:6] = 1.0
    envs = []
    obs_r, rew_r, te_r, tr_r, tobs_r = run_vec(acts, E, act=act, integrator="bullet", envs=envs)
    sim = _sim(n_envs=E, task="hover", precision="f64", act=ActionType(act), physics=_physics(()))
    n_done = 0
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        te, tr = te.cpu().numpy().astype(bool), tr.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(te, te_r[t])
        np.testing.assert_array_equal(tr, tr_r[t])
        assert_obs_match(o.cpu().numpy(), obs_r[t], 1e-5, 1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), rew_r[t], rtol=1e-6, atol=1e-6)
        tobs = sim.terminal_obs.cpu().numpy()
        for e in np.nonzero(te | tr)[0]:
            n_done += 1
            assert_obs_match(tobs[e], tobs_r[(t, e)], 1e-5, 1e-6)
    assert n_done > 0
    err = state_rel_err(sim.state20().cpu().numpy(), np.concatenate([e.state20() for e in envs]))
    assert err.max() <= TOL["f64"], err.max()
    sim.close()


def test_step_parity_multihover_pyb_all_terms():
    """MultiHoverAviary, Physics.PYB_GND_DRAG_DW, staggered 8-drone start (downwash active)."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(35)
    E, D, T = 4, 8, 40
    xyz = [[0.15 * math.cos(2 * math.pi * i / 8), 0.15 * math.sin(2 * math.pi * i / 8), 0.5 + 0.1 * i]
           for i in range(8)]
    acts = np.clip(rng.normal(0, 0.2, (T, E, D, 4)), -1, 1).astype(np.float32)
    aero = ("gnd", "drag", "dw")
    envs = []
    obs_r, rew_r, te_r, tr_r, _ = run_vec(acts, E, drones_per_env=D, task="multihover", aero=aero,
                                          initial_xyzs=xyz, integrator="bullet", envs=envs)
    sim = _sim(n_envs=E, drones_per_env=D, task="multihover", precision="f64", act=ActionType.RPM,
               physics=_physics(aero), initial_xyzs=xyz)
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        np.testing.assert_array_equal(te.cpu().numpy().astype(bool), te_r[t])
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), tr_r[t])
        assert_obs_match(o.cpu().numpy(), obs_r[t], 1e-5, 1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), rew_r[t], rtol=1e-6, atol=1e-5)
    err = state_rel_err(sim.state20().cpu().numpy(), np.concatenate([e.state20() for e in envs]))
    assert err.max() <= TOL["f64"], err.max()
    sim.close()


def test_pyb_and_dyn_differ():
    """The PYB path is not the DYN path in disguise: damping and the prop placement change the
    trajectory (same inputs, 1 s)."""
    rng = np.random.default_rng(36)
    n, T = 8, 240
    raw0 = _random_raw(rng, n)
    rpms = _rpms(rng, T, n, scale=0.5)
    out = {}
    for name, phys in (("dyn", None), ("pyb", _physics(()))):
        kw = {} if phys is None else {"physics": phys}
        sim = _sim(n_envs=n, task="none", precision="f64", **kw)
        sim.set_raw_state(raw0)
        out[name] = sim.integrate(rpms, record=True).cpu().numpy()
        sim.close()
    assert np.abs(out["dyn"][-1, :, :3] - out["pyb"][-1, :, :3]).max() > 1e-3
    assert HOVER > 0
