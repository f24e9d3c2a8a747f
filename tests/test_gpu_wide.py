"""Envs of more than 64 drones (MultiHoverAviary(num_drones=D) with D in 65..1024): the
multi-wave-workgroup kernels step_kernel_wide / integrate_kernel_wide (csrc/gpd_kernels.h),
through the C ABI, against the C fp64 restatement (oracle/gpd_oracle.c, downwash O(D^2) as
BaseAviary._downwash :785-811) and, for the PID and Physics.PYB paths, the numpy oracle.

Gates as in tests/test_gpu_fullsize.py: f64 state per-drone relative L2 <= 1e-10 after every
step, terminated / truncated exact, action-history obs columns bit-exact, the rest to float32
rounding.  The reference has no bound on num_drones; this implementation's bound is one
workgroup (1024 lanes) per env.
"""
import math

import numpy as np
import pytest
import torch

from oracle.c_oracle import COracle
from oracle.ref_aviary import RefAviary
from tests.oracle_runs import (assert_obs_match, oracle_raw, resynced_substep_errors, state_rel_err)

pytestmark = pytest.mark.gpu


def _spiral(D, z0=0.3, z1=1.9, r=1.5):
    """Golden-angle spiral of D drones at strictly increasing heights.  The downwash force
    (BaseAviary.py:801-809) grows as 1/dz^2 for drones at nearly equal heights and is damped only
    by exp(-dxy^2 / (2 beta^2)): drones close in height here are far apart horizontally
    (consecutive ones ~2.8 m), so every pair force stays bounded."""
    i = np.arange(D)
    ang = i * np.pi * (3 - np.sqrt(5))
    return np.stack([r * np.cos(ang), r * np.sin(ang), z0 + (z1 - z0) * i / max(D - 1, 1)], 1)


def _sim(**kw):
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    return BatchedAviarySim(device="cuda:0", **kw)


# D = 300 (5 waves) runs without downwash: with 300 drones below 2 m some pair forces reach twice
# the weight, and the oracle itself then turns a 1e-15 start perturbation into 5e-9 by step 40.
@pytest.mark.parametrize("D,act,aero", [(65, "rpm", ("dw",)), (96, "one_d_rpm", ("dw",)),
                                        (200, "rpm", ("dw", "gnd", "drag")), (300, "rpm", ("gnd", "drag"))])
def test_wide_multihover_step_parity(D, act, aero):
    from gym_pybullet_drones_routing_amd.enums import ActionType
    E, T = 3, 40
    A = 4 if act == "rpm" else 1
    rng = np.random.default_rng(D)
    xyz = _spiral(D)
    acts = np.clip(rng.normal(0, 0.2, (T, E, D, A)), -1, 1).astype(np.float32)
    acts[:, 0] = rng.uniform(-1, 1, (T, D, A)).astype(np.float32)     # env 0 ends episodes
    sim = _sim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType(act), aero=aero, initial_xyzs=xyz)
    assert sim.constants.drones_per_block == D
    orc = COracle(n_envs=E, drones_per_env=D, task="multihover", act=act, aero=aero, initial_xyzs=xyz)
    worst, n_done = 0.0, 0
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        o_o, r_o, te_o, tr_o = orc.step(acts[t])
        te, tr = te.cpu().numpy().astype(bool), tr.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(te, te_o, err_msg=f"terminated differs at step {t}")
        np.testing.assert_array_equal(tr, tr_o, err_msg=f"truncated differs at step {t}")
        assert_obs_match(o.cpu().numpy(), o_o, 1e-5, 1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), r_o, rtol=1e-6, atol=1e-5)
        done = te | tr
        if done.any():
            n_done += int(done.sum())
            assert_obs_match(sim.terminal_obs.cpu().numpy()[done], orc.terminal_obs[done], 1e-5, 1e-6)
        err = state_rel_err(sim.state20().cpu().numpy(), orc.state20())
        worst = max(worst, float(err.max()))
        assert worst <= 1e-10, f"state rel L2 {worst:.3g} at step {t}"
    print(f"\n[wide] D={D} {act} {aero}: {n_done} episode ends, max state rel L2 {worst:.3g}")
    sim.close()
    orc.close()


def test_wide_integrate_parity_1024():
    """The largest env (1024 drones, 16 waves), downwash + ground effect + drag, 60 substeps."""
    D, T = 1024, 60
    rng = np.random.default_rng(7)
    xyz = _spiral(D, 0.5, 10.7)
    rpm = 14468.429183500699 * (1 + 0.05 * rng.uniform(-1, 1, (T, D, 4)))
    aero = ("dw", "gnd", "drag")
    sim = _sim(n_envs=1, drones_per_env=D, task="none", aero=aero, initial_xyzs=xyz)
    traj = sim.integrate(rpm, record=True).cpu().numpy()
    orc = COracle(n_envs=1, drones_per_env=D, task="none", aero=aero, initial_xyzs=xyz)
    ref = orc.integrate(rpm)
    err = state_rel_err(traj, ref)
    print(f"\n[wide] integrate D=1024: max rel err {err.max():.3e}")
    assert err.max() <= 1e-10
    sim.close()
    orc.close()


def test_wide_one_d_pid_matches_numpy_oracle():
    """DSLPIDControl in an env of 70 drones (no downwash: the numpy oracle is per-drone)."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    D, T = 70, 12
    rng = np.random.default_rng(3)
    xyz = _spiral(D)
    acts = rng.uniform(-1, 1, (T, 1, D, 1)).astype(np.float32)
    sim = _sim(n_envs=1, drones_per_env=D, task="multihover", act=ActionType.ONE_D_PID, initial_xyzs=xyz)
    env = RefAviary(num_drones=D, act="one_d_pid", task="multihover", initial_xyzs=xyz)
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        ob, rw, tm, tc, _ = env.step(acts[t, 0])
        assert bool(te.item()) == bool(tm) and bool(tr.item()) == bool(tc)
        assert_obs_match(o.cpu().numpy()[0], ob, 1e-5, 1e-6)
        if tm or tc:
            break
    assert state_rel_err(sim.state20().cpu().numpy(), env.state20()).max() <= 1e-10
    sim.close()


def test_wide_pyb_requires_opt_out_of_drone_contact():
    """Envs of more than 64 drones run the multi-wave kernels, which do not restate the drone <->
    drone contact: under Physics.PYB* that is an error, not a silently dropped physics term."""
    from gym_pybullet_drones_routing_amd.enums import Physics
    with pytest.raises(NotImplementedError, match="no_drone_contact"):
        _sim(n_envs=1, drones_per_env=65, task="multihover", physics=Physics.PYB)


def test_wide_pyb_contact_resynced():
    """Physics.PYB in an env of 80 drones crashing into the plane: the waves take turns in the
    contact solve's LDS rows; resynced per-substep parity as in test_gpu_bullet.py."""
    from tests.test_gpu_bullet import _crash_case
    from tests.test_gpu_parity import _rpms
    from gym_pybullet_drones_routing_amd.enums import Physics
    D, T = 80, 60
    rng = np.random.default_rng(45)
    raw0 = _crash_case(rng, D)
    rpms = _rpms(rng, T, D, scale=0.5) * 0.6
    env = RefAviary(num_drones=D, task="none", integrator="bullet")
    env.set_raw_state(raw0)
    # the oracle env steps its 80 drones independently (drones_per_env 1): no drone <-> drone
    # contact on either side (the multi-wave kernels do not restate it)
    sim = _sim(n_envs=1, drones_per_env=D, task="none", physics=Physics.PYB, aero=("no_drone_contact",))
    err = resynced_substep_errors(sim, env, rpms)
    print(f"\n[wide] PYB contact resynced D=80: max {err.max():.3e}")
    assert (oracle_raw(env)[:, 2] < 0.02).sum() > D // 4
    assert err.max() <= 1e-12
    sim.close()


def test_wide_bound():
    from gym_pybullet_drones_routing_amd import _lib
    with pytest.raises(_lib.GpdError):
        _sim(n_envs=1, drones_per_env=1025, task="multihover")
    assert math.isfinite(1.0)
