"""The C restatement (oracle/gpd_oracle.c) agrees with the numpy restatement (oracle/ref_aviary.py).

Both are test infrastructure; agreement between two independent codings of the same
reference lines is what lets the C one stand in for the numpy one at large sizes."""
import os

import numpy as np
import pytest

from oracle.c_oracle import COracle
from oracle.ref_aviary import RefAviary, rpm_from_action
from tests.oracle_runs import assert_obs_match, run_vec, state_rel_err

HOVER = 14468.429183500699


def _raw(rng, n, z=1.0):
    from oracle.bullet_math import quat_from_euler, quat_roundtrip
    raw = np.zeros((n, 20))
    raw[:, 0:2] = rng.uniform(-0.5, 0.5, (n, 2))
    raw[:, 2] = z
    for i in range(n):
        raw[i, 3:7] = quat_roundtrip(quat_from_euler(rng.uniform(-0.3, 0.3, 3)))
    raw[:, 7:10] = rng.uniform(-0.5, 0.5, (n, 3))
    raw[:, 10:13] = rng.uniform(-2, 2, (n, 3))
    raw[:, 16:20] = HOVER
    return raw


@pytest.mark.parametrize("aero,wrench,model", [((), "dyn", "cf2x"), (("gnd", "drag"), "dyn", "cf2x"),
                                               ((), "geom", "cf2x"), ((), "dyn", "cf2p"), ((), "dyn", "racer")])
def test_integrate_c_vs_numpy(aero, wrench, model):
    rng = np.random.default_rng(0)
    n, T = 8, 300
    raw0 = _raw(rng, n, z=0.08 if aero else 1.0)
    p_hover = {"cf2x": HOVER, "cf2p": HOVER, "racer": None}[model]
    if p_hover is None:
        from oracle.params import derived
        p_hover = derived("racer")["hover_rpm"]
    raw0[:, 16:20] = p_hover
    rpm = rpm_from_action(p_hover, rng.uniform(-1, 1, (T, n, 4)).astype(np.float32))
    ref = RefAviary(num_drones=n, task="none", aero=aero, wrench=wrench, model=model)
    ref.set_raw_state(raw0)
    tr_ref = ref.integrate(rpm)
    c = COracle(n_envs=n, task="none", aero=aero, wrench=wrench, model=model)
    c.set_raw_state(raw0)
    tr_c = c.integrate(rpm)
    assert state_rel_err(tr_c, tr_ref).max() <= 1e-11
    np.testing.assert_array_equal(tr_c[..., 16:], tr_ref[..., 16:])


def test_downwash_c_vs_numpy():
    rng = np.random.default_rng(1)
    D, T = 8, 240
    i = np.arange(D)
    xyz = np.stack([0.15 * np.cos(2 * np.pi * i / D), 0.15 * np.sin(2 * np.pi * i / D), 0.5 + 0.1 * i], 1)
    rpm = rpm_from_action(HOVER, (0.3 * rng.uniform(-1, 1, (T, D, 4))).astype(np.float32))
    ref = RefAviary(num_drones=D, task="none", aero=("dw",), initial_xyzs=xyz).integrate(rpm)
    c = COracle(n_envs=1, drones_per_env=D, task="none", aero=("dw",), initial_xyzs=xyz).integrate(rpm)
    assert state_rel_err(c, ref).max() <= 1e-11


@pytest.mark.parametrize("act,task,D", [("rpm", "hover", 1), ("one_d_rpm", "hover", 1), ("rpm", "multihover", 2)])
def test_step_c_vs_numpy(act, task, D):
    rng = np.random.default_rng(2)
    E, T = 6, 60
    A = 4 if act == "rpm" else 1
    acts = np.clip(rng.normal(0, 0.15, (T, E, D, A)), -1, 1).astype(np.float32)
    acts[:, 0] = rng.uniform(-1, 1, (T, D, A)).astype(np.float32)    # forces resets
    obs_r, rew_r, te_r, tr_r, tobs_r = run_vec(acts, E, drones_per_env=D, act=act, task=task)
    c = COracle(n_envs=E, drones_per_env=D, act=act, task=task)
    for t in range(T):
        o, r, te, tr = c.step(acts[t])
        np.testing.assert_array_equal(te, te_r[t])
        np.testing.assert_array_equal(tr, tr_r[t])
        assert_obs_match(o, obs_r[t], 1e-6, 1e-7)
        np.testing.assert_allclose(r, rew_r[t], rtol=1e-6, atol=1e-6)
        for e in np.nonzero(te | tr)[0]:
            assert_obs_match(c.terminal_obs[e], tobs_r[(t, e)], 1e-6, 1e-7)
    c.close()


def test_oracle_under_asan():
    """the C restatement under AddressSanitizer + UBSan (oracle/asan_driver.c drives
    every entry point on single- and 8-drone envs with every force flag); no report, exit 0."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"], capture_output=True, text=True,
                       timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "OK" in r.stdout and "Sanitizer" not in out and "runtime error" not in out, out[-3000:]
