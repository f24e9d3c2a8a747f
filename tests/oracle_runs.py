"""Helpers that drive the CPU oracle (oracle/) the way the GPU path is driven.

Test infrastructure only.  ``run_vec`` reproduces SB3 DummyVecEnv auto-reset semantics on a
list of reference-shaped envs: when an env finishes, its last obs becomes the terminal
observation and the returned obs is the reset observation.
"""
import numpy as np

from oracle.ref_aviary import RefAviary


# f64 gate for Physics.PYB* runs whose drones touch the ground plane.  Contact events are
# discontinuous in the state (a speculative row enters the solve at the breaking threshold with
# a nonzero impulse; the solver stops on a residual threshold), so a rounding-level difference
# can be amplified: the oracle itself turns a 1e-15 perturbation of integrate_pyb_gnd_drag's
# start state into 1.1e-9 on one drone within 2.5 s (tests/test_golden.py
# test_oracle_contact_self_sensitivity_within_gate).  Max over drones and samples <= 1e-7; the
# median stays at the 1e-10 gate of the contact-free paths.
TOL_CONTACT = 1e-7


def state_rel_err(a, b):
    """Per-drone relative L2 error of the state (SURVEY §8(d) gate): pos, quat, rpy, vel, ang_v -
    columns 0..15 of the 20-float state vector.  q and -q are the same orientation, so the
    quaternion difference is taken with the sign of b that is closer to a (canonicalising both to
    w >= 0 would flip one of two nearly equal quaternions whose w straddles 0 near 180 deg).
    The last_clipped_action columns (16..19) are inputs, not integrated state, and are left out
    so that their ~1.4e4 magnitude cannot hide errors."""
    a = np.array(a, dtype=np.float64)[..., :16]
    b = np.array(b, dtype=np.float64)[..., :16]
    d = a - b
    dq_flip = a[..., 3:7] + b[..., 3:7]
    flip = (dq_flip ** 2).sum(-1, keepdims=True) < (d[..., 3:7] ** 2).sum(-1, keepdims=True)
    d[..., 3:7] = np.where(flip, dq_flip, d[..., 3:7])
    num = np.linalg.norm(d, axis=-1)
    den = np.maximum(np.linalg.norm(b, axis=-1), 1e-6)
    return num / den


def run_integrate(rpms, raw0=None, **kw):
    """Oracle trajectory for rpm [T, N, 4]; one RefAviary holding all N drones (no downwash
    unless requested, so drones are independent)."""
    T, N, _ = rpms.shape
    env = RefAviary(num_drones=N, task="none", **kw)
    if raw0 is not None:
        env.set_raw_state(raw0)
    return env.integrate(rpms)


def run_vec(actions, n_envs, drones_per_env=1, act="rpm", task="hover", envs=None, **kw):
    """actions [T, E, D, A] float32 -> obs [T, E, D, W], reward [T, E], term/trunc [T, E],
    terminal obs dict {(t, e): [D, W]}.  Pass a list as ``envs`` to get the RefAviary objects
    back (or to continue from existing ones)."""
    if envs is None:
        envs = []
    if not envs:
        envs.extend(RefAviary(num_drones=drones_per_env, act=act, task=task, **kw) for _ in range(n_envs))
    T = actions.shape[0]
    obs_l, rew, te, tr, term_obs = [], np.zeros((T, n_envs)), np.zeros((T, n_envs), bool), np.zeros((T, n_envs), bool), {}
    for t in range(T):
        row = []
        for e, env in enumerate(envs):
            o, r, a_t, b_t, _ = env.step(actions[t, e])
            rew[t, e], te[t, e], tr[t, e] = r, a_t, b_t
            if a_t or b_t:
                term_obs[(t, e)] = o
                o, _ = env.reset()
            row.append(o)
        obs_l.append(np.stack(row))
    return np.stack(obs_l), rew, te, tr, term_obs


def assert_obs_match(gpu, ref, rtol=1e-5, atol=1e-6, err_msg=""):
    """KIN observation rows [..., 12 + 15A]: the 12 kinematic columns within tolerance, the 15A
    action-history columns (float32 copies of past actions placed by ring index,
    BaseRLAviary.py:307-319) bit-exact."""
    gpu, ref = np.asarray(gpu), np.asarray(ref)
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    np.testing.assert_array_equal(gpu[..., 12:], ref[..., 12:], err_msg=f"action history {err_msg}")
    np.testing.assert_allclose(gpu[..., :12], ref[..., :12], rtol=rtol, atol=atol, err_msg=err_msg)


def oracle_raw(env):
    """The oracle's physics-client state as a raw [N, 20] array (gpd_get_raw_state layout):
    pos, stored quat, vel, integrated rate (world rate on the Bullet path), ang_v, last action."""
    n = env.NUM_DRONES
    raw = np.zeros((n, 20))
    raw[:, 0:3] = env._b_pos
    raw[:, 3:7] = env._b_quat
    raw[:, 7:10] = env._b_vel
    raw[:, 10:13] = env._b_angv if env.INTEGRATOR == "bullet" else env.rpy_rates
    raw[:, 13:16] = env._b_angv
    raw[:, 16:20] = env.last_clipped_action
    return raw


def resynced_substep_errors(sim, env, rpms):
    """Local parity of chaotic runs (drones crashing into the plane): before every substep the
    GPU sim is set to the oracle's state, both take ONE substep on the same RPMs, and the
    per-drone relative state error of that substep is recorded.  Rounding differences cannot
    compound, so an identical algorithm agrees to rounding at every substep.  An f32 sim holds
    the state rounded to f32, so the oracle is then set to those same values: both step from the
    same input (a contact decided at a tie - a symmetric squeezed stack - can jump under a 1e-8
    change of the input; the f64 oracle itself moves 0.1 when its input is rounded to f32).
    Returns [T, N]."""
    errs = []
    same_input = getattr(sim, "precision", "f64") == "f32"
    for t in range(rpms.shape[0]):
        sim.set_raw_state(oracle_raw(env))
        if same_input:
            env.set_raw_state(sim.raw_state().cpu().numpy())
        g = sim.integrate(rpms[t:t + 1], record=True).cpu().numpy()
        r = env.integrate(rpms[t:t + 1])
        errs.append(state_rel_err(g, r)[0])
    return np.array(errs)
