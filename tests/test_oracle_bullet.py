"""Analytic checks that pin the Bullet multibody restatement (oracle/bullet_mb.py).

pybullet cannot run in this pipeline, so the restated btMultiBody base step is pinned by closed
forms: hover equilibrium, damped free fall (recurrence and terminal velocity), the coordinate
velocity clamp, a damped spin about a principal axis, the exponential map against scipy, the
prop-placement roll sign, and the world-frame form the GPU kernel evaluates.  The ground-plane
contact restatement (``plane_contact``) is pinned by rest / no-force / sliding-friction / tilted
landing checks.
"""
import math

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from oracle.bullet_math import quat_to_mat
from oracle.bullet_mb import (ANG_DAMP, FRICTION, LIN_DAMP, LINEAR_SLOP, MAX_COORD_VEL, base_quat_update,
                              breaking_threshold, multibody_step, plane_contact, qconj)
from oracle.params import derived
from oracle.ref_aviary import RefAviary

P = derived("cf2x")
HOVER = P["hover_rpm"]
DT = 1.0 / 240
M = P["m"]
INERTIA = np.array([P["ixx"], P["iyy"], P["izz"]])


def _env(**kw):
    return RefAviary(task="none", integrator="bullet", **kw)


def test_hover_equilibrium():
    traj = _env().integrate(np.full((1200, 1, 4), HOVER))
    assert np.abs(traj[:, 0, :16] - traj[0, 0, :16]).max() <= 1e-12
    assert traj[-1, 0, 2] == pytest.approx(0.1125, abs=1e-12)


def test_damped_free_fall_recurrence_and_terminal_velocity():
    """rpm = 0: vz' = vz + dt (-G - k (1 + |vz|) vz), z' = z + dt vz' (damping K1 = K2 = 0.04)."""
    T = 2400
    traj = _env(initial_xyzs=[[0.0, 0.0, 500.0]]).integrate(np.zeros((T, 1, 4)))
    vz, z = 0.0, 500.0
    ref_v, ref_z = [], []
    for _ in range(T):
        vz = vz + DT * (-P["G"] - LIN_DAMP * (1 + abs(vz)) * vz)
        z = z + DT * vz
        ref_v.append(vz)
        ref_z.append(z)
    np.testing.assert_allclose(traj[:, 0, 12], ref_v, rtol=1e-12)
    np.testing.assert_allclose(traj[:, 0, 2], ref_z, rtol=1e-12)
    vt = (-1 + math.sqrt(1 + 4 * P["G"] / LIN_DAMP)) / 2        # k (1 + v) v = G
    assert traj[-1, 0, 12] == pytest.approx(-vt, rel=1e-3)
    np.testing.assert_array_equal(traj[:, 0, 3:7], np.tile([0, 0, 0, 1.0], (T, 1)))


def test_velocity_coordinates_clamped():
    out = multibody_step(np.zeros(3), np.array([0, 0, 0, 1.0]), np.array([0, 0, -150.0]), np.array([130.0, 0, 0]),
                         np.zeros(3), np.zeros(3), np.array([0, 0, -P["gravity"]]), M, INERTIA, DT)
    assert out[2][2] == -MAX_COORD_VEL
    assert out[3][0] == MAX_COORD_VEL


def test_damped_spin_about_a_principal_axis():
    """No torque, w = (0,0,w0): w' = w - dt k (1 + |w|) w; yaw accumulates sum(w' dt)."""
    env = _env()
    raw = env.state20()[0].copy()
    raw0 = np.zeros(20)
    raw0[0:3] = raw[0:3]
    raw0[3:7] = [0, 0, 0, 1.0]
    raw0[10:13] = [0, 0, 20.0]
    env.set_raw_state(raw0[None])
    T = 480
    rpm = np.full((T, 1, 4), HOVER)              # thrust balances gravity, sum of z torques is 0
    traj = env.integrate(rpm)
    w, psi = 20.0, 0.0
    ws, psis = [], []
    for _ in range(T):
        w = w - DT * ANG_DAMP * (1 + w) * w
        psi += w * DT
        ws.append(w)
        psis.append(psi)
    np.testing.assert_allclose(traj[:, 0, 15], ws, rtol=1e-12)
    q = traj[:, 0, 3:7] * np.sign(traj[:, 0, 6:7])
    psis = np.array(psis)
    np.testing.assert_allclose(q[:, 2], np.sin(psis / 2) * np.sign(np.cos(psis / 2)), atol=1e-10)
    np.testing.assert_allclose(traj[:, 0, 13:15], 0, atol=1e-12)


def test_exponential_map_against_scipy():
    rng = np.random.default_rng(3)
    for _ in range(200):
        q_s = Rotation.random(random_state=rng).as_quat()
        w = rng.normal(size=3) * rng.choice([1e-4, 1.0, 50.0])
        q_wb = qconj(q_s)
        new_s = qconj(base_quat_update(q_wb, w, DT))
        ref = (Rotation.from_rotvec(w * DT) * Rotation.from_quat(q_s)).as_quat()
        assert min(np.abs(new_s - ref).max(), np.abs(new_s + ref).max()) < 1e-13


def test_angular_motion_threshold():
    """|w| dt > pi/4: the angle used in sin/cos is clamped to pi/4 (btTransformUtil)."""
    w = np.array([0.0, 0.0, 300.0])
    q = base_quat_update(np.array([0, 0, 0, 1.0]), w, DT)
    f = 0.5 * (0.5 * math.pi) / DT
    ax = 300.0 * math.sin(0.5 * f * DT) / f
    ref = np.array([0, 0, -ax, math.cos(0.5 * f * DT)])
    np.testing.assert_allclose(q, ref / np.linalg.norm(ref), rtol=1e-15, atol=1e-16)


def test_prop_placement_roll_sign():
    """Bullet places the thrust at the URDF props: faster props 0,1 (y = -0.028) roll NEGATIVE,
    the opposite of the DYN formula's quirk (BaseAviary.py:847)."""
    d = 0.02 * HOVER
    traj = _env().integrate(np.tile([HOVER + d, HOVER + d, HOVER - d, HOVER - d], (24, 1, 1)))
    assert traj[-1, 0, 7] < -1e-4
    dyn = RefAviary(task="none").integrate(np.tile([HOVER + d, HOVER + d, HOVER - d, HOVER - d], (24, 1, 1)))
    assert dyn[-1, 0, 7] > 1e-4


def _world_form(pos, q_s, v, w, fz, tau, drag_w):
    """The world-frame form the GPU kernel evaluates (gpd_device.h bullet_substep)."""
    R = quat_to_mat(q_s)
    wb = R.T @ w
    iw = INERTIA * wb
    k_w = ANG_DAMP + ANG_DAMP * np.linalg.norm(w)
    k_v = LIN_DAMP + LIN_DAMP * np.linalg.norm(v)
    wdot = R @ ((tau - np.cross(wb, iw)) / INERTIA) - k_w * w
    vdot = (R @ np.array([0, 0, fz]) + drag_w - np.array([0, 0, P["gravity"]])) / M - k_v * v
    w2 = np.clip(w + DT * wdot, -100, 100)
    v2 = np.clip(v + DT * vdot, -100, 100)
    return pos + DT * v2, v2, w2


def test_spatial_form_equals_world_form():
    """The restated articulated-body step (base frame, bias forces) and the world-frame form
    the kernel uses agree to rounding: the m w x v terms cancel and I^-1 I w = w."""
    rng = np.random.default_rng(7)
    for _ in range(100):
        q_s = Rotation.random(random_state=rng).as_quat()
        v, w = rng.normal(size=3) * 3, rng.normal(size=3) * 10
        fz, tau = 0.3 * rng.random(), rng.normal(size=3) * 1e-4
        drag_w = rng.normal(size=3) * 1e-3
        R = quat_to_mat(q_s)
        out = multibody_step(np.zeros(3), q_s, v, w, np.array([0, 0, fz]) + R.T @ drag_w, tau,
                             np.array([0, 0, -P["gravity"]]), M, INERTIA, DT)
        p2, v2, w2 = _world_form(np.zeros(3), q_s, v, w, fz, tau, drag_w)
        np.testing.assert_allclose(out[2], v2, rtol=0, atol=1e-13)
        np.testing.assert_allclose(out[3], w2, rtol=0, atol=1e-12)
        np.testing.assert_allclose(out[0], p2, rtol=0, atol=1e-15)


# ---------------------------------------------------------------------------- ground-plane contact
HH = P["collision_h"] / 2


def test_contact_zero_rpm_drop_comes_to_rest_on_the_plane():
    """KAT: zero RPM from the reference's start height (0.1125 m, BaseAviary.py:196) lands and
    rests with the cylinder's bottom on z = 0 (to the linear slop), level and at rest."""
    T = 480
    traj = _env().integrate(np.zeros((T, 1, 4)))
    z = traj[:, 0, 2]
    assert z.min() > HH - 2e-3                                 # no tunnelling through the plane
    assert z[-1] == pytest.approx(HH - LINEAR_SLOP, abs=1e-6)
    assert np.abs(traj[-1, 0, 10:16]).max() < 1e-5             # at rest (vel, ang_v; PGS leaves ~1e-6 yaw)
    assert np.abs(traj[-1, 0, 7:9]).max() < 1e-5               # level (roll, pitch)


def test_contact_no_force_above_the_plane():
    """Above the breaking threshold the contact adds nothing: hover / free fall / tumbling flight
    from 0.5 m are bit-identical with and without the plane for 0.25 s."""
    rng = np.random.default_rng(5)
    rpms = HOVER * (1 + 0.05 * rng.uniform(-1, 1, (60, 1, 4)))
    xyz = [[0.1, -0.2, 0.5]]
    a = _env(initial_xyzs=xyz).integrate(rpms)
    b = _env(initial_xyzs=xyz, aero=("no_plane",)).integrate(rpms)
    np.testing.assert_array_equal(a, b)
    assert a[:, 0, 2].min() > 0.3


def test_contact_breaking_threshold_value():
    r, h = P["collision_r"] + 0.001, HH + 0.001
    assert breaking_threshold(P["collision_r"], HH) == pytest.approx(0.02 * math.sqrt(2 * r * r + h * h), rel=1e-15)


def test_contact_sliding_friction_stops_the_drone():
    """A drone resting on the plane with a horizontal velocity slides under Coulomb friction:
    deceleration mu*G (plus the small multibody damping), stopping distance ~ v^2 / (2 mu G)."""
    v0 = 0.5
    env = _env(initial_xyzs=[[0.0, 0.0, HH - LINEAR_SLOP]])
    env._b_vel[0] = [v0, 0.0, 0.0]
    traj = env.integrate(np.zeros((120, 1, 4)))
    x_stop = traj[-1, 0, 0]
    d_ref = v0 * v0 / (2 * FRICTION * P["G"])
    assert abs(traj[-1, 0, 10]) < 1e-6
    assert x_stop == pytest.approx(d_ref, rel=0.1)
    assert abs(traj[-1, 0, 1]) < 1e-6                        # no sideways drift
    assert traj[:, 0, 2].min() > HH - 1e-3


def test_contact_tilted_landing_settles_flat():
    """Dropped from 0.1125 m with 0.3 rad roll, the cylinder lands on its rim and settles on its
    bottom cap (level, at rest, bottom on the plane)."""
    traj = _env(initial_rpys=[[0.3, 0.0, 0.0]]).integrate(np.zeros((720, 1, 4)))
    assert abs(traj[-1, 0, 7]) < 1e-4 and abs(traj[-1, 0, 8]) < 1e-4
    assert traj[-1, 0, 2] == pytest.approx(HH - LINEAR_SLOP, abs=1e-5)
    assert np.abs(traj[-1, 0, 10:16]).max() < 1e-4


def test_contact_velocity_level_constraints_hold():
    """After one contact solve on a penetrating resting drone, every active point's normal
    velocity matches its ERP target (residual threshold) and its normal impulse is >= 0."""
    rot = quat_to_mat(np.array([0.0, 0.0, 0.0, 1.0]))
    pos = np.array([0.0, 0.0, HH - 1e-3])                      # 1 mm into the plane
    v, w = plane_contact(pos, rot, np.array([0.0, 0.0, -0.3]), np.zeros(3), M, INERTIA, DT,
                         P["collision_r"], HH, 0.0)
    target = (1e-3 - LINEAR_SLOP) * 0.08 / DT                   # -penetration * erp / dt
    # every point's normal velocity at its target, to the solver's stopping residual
    # (sqrt(1e-7) ~ 3e-4 in velocity units)
    for rx, ry in ((0.06, 0), (0, 0.06), (-0.06, 0), (0, -0.06)):
        vn = v[2] + (w[0] * ry - w[1] * rx)
        assert vn == pytest.approx(target, abs=1e-3)
    assert np.abs(v[:2]).max() < 1e-4
