"""Analytic known-answer tests that pin the CPU oracle.

The reference holds no golden vectors for the DYN path and cannot be run here, so these
closed-form checks (plus scipy's independent rotation code) are what pins the oracle.
"""
import math

import numpy as np
import pytest

from oracle.bullet_math import euler_from_quat, quat_from_euler, quat_roundtrip, quat_to_mat
from oracle.params import derived
from oracle.ref_aviary import RefAviary, rpm_from_action

P = derived("cf2x")
HOVER = P["hover_rpm"]
DT = 1.0 / 240


def _state(env, i=0):
    return env.state20()[i]


def test_derived_constants():
    """BaseAviary.py:117-128 for cf2x."""
    assert HOVER == pytest.approx(14468.429183500699, rel=1e-15)
    assert P["max_rpm"] == pytest.approx(21702.64377525105, rel=1e-15)
    assert P["gnd_eff_h_clip"] == pytest.approx(0.03776371349209501, rel=1e-12)
    assert P["gravity"] == pytest.approx(0.2646, rel=1e-15)


def test_kat1_hover_equilibrium():
    env = RefAviary(task="none")
    traj = env.integrate(np.full((1200, 1, 4), HOVER))
    assert np.abs(traj[:, 0, :16] - traj[0, 0, :16]).max() <= 1e-12
    assert traj[-1, 0, 2] == pytest.approx(0.1125, abs=1e-12)


def test_kat2_free_fall_semi_implicit_euler():
    env = RefAviary(task="none")
    n = np.arange(1, 241)
    traj = env.integrate(np.zeros((240, 1, 4)))
    g = P["gravity"] / P["m"]
    np.testing.assert_allclose(traj[:, 0, 12], -g * n * DT, rtol=1e-12)
    np.testing.assert_allclose(traj[:, 0, 2], 0.1125 - g * DT * DT * n * (n + 1) / 2, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(traj[:, 0, 3:7], np.tile([0, 0, 0, 1.0], (240, 1)))


def test_kat3_pure_yaw():
    a, b = HOVER * 0.99, HOVER * 1.01
    env = RefAviary(task="none")
    T = 240
    traj = env.integrate(np.tile([a, b, a, b], (T, 1, 1)))
    c = 2 * P["km"] * (b * b - a * a) / P["izz"]
    n = np.arange(1, T + 1)
    psi = DT * DT * c * n * (n + 1) / 2
    np.testing.assert_allclose(traj[:, 0, 9], np.arctan2(np.sin(psi), np.cos(psi)), rtol=0, atol=1e-9)
    q = traj[:, 0, 3:7] * np.sign(traj[:, 0, 6:7])
    np.testing.assert_allclose(q[:, 2], np.sin(psi / 2) * np.sign(np.cos(psi / 2)), atol=1e-9)
    np.testing.assert_allclose(traj[:, 0, 7:9], 0, atol=1e-12)       # no roll / pitch


def test_kat4_roll_sign_quirk():
    """BaseAviary.py:847: props 0,1 faster -> positive roll (opposite to the URDF geometry)."""
    d = 0.01 * HOVER
    env = RefAviary(task="none")
    traj = env.integrate(np.tile([HOVER + d, HOVER + d, HOVER - d, HOVER - d], (24, 1, 1)))
    assert traj[-1, 0, 7] > 0
    geom = RefAviary(task="none", wrench="geom")
    traj_g = geom.integrate(np.tile([HOVER + d, HOVER + d, HOVER - d, HOVER - d], (24, 1, 1)))
    assert traj_g[-1, 0, 7] < 0


def test_kat5_zero_rate_keeps_quaternion():
    env = RefAviary(task="none")
    q = np.array([0.0, 0.0, 0.3, 0.9539392014169456])
    assert env._integrateQ(q, np.array([0.0, 0.0, 5e-9]), DT) is q
    assert not np.array_equal(env._integrateQ(q, np.array([0.0, 0.0, 2e-8]), DT), q)


def test_kat6_euler_vs_scipy():
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(0)
    qs = Rotation.random(10000, random_state=1).as_quat()  # [x, y, z, w]
    ref = Rotation.from_quat(qs).as_euler("xyz")
    keep = np.abs(ref[:, 1]) < 1.5
    ours = np.array([euler_from_quat(q) for q in qs[keep]])
    np.testing.assert_allclose(ours, ref[keep], rtol=0, atol=1e-9)
    # matrix helper agrees with scipy, for non-unit quaternions too (s = 2/|q|^2)
    for q in qs[:200] * rng.uniform(0.5, 2.0, (200, 1)):
        np.testing.assert_allclose(quat_to_mat(q), Rotation.from_quat(q).as_matrix(), atol=1e-12)


def test_bullet_roundtrip_properties():
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(2)
    for q in Rotation.random(2000, random_state=3).as_quat() * rng.uniform(0.3, 3.0, (2000, 1)):
        r = quat_roundtrip(q)
        assert abs(np.linalg.norm(r) - 1) < 1e-12                    # re-normalised
        assert min(np.abs(r - q / np.linalg.norm(q)).max(), np.abs(r + q / np.linalg.norm(q)).max()) < 1e-12
        if np.trace(quat_to_mat(q)) > 0:
            assert r[3] > 0                                           # w > 0 branch
    for rpy in rng.uniform([-3, -1.5, -3], [3, 1.5, 3], (500, 3)):
        np.testing.assert_allclose(euler_from_quat(quat_from_euler(rpy)), rpy, atol=1e-9)


def test_gimbal_branches():
    # pitch = +-pi/2 exactly: the two getEulerZYX branches
    q = quat_from_euler([0.3, math.pi / 2, 0.2])
    e = euler_from_quat(q)
    assert e[0] == 0.0 and e[1] == pytest.approx(math.pi / 2)
    q = quat_from_euler([0.3, -math.pi / 2, 0.2])
    e = euler_from_quat(q)
    assert e[0] == 0.0 and e[1] == pytest.approx(-math.pi / 2)


def test_kat7_ground_effect_magnitude():
    env = RefAviary(task="none", aero=("gnd",))
    R = np.eye(3)
    rpm = np.full(4, HOVER)
    fz, tx, ty = env._ground_effect_wrench(rpm, 0, R)
    per_prop = fz / 4
    assert per_prop == pytest.approx(0.0300478 * P["kf"] * HOVER ** 2, rel=1e-5)
    assert abs(tx) < 1e-18 and abs(ty) < 1e-18                         # symmetric props
    # clip: at (and below) GND_EFF_H_CLIP the force stops growing
    env._b_pos[0, 2] = 0.01
    env._updateAndStoreKinematicInformation()
    low, _, _ = env._ground_effect_wrench(rpm, 0, R)
    env._b_pos[0, 2] = P["gnd_eff_h_clip"]
    env._updateAndStoreKinematicInformation()
    at_clip, _, _ = env._ground_effect_wrench(rpm, 0, R)
    assert low == pytest.approx(at_clip, rel=1e-12)


def test_kat8_downwash_magnitude_and_culling():
    xyz = np.array([[0, 0, 0.5], [0, 0, 1.0]])
    env = RefAviary(num_drones=2, task="none", aero=("dw",), initial_xyzs=xyz)
    assert env._downwash_force(0) == pytest.approx(-0.3033594, rel=1e-6)
    assert env._downwash_force(1) == 0.0                               # nobody above drone 1
    far = RefAviary(num_drones=2, task="none", aero=("dw",), initial_xyzs=[[0, 0, 0.5], [10, 0, 1.0]])
    assert far._downwash_force(0) == 0.0                               # delta_xy >= 10


def test_kat9_truncation_reward_obs_and_history():
    env = RefAviary(act="rpm", task="hover")
    obs, info = env.reset()
    assert obs.shape == (1, 72) and obs.dtype == np.float32 and info == {"answer": 42}
    trunc_at = None
    for k in range(1, 260):
        a = np.full((1, 4), (k % 7) * 0.01, np.float32)
        obs, r, te, tr, _ = env.step(a)
        assert 0 <= r <= 2
        if tr:
            trunc_at = k
            break
    assert trunc_at == 242
    obs, _ = env.reset()
    np.testing.assert_allclose(obs[0, -4:], (242 % 7) * 0.01, rtol=1e-6)   # history survives reset
    one_d = RefAviary(act="one_d_rpm", task="hover")
    assert one_d.reset()[0].shape == (1, 27)
    multi = RefAviary(num_drones=2, act="rpm", task="multihover")
    assert multi.reset()[0].shape == (2, 72)
    np.testing.assert_allclose(multi.TARGET_POS[:, 2], 0.1125 + np.array([1.0, 0.5]))


def test_action_mapping_is_float32():
    """numpy ^1.24 value-based casting: the RPM of a float32 action is computed in float32."""
    a = np.float32(0.5014336)
    got = rpm_from_action(HOVER, np.array([a]))[0]
    expect = np.float32(HOVER) * (np.float32(1) + np.float32(0.05) * a)
    assert got == float(expect)
    fused = np.float32(np.float32(HOVER) * np.float32(np.float64(np.float32(0.05)) * np.float64(a) + 1.0))
    assert got != float(fused)  # the FMA-contracted value the GPU must NOT produce
