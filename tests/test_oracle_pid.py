"""Known-answer and self-consistency tests of the DSLPIDControl restatement (oracle/ref_pid.py).

The reference holds no numeric tests for the controller either; these pin the
restatement analytically and check the one simplification the HIP path makes (the target
rotation is used directly instead of scipy's matrix -> 'XYZ' Euler -> matrix round trip).
"""
import math

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from oracle import ref_pid
from oracle.params import derived
from oracle.ref_aviary import RefAviary

HOVER = derived("cf2x")["hover_rpm"]


def test_hover_equilibrium_rpm():
    """At rest on target: target_thrust = (0,0,GRAVITY), R = I -> rpm == HOVER_RPM on all motors."""
    c = ref_pid.RefDSLPID()
    rpm, pos_e, yaw_e = c.computeControl(1 / 30, np.zeros(3), np.array([0, 0, 0, 1.0]), np.zeros(3), np.zeros(3),
                                         target_pos=np.zeros(3))
    np.testing.assert_allclose(rpm, HOVER, rtol=1e-12)
    assert np.all(pos_e == 0) and yaw_e == 0


def test_pwm_clip_and_thrust_floor():
    """Far below the target the integral and pwm clip; a target straight below -> scalar thrust
    floor max(0, .) -> MIN_PWM on every motor."""
    c = ref_pid.RefDSLPID()
    rpm, _, _ = c.computeControl(1 / 30, np.array([0, 0, 100.0]), np.array([0, 0, 0, 1.0]), np.zeros(3), np.zeros(3),
                                 target_pos=np.zeros(3))
    np.testing.assert_allclose(rpm, ref_pid.PWM2RPM_SCALE * ref_pid.MIN_PWM + ref_pid.PWM2RPM_CONST)
    assert c.integral_pos_e[2] == -0.15
    c = ref_pid.RefDSLPID()
    rpm, _, _ = c.computeControl(1 / 30, np.array([0, 0, -100.0]), np.array([0, 0, 0, 1.0]), np.zeros(3), np.zeros(3),
                                 target_pos=np.zeros(3))
    np.testing.assert_allclose(rpm, ref_pid.PWM2RPM_SCALE * ref_pid.MAX_PWM + ref_pid.PWM2RPM_CONST)


def test_calculate_next_step():
    """BaseAviary._calculateNextStep: within 1 m the float32 destination itself, else a unit step."""
    cur = np.array([0.1, 0.2, 0.3])
    dst = np.array([0.5, 0.1, 0.9], np.float32)
    out = ref_pid.calculate_next_step(cur, dst)
    assert out is dst
    dst = np.array([3.0, -1.0, 2.0], np.float32)
    out = ref_pid.calculate_next_step(cur, dst)
    assert abs(np.linalg.norm(out - cur) - 1.0) < 1e-15
    d = dst - cur
    np.testing.assert_allclose(out, cur + d / np.linalg.norm(d), rtol=0, atol=1e-15)


def _direct_matrix(target_thrust, yaw):
    z = target_thrust / np.linalg.norm(target_thrust)
    xc = np.array([math.cos(yaw), math.sin(yaw), 0])
    y = np.cross(z, xc) / np.linalg.norm(np.cross(z, xc))
    x = np.cross(y, z)
    return np.vstack([x, y, z]).transpose()


def test_scipy_euler_round_trip_is_identity():
    """DSLPIDControl.py:205 + :242-244 (matrix -> intrinsic XYZ -> quaternion (mislabelled but
    passed back in the same order) -> matrix) returns the input rotation to rounding, which is
    why the HIP path uses the target rotation directly."""
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(2000):
        tt = rng.normal(0, 1, 3) + np.array([0, 0, 0.3])
        yaw = rng.uniform(-math.pi, math.pi)
        M = _direct_matrix(tt, yaw)
        e = Rotation.from_matrix(M).as_euler('XYZ', degrees=False)
        q = Rotation.from_euler('XYZ', e, degrees=False).as_quat()
        w, x, y, z = q
        M2 = Rotation.from_quat([w, x, y, z]).as_matrix()
        worst = max(worst, np.abs(M2 - M).max())
    assert worst < 5e-15


def test_controller_persists_across_reset():
    """BaseAviary.reset never resets the controllers (created once in BaseRLAviary.__init__)."""
    env = RefAviary(act="one_d_pid", task="hover")
    for _ in range(5):
        env.step(np.array([[0.7]], np.float32))
    cs = env.ctrl_state().copy()
    assert np.abs(cs).max() > 0
    env.reset()
    np.testing.assert_array_equal(env.ctrl_state(), cs)


def test_vel_zero_direction_and_f32_norm():
    env = RefAviary(act="vel", task="none")
    env.step(np.zeros((1, 4), np.float32))
    # norm3_f32 is the fixed float32 order the HIP path uses
    t = np.array([0.3, -0.4, 0.1], np.float32)
    n = ref_pid.norm3_f32(t)
    assert n.dtype == np.float32
    assert abs(float(n) - math.sqrt(0.26)) < 1e-7


def test_geom_wrench_pid_tracks_waypoint():
    """With the PYB force placement (prop-position torques) the DSL PID flies to a waypoint; on
    DYN the reference's cf2x roll-sign quirk (BaseAviary.py:847) makes the same controller
    diverge in roll - reproduced, not fixed."""
    env = RefAviary(act="pid", task="none", ctrl_freq=48, wrench="geom")
    for _ in range(240):
        env.step(np.array([[0.3, 0.2, 0.5]], np.float32))
    assert np.linalg.norm(env.pos[0] - [0.3, 0.2, 0.5]) < 0.05
    dyn = RefAviary(act="pid", task="none", ctrl_freq=48)
    for _ in range(60):
        dyn.step(np.array([[0.3, 0.2, 0.5]], np.float32))
    assert np.abs(dyn.rpy[0, 0]) > 0.4


@pytest.mark.parametrize("act", ["pid", "vel", "one_d_pid"])
def test_obs_width_and_action_buffer(act):
    env = RefAviary(act=act, task="hover")
    A = {"pid": 3, "vel": 4, "one_d_pid": 1}[act]
    obs, _ = env.reset()
    assert obs.shape == (1, 12 + 15 * A)
    a = np.full((1, A), 0.25, np.float32)
    obs, *_ = env.step(a)
    np.testing.assert_array_equal(obs[0, -A:], a[0])
