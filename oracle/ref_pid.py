"""CPU restatement of DSLPIDControl and the PID / VEL / ONE_D_PID action paths
(TEST INFRASTRUCTURE ONLY - only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module).

What it restates (paths relative to the reference root, ``gym_pybullet_drones/``):
  * ``control/DSLPIDControl.py:37-78``   coefficients, mixer, reset()
  * ``control/DSLPIDControl.py:82-145``  computeControl()
  * ``control/DSLPIDControl.py:149-208`` _dslPIDPositionControl()
  * ``control/DSLPIDControl.py:212-259`` _dslPIDAttitudeControl()
  * ``control/BaseControl.py:35-39``     GRAVITY = g*m, KF read from the cf2x URDF
  * ``envs/BaseRLAviary.py:73-76``       one DSLPIDControl(CF2X) per drone, also for CF2P
  * ``envs/BaseRLAviary.py:93-95``       SPEED_LIMIT = 0.03 * MAX_SPEED_KMH * (1000/3600)
  * ``envs/BaseRLAviary.py:193-235``     PID / VEL / ONE_D_PID branches of _preprocessAction
  * ``envs/BaseAviary.py:1105-1147``     _calculateNextStep() (the routing waypoint)

The rotation helpers are the reference's own third-party calls: ``scipy.spatial.transform
.Rotation`` (installed here; the reference pins scipy ^1.10, ``pyproject.toml:19``) and the
pybullet helpers restated in ``bullet_math.py``.  Controllers are never reset by env.reset()
(the reference creates them once in ``BaseRLAviary.__init__`` and ``BaseAviary.reset`` does not
touch them), so integral errors and ``last_rpy`` carry over episodes.

Float32 conventions (numpy ^1.24 value-based casting, the reference's pinned toolchain):
  * VEL: ``np.linalg.norm(target[0:3])`` of the float32 action is a float32 BLAS ``sdot``
    whose rounding depends on the BLAS kernel of the host; this restatement fixes it to
    ``sqrtf((t0*t0 + t1*t1) + t2*t2)`` in float32 without FMA (``norm3_f32``) and the HIP
    path uses the same order.  ``SPEED_LIMIT * np.abs(target[3])`` is a float64 scalar
    (python float x numpy float32 scalar) that numpy 1.x then casts to float32 when it
    multiplies the float32 unit vector.
  * PID: ``destination - current_position`` promotes the float32 action to float64; with
    ``distance <= 1`` the float32 destination itself (exact in float64) becomes the target.
  * ONE_D_PID: ``np.array([0, 0, target[0]])`` is float64.
"""
import math

import numpy as np
from scipy.spatial.transform import Rotation

from .bullet_math import euler_from_quat, quat_to_mat
from .params import derived

# DSLPIDControl.py:37-60 (CF2X mixer: BaseRLAviary always builds the CF2X controller)
P_COEFF_FOR = np.array([.4, .4, 1.25])
I_COEFF_FOR = np.array([.05, .05, .05])
D_COEFF_FOR = np.array([.2, .2, .5])
P_COEFF_TOR = np.array([70000., 70000., 60000.])
I_COEFF_TOR = np.array([.0, .0, 500.])
D_COEFF_TOR = np.array([20000., 20000., 12000.])
PWM2RPM_SCALE = 0.2685
PWM2RPM_CONST = 4070.3
MIN_PWM = 20000
MAX_PWM = 65535
MIXER_MATRIX = np.array([[-.5, -.5, -1], [-.5, .5, 1], [.5, .5, -1], [.5, -.5, 1]])


def norm3_f32(t):
    """float32 Euclidean norm of a 3-vector in the fixed order used by the HIP path."""
    t = np.asarray(t, dtype=np.float32)
    with np.errstate(all="ignore"):
        s = np.float32(np.float32(t[0] * t[0]) + np.float32(t[1] * t[1]))
        s = np.float32(s + np.float32(t[2] * t[2]))
        return np.float32(np.sqrt(s))


class RefDSLPID:
    """One DSLPIDControl(DroneModel.CF2X) instance, reference-shaped."""

    def __init__(self, g=9.8):
        cf2x = derived("cf2x")
        self.GRAVITY = g * cf2x["m"]      # BaseControl.py:35
        self.KF = cf2x["kf"]              # BaseControl.py:37
        self.P_COEFF_FOR, self.I_COEFF_FOR, self.D_COEFF_FOR = P_COEFF_FOR.copy(), I_COEFF_FOR.copy(), D_COEFF_FOR.copy()
        self.P_COEFF_TOR, self.I_COEFF_TOR, self.D_COEFF_TOR = P_COEFF_TOR.copy(), I_COEFF_TOR.copy(), D_COEFF_TOR.copy()
        self.MIXER_MATRIX = MIXER_MATRIX
        self.reset()

    def reset(self):
        self.control_counter = 0
        self.last_rpy = np.zeros(3)
        self.last_pos_e = np.zeros(3)
        self.integral_pos_e = np.zeros(3)
        self.last_rpy_e = np.zeros(3)
        self.integral_rpy_e = np.zeros(3)

    def computeControl(self, control_timestep, cur_pos, cur_quat, cur_vel, cur_ang_vel, target_pos,
                       target_rpy=np.zeros(3), target_vel=np.zeros(3), target_rpy_rates=np.zeros(3)):
        self.control_counter += 1
        thrust, computed_target_rpy, pos_e = self._position(control_timestep, cur_pos, cur_quat, cur_vel,
                                                            target_pos, target_rpy, target_vel)
        rpm = self._attitude(control_timestep, thrust, cur_quat, computed_target_rpy, target_rpy_rates)
        cur_rpy = euler_from_quat(cur_quat)
        return rpm, pos_e, computed_target_rpy[2] - cur_rpy[2]

    def _position(self, control_timestep, cur_pos, cur_quat, cur_vel, target_pos, target_rpy, target_vel):
        """DSLPIDControl.py:187-208."""
        cur_rotation = quat_to_mat(cur_quat)
        pos_e = target_pos - cur_pos
        vel_e = target_vel - cur_vel
        self.integral_pos_e = self.integral_pos_e + pos_e * control_timestep
        self.integral_pos_e = np.clip(self.integral_pos_e, -2., 2.)
        self.integral_pos_e[2] = np.clip(self.integral_pos_e[2], -0.15, .15)
        target_thrust = np.multiply(self.P_COEFF_FOR, pos_e) \
            + np.multiply(self.I_COEFF_FOR, self.integral_pos_e) \
            + np.multiply(self.D_COEFF_FOR, vel_e) + np.array([0, 0, self.GRAVITY])
        scalar_thrust = max(0., np.dot(target_thrust, cur_rotation[:, 2]))
        thrust = (math.sqrt(scalar_thrust / (4 * self.KF)) - PWM2RPM_CONST) / PWM2RPM_SCALE
        target_z_ax = target_thrust / np.linalg.norm(target_thrust)
        target_x_c = np.array([math.cos(target_rpy[2]), math.sin(target_rpy[2]), 0])
        target_y_ax = np.cross(target_z_ax, target_x_c) / np.linalg.norm(np.cross(target_z_ax, target_x_c))
        target_x_ax = np.cross(target_y_ax, target_z_ax)
        target_rotation = (np.vstack([target_x_ax, target_y_ax, target_z_ax])).transpose()
        target_euler = (Rotation.from_matrix(target_rotation)).as_euler('XYZ', degrees=False)
        return thrust, target_euler, pos_e

    def _attitude(self, control_timestep, thrust, cur_quat, target_euler, target_rpy_rates):
        """DSLPIDControl.py:240-259."""
        cur_rotation = quat_to_mat(cur_quat)
        cur_rpy = np.array(euler_from_quat(cur_quat))
        target_quat = (Rotation.from_euler('XYZ', target_euler, degrees=False)).as_quat()
        w, x, y, z = target_quat
        target_rotation = (Rotation.from_quat([w, x, y, z])).as_matrix()
        rot_matrix_e = np.dot((target_rotation.transpose()), cur_rotation) - np.dot(cur_rotation.transpose(), target_rotation)
        rot_e = np.array([rot_matrix_e[2, 1], rot_matrix_e[0, 2], rot_matrix_e[1, 0]])
        rpy_rates_e = target_rpy_rates - (cur_rpy - self.last_rpy) / control_timestep
        self.last_rpy = cur_rpy
        self.integral_rpy_e = self.integral_rpy_e - rot_e * control_timestep
        self.integral_rpy_e = np.clip(self.integral_rpy_e, -1500., 1500.)
        self.integral_rpy_e[0:2] = np.clip(self.integral_rpy_e[0:2], -1., 1.)
        target_torques = - np.multiply(self.P_COEFF_TOR, rot_e) \
            + np.multiply(self.D_COEFF_TOR, rpy_rates_e) \
            + np.multiply(self.I_COEFF_TOR, self.integral_rpy_e)
        target_torques = np.clip(target_torques, -3200, 3200)
        pwm = thrust + np.dot(self.MIXER_MATRIX, target_torques)
        pwm = np.clip(pwm, MIN_PWM, MAX_PWM)
        return PWM2RPM_SCALE * pwm + PWM2RPM_CONST

    # the controller state the HIP path keeps per drone: [int_pos(3), int_rpy(3), last_rpy(3)]
    def get_state(self):
        return np.concatenate([self.integral_pos_e, self.integral_rpy_e, self.last_rpy])

    def set_state(self, v):
        v = np.asarray(v, dtype=np.float64)
        self.integral_pos_e, self.integral_rpy_e, self.last_rpy = v[0:3].copy(), v[3:6].copy(), v[6:9].copy()


def calculate_next_step(current_position, destination, step_size=1):
    """BaseAviary._calculateNextStep (:1105-1147)."""
    direction = destination - current_position
    distance = np.linalg.norm(direction)
    if distance <= step_size:
        return destination
    normalized_direction = direction / distance
    return current_position + normalized_direction * step_size


def pid_action_rpm(kind, ctrl, state, target, ctrl_timestep, speed_limit):
    """BaseRLAviary._preprocessAction PID (:193-207), VEL (:208-223), ONE_D_PID (:226-235) for
    one drone; ``state`` is its 20-float state vector, ``target`` its float32 action row."""
    target = np.asarray(target, dtype=np.float32)
    if kind == "pid":
        next_pos = calculate_next_step(current_position=state[0:3], destination=target, step_size=1)
        rpm, _, _ = ctrl.computeControl(control_timestep=ctrl_timestep, cur_pos=state[0:3], cur_quat=state[3:7],
                                        cur_vel=state[10:13], cur_ang_vel=state[13:16], target_pos=next_pos)
        return rpm
    if kind == "vel":
        n = norm3_f32(target[0:3])
        if n != 0:
            with np.errstate(all="ignore"):
                v_unit_vector = (target[0:3] / n).astype(np.float32)
        else:
            v_unit_vector = np.zeros(3)
        # numpy 1.x: float64 scalar * float32 array -> float32 array
        scale = np.float32(np.float64(speed_limit) * np.float64(np.abs(target[3])))
        target_vel = (scale * v_unit_vector.astype(np.float32)).astype(np.float32) if n != 0 else \
            np.float64(speed_limit) * np.float64(np.abs(target[3])) * v_unit_vector
        rpm, _, _ = ctrl.computeControl(control_timestep=ctrl_timestep, cur_pos=state[0:3], cur_quat=state[3:7],
                                        cur_vel=state[10:13], cur_ang_vel=state[13:16], target_pos=state[0:3],
                                        target_rpy=np.array([0, 0, state[9]]), target_vel=target_vel)
        return rpm
    if kind == "one_d_pid":
        rpm, _, _ = ctrl.computeControl(control_timestep=ctrl_timestep, cur_pos=state[0:3], cur_quat=state[3:7],
                                        cur_vel=state[10:13], cur_ang_vel=state[13:16],
                                        target_pos=state[0:3] + 0.1 * np.array([0, 0, target[0]]))
        return rpm
    raise ValueError(kind)
