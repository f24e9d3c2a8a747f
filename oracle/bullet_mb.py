"""Bullet3 ``btMultiBody`` base integration restated in numpy fp64 (TEST INFRASTRUCTURE ONLY).

ORACLE - only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.

What it restates.  Under ``Physics.PYB*`` the reference does not integrate the drone itself: it
applies the propeller / aero forces through ``p.applyExternalForce`` / ``applyExternalTorque``
(``envs/BaseAviary.py:679-811``) and calls ``p.stepSimulation()`` (``:369-370``).  The drone is a
URDF multibody (``p.loadURDF`` at ``:486-491``, no ``useMaximalCoordinates``): a 6-DOF base
(``cf2x.urdf:7-36``) with five zero-mass links on fixed joints (four props, the centre-of-mass
link, ``cf2x.urdf:38-98``).  Default multibody damping stays on - the reference's
``changeDynamics(linearDamping=0, angularDamping=0)`` is commented out (``:492-494``).  For one
such body in free flight one ``stepSimulation`` (``setTimeStep(PYB_TIMESTEP)``, ``:481``) is, in
Bullet3 (third-party: ``pybullet ^3.2.5``, ``pyproject.toml:20``; absent from this image and from
the reference tree):

* ``btDiscreteDynamicsWorld::stepSimulation(dt, maxSubSteps=0)``: one internal step of ``dt``;
  ``btMultiBodyDynamicsWorld::applyGravity`` adds ``m_gravity * mass`` to the base force
  (``setGravity(0, 0, -G)``, ``:479``; the links have zero mass).
* ``btMultiBodyDynamicsWorld::solveExternalForces`` ->
  ``btMultiBody::computeAccelerationsArticulatedBodyAlgorithmMultiDof``: base spatial velocity in
  the base frame (``rot = btMatrix3x3(m_baseQuat)``, world -> base), the bias force
  ``-(rot*torque, rot*force)`` + damping ``(I w k(1+|w|), m v k(1+|v|))``, ``k`` =
  ``m_angularDamping`` / ``m_linearDamping`` = 0.04 (btMultiBody constructor defaults, the
  DAMPING_K1 = DAMPING_K2 = damping form) + gyroscopic ``w x I w`` + ``m w x v``.  The zero-mass
  fixed links contribute only the forces applied to them, moved to the base as
  ``(r x f, f)``.  Base accelerations ``-I^-1 bias``, back to world:
  ``wdot = rot^T acc_w``, ``vdot = rot^T (acc_v + w x v)``.  Then
  ``applyDeltaVeeMultiDof(acc, dt)``: every velocity coordinate ``+= acc*dt`` and is clamped to
  ``+-m_maxCoordinateVelocity`` (100).
* ``btMultiBodyDynamicsWorld::integrateTransforms`` -> ``btMultiBody::stepPositionsMultiDof``:
  ``pos += dt * v`` with the NEW velocity, and the base quaternion (``m_baseQuat`` = world ->
  base) through the exponential map of ``btTransformUtil::integrateTransform``: with
  ``f = |w|`` clamped to ``0.5*SIMD_HALF_PI/dt`` when ``f*dt > ANGULAR_MOTION_THRESHOLD``
  (``0.5*SIMD_HALF_PI``), ``axis = w*(0.5 dt - dt^3/48 f^2)`` for ``f < 0.001`` else
  ``w*sin(0.5 f dt)/f``, ``m_baseQuat = m_baseQuat * (-axis, cos(0.5 f dt))``, normalised.
* readback (``getBasePositionAndOrientation`` / ``getBaseVelocity``, ``:517-519``): base position,
  the orientation ``m_baseQuat.inverse()`` through a ``btTransform`` basis (the same round trip
  as on the DYN path), world linear and angular velocity.

Not restated: contacts.  The collision cylinder (``cf2x.urdf:31-35``) against ``plane.urdf`` and
against other drones is Bullet's constraint solver (PGS, ERP, friction), which this path does
not model: a body below the plane keeps falling.  Bit-level rounding of Bullet's own operation
order (the world <-> base round trips of the link forces, the 6x6 inverse of the articulated
inertia) is not reproduced either; the restatement is exact in exact arithmetic.

Parity status: **parity unpinned** - restated from Bullet3 knowledge; pybullet cannot be run
in this pipeline.  Pinned by the analytic checks in ``tests/test_oracle_bullet.py`` (hover
equilibrium, damped free fall, terminal velocity, velocity clamp, damped spin, exponential map
against scipy).

Quaternions are [x, y, z, w].  The state keeps the *reported-frame* stored orientation
``q_s = m_baseQuat.inverse()`` (body -> world), the world linear velocity and the world angular
velocity (``m_realBuf[0:6]``).
"""
import math

import numpy as np

from .bullet_math import quat_to_mat

LIN_DAMP = 0.04                      # btMultiBody::m_linearDamping default
ANG_DAMP = 0.04                      # btMultiBody::m_angularDamping default
MAX_COORD_VEL = 100.0                # btMultiBody::m_maxCoordinateVelocity default
SIMD_HALF_PI = 0.5 * math.pi
ANGULAR_MOTION_THRESHOLD = 0.5 * SIMD_HALF_PI   # btTransformUtil.h


def qmul(a, b):
    """btQuaternion operator* (Hamilton product, [x, y, z, w])."""
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz])


def qnormalize(q):
    """btQuaternion::normalize: q *= 1/length()."""
    ln = math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return q * (1.0 / ln)


def qconj(q):
    """btQuaternion::inverse() (conjugate, no division)."""
    return np.array([-q[0], -q[1], -q[2], q[3]])


def base_quat_update(q_wb, omega_w, dt):
    """stepPositionsMultiDof's pQuatUpdateFun for the base (omega in world coordinates)."""
    ang = np.asarray(omega_w, dtype=np.float64)
    f = math.sqrt(ang[0] * ang[0] + ang[1] * ang[1] + ang[2] * ang[2])
    if f * dt > ANGULAR_MOTION_THRESHOLD:
        f = 0.5 * SIMD_HALF_PI / dt
    if f < 0.001:
        axis = ang * (0.5 * dt - (dt * dt * dt) * 0.020833333333 * f * f)
    else:
        axis = ang * (math.sin(0.5 * f * dt) / f)
    q = qmul(q_wb, np.array([-axis[0], -axis[1], -axis[2], math.cos(f * dt * 0.5)]))
    return qnormalize(q)


def multibody_step(pos, q_s, vel_w, omega_w, f_base, t_base, f_world, m, inertia, dt,
                   lin_damp=LIN_DAMP, ang_damp=ANG_DAMP, max_vel=MAX_COORD_VEL):
    """One ``stepSimulation`` of a free base with no contacts.

    ``f_base`` / ``t_base``: force and torque in the base frame (the link forces moved to the
    base COM); ``f_world``: world-frame base force (gravity).  Returns the new
    (pos, q_s, vel_w, omega_w)."""
    inertia = np.asarray(inertia, dtype=np.float64)
    q_wb = qconj(q_s)                                        # m_baseQuat
    rot = quat_to_mat(q_wb)                                  # rot_from_parent[0]: world -> base
    w = rot @ np.asarray(omega_w, dtype=np.float64)          # spatVel[0] angular
    v = rot @ np.asarray(vel_w, dtype=np.float64)            # spatVel[0] linear
    force = np.asarray(f_base, dtype=np.float64) + rot @ np.asarray(f_world, dtype=np.float64)
    torque = np.asarray(t_base, dtype=np.float64)
    kw = ang_damp + ang_damp * math.sqrt(w @ w)
    kv = lin_damp + lin_damp * math.sqrt(v @ v)
    iw = inertia * w
    zero_ang = -torque + iw * kw + np.cross(w, iw)           # zeroAccSpatFrc[0] (+ gyro term)
    zero_lin = -force + m * v * kv + m * np.cross(w, v)
    acc_ang = -(zero_ang / inertia)                          # spatAcc[0] = -I^-1 zeroAccSpatFrc[0]
    acc_lin = -(zero_lin / m)
    wdot = rot.T @ acc_ang                                   # back to the world frame
    vdot = rot.T @ (acc_lin + np.cross(w, v))
    omega_new = np.clip(np.asarray(omega_w, dtype=np.float64) + wdot * dt, -max_vel, max_vel)
    vel_new = np.clip(np.asarray(vel_w, dtype=np.float64) + vdot * dt, -max_vel, max_vel)
    pos_new = np.asarray(pos, dtype=np.float64) + dt * vel_new
    q_s_new = qconj(base_quat_update(q_wb, omega_new, dt))
    return pos_new, q_s_new, vel_new, omega_new
