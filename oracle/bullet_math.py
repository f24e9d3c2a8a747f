"""PyBullet/Bullet3 rotation helpers restated in numpy fp64 (TEST INFRASTRUCTURE ONLY).

The reference's DYN path calls four pybullet helpers (third-party, ``pybullet ^3.2.5``,
``pyproject.toml:20``; Bullet3 compiled with double precision).  pybullet is not installed
in this image and the reference may not be imported here, so the published Bullet3
algorithms are restated below and cross-checked against scipy ``Rotation`` in
``tests/test_oracle_kat.py`` (KAT-6):

* ``getMatrixFromQuaternion`` (call sites ``BaseAviary.py:771, :836``)
    -> ``btMatrix3x3::setRotation``: s = 2/|q|^2, row-major 3x3.
* the state round trip ``resetBasePositionAndOrientation`` -> ``getBasePositionAndOrientation``
  (``BaseAviary.py:862`` then ``:517``): the base orientation goes through a ``btTransform``
  (quaternion -> basis -> quaternion), i.e. ``btMatrix3x3::getRotation`` of the basis above.
  That re-normalises q and fixes its sign (w > 0 when trace > 0).
* ``getEulerFromQuaternion`` (``BaseAviary.py:518``) -> ``btQuaternion::getEulerZYX``
  with its two gimbal branches at |sarg| >= 0.99999.
* ``getQuaternionFromEuler`` (``BaseAviary.py:488``) -> ``btQuaternion::setEulerZYX(yaw, pitch, roll)``.

Quaternions are [x, y, z, w] (pybullet order).  All functions are scalar (one quaternion)
so that the reference-shaped oracle keeps the reference's per-drone call structure; the
``*_batch`` variants are vectorised equivalents used for golden-vector generation.

Parity status: these semantics are *restated from Bullet3 knowledge* and cannot be run
against real pybullet in this pipeline -> the Bullet-helper part of the oracle is
"parity unpinned" except through the analytic checks (scipy cross-check, orthogonality,
round-trip identities).
"""
import math

import numpy as np


def quat_to_mat(q):
    """btMatrix3x3::setRotation(q) -> 3x3 row-major (pybullet getMatrixFromQuaternion)."""
    x, y, z, w = float(q[0]), float(q[1]), float(q[2]), float(q[3])
    d = x * x + y * y + z * z + w * w
    s = 2.0 / d
    xs, ys, zs = x * s, y * s, z * s
    wx, wy, wz = w * xs, w * ys, w * zs
    xx, xy, xz = x * xs, x * ys, x * zs
    yy, yz, zz = y * ys, y * zs, z * zs
    return np.array([[1.0 - (yy + zz), xy - wz, xz + wy],
                     [xy + wz, 1.0 - (xx + zz), yz - wx],
                     [xz - wy, yz + wx, 1.0 - (xx + yy)]])


def mat_to_quat(m):
    """btMatrix3x3::getRotation(basis) -> [x, y, z, w]."""
    trace = m[0, 0] + m[1, 1] + m[2, 2]
    t = [0.0, 0.0, 0.0, 0.0]
    if trace > 0.0:
        s = math.sqrt(trace + 1.0)
        t[3] = s * 0.5
        s = 0.5 / s
        t[0] = (m[2, 1] - m[1, 2]) * s
        t[1] = (m[0, 2] - m[2, 0]) * s
        t[2] = (m[1, 0] - m[0, 1]) * s
    else:
        if m[0, 0] < m[1, 1]:
            i = 2 if m[1, 1] < m[2, 2] else 1
        else:
            i = 2 if m[0, 0] < m[2, 2] else 0
        j = (i + 1) % 3
        k = (i + 2) % 3
        s = math.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        t[i] = s * 0.5
        s = 0.5 / s
        t[3] = (m[k, j] - m[j, k]) * s
        t[j] = (m[j, i] + m[i, j]) * s
        t[k] = (m[k, i] + m[i, k]) * s
    return np.array(t)


def quat_roundtrip(q):
    """Orientation as read back after a reset: quaternion -> btTransform basis -> quaternion."""
    return mat_to_quat(quat_to_mat(q))


def _asin_clamped(x):
    # btAsin clamps its argument to [-1, 1]
    return math.asin(min(1.0, max(-1.0, x)))


def euler_from_quat(q):
    """btQuaternion::getEulerZYX -> (roll, pitch, yaw) as pybullet returns them."""
    x, y, z, w = float(q[0]), float(q[1]), float(q[2]), float(q[3])
    sqx, sqy, sqz, squ = x * x, y * y, z * z, w * w
    sarg = -2.0 * (x * z - w * y)
    if sarg <= -0.99999:
        pitch = -0.5 * math.pi
        roll = 0.0
        yaw = 2.0 * math.atan2(x, -y)
    elif sarg >= 0.99999:
        pitch = 0.5 * math.pi
        roll = 0.0
        yaw = 2.0 * math.atan2(-x, y)
    else:
        pitch = _asin_clamped(sarg)
        roll = math.atan2(2.0 * (y * z + w * x), squ - sqx - sqy + sqz)
        yaw = math.atan2(2.0 * (x * y + w * z), squ + sqx - sqy - sqz)
    return np.array([roll, pitch, yaw])


def quat_from_euler(rpy):
    """btQuaternion::setEulerZYX(yaw, pitch, roll) -> [x, y, z, w]."""
    roll, pitch, yaw = float(rpy[0]), float(rpy[1]), float(rpy[2])
    hy, hp, hr = yaw * 0.5, pitch * 0.5, roll * 0.5
    cy, sy = math.cos(hy), math.sin(hy)
    cp, sp = math.cos(hp), math.sin(hp)
    cr, sr = math.cos(hr), math.sin(hr)
    return np.array([sr * cp * cy - cr * sp * sy,
                     cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy,
                     cr * cp * cy + sr * sp * sy])
