"""Stored quaternions whose reference attitude decisions sit at their thresholds (test helper).

The reference decides on libm outputs of the readback quaternion (pybullet's getEulerZYX:
``atan2`` / ``asin``, BaseAviary.py:517-518):
* truncation: ``abs(roll) > .4 or abs(pitch) > .4`` (HoverAviary.py:111, MultiHoverAviary.py:124);
* the ground-effect gate: ``abs(roll) < np.pi/2 and abs(pitch) < np.pi/2`` (BaseAviary.py:742),
  which flips where atan2 rounds to RN(pi/2) (roll within ~2e-16 of pi/2) and at the
  getEulerZYX gimbal branch (|sarg| >= 0.99999, pitch = +-pi/2).
The candidates below walk ulp grids around each threshold and keep the stored quaternions whose
oracle decision (``oracle.bullet_math``: literal Bullet readback + Python's math = glibc) lands
within a few ulp of it, on both sides.
"""
import math

import numpy as np

from oracle.bullet_math import euler_from_quat, quat_roundtrip


def literal_args(q):
    """getEulerZYX's (sarg, a, b) of the readback of stored quaternion q."""
    x, y, z, w = (float(v) for v in quat_roundtrip(q))
    return -2.0 * (x * z - w * y), 2.0 * (y * z + w * x), w * w - x * x - y * y + z * z


def oracle_rpy(q):
    return euler_from_quat(quat_roundtrip(q))


def tilted(q):
    r = oracle_rpy(q)
    return abs(r[0]) > .4 or abs(r[1]) > .4


def upright(q):
    r = oracle_rpy(q)
    return bool(np.abs(r[0]) < np.pi / 2 and np.abs(r[1]) < np.pi / 2)


def _ulps(x, k):
    for _ in range(abs(k)):
        x = math.nextafter(x, math.inf if k > 0 else -math.inf)
    return x


def tilt_cases(span=12):
    """Stored quaternions with |roll| or |pitch| within a few ulp of 0.4: pure roll / pitch of
    both signs, roll with a yaw (so every readback component is nonzero), and roll beside a
    pitch.  Returns [K, 4] and the ulp distance of the deciding angle from 0.4."""
    out, dist = [], []
    for axis, sign, yaw, other in ((0, 1, 0.0, 0.0), (0, -1, 0.0, 0.0), (1, 1, 0.0, 0.0), (1, -1, 0.0, 0.0),
                                   (0, 1, 1.0, 0.0), (0, -1, -2.5, 0.1), (1, 1, 0.7, 0.2)):
        half = 0.2
        for k in range(-span, span + 1):
            h = _ulps(half, k)
            # compose: (roll or pitch) then a small other-axis tilt and the yaw, Bullet order ZYX
            ang = [0.0, 0.0, yaw]
            ang[axis] = sign * 2 * h
            ang[1 - axis] = other
            q = _from_euler(ang)
            r = oracle_rpy(q)
            d = (abs(r[axis]) - 0.4) / math.ulp(0.4)
            out.append(q)
            dist.append(d)
    return np.array(out), np.array(dist)


def _from_euler(rpy):
    from oracle.bullet_math import quat_from_euler
    return quat_from_euler(rpy)


def roll_beyond_half_pi_cases():
    """b <= 0 and the roll = +-pi/2 edge for truncation: roll near +-pi, exactly b = +0 / -0."""
    s = math.sqrt(0.5)
    qs = [[s, 0.0, 0.0, s], [-s, 0.0, 0.0, s], [1.0, 0.0, 0.0, 0.0], [math.sin(1.5), 0.0, 0.0, math.cos(1.5)],
          [math.sin(-1.55), 0.0, 0.0, math.cos(-1.55)], [0.0, 0.0, 0.0, 1.0]]
    return np.array(qs)


def upright_edge_cases(span=10):
    """Stored quaternions around roll = pi/2 (b ~ 1e-16) and the gimbal edge |sarg| = 0.99999."""
    qs = []
    # roll within ~1e-15 of +-pi/2, with and without a yaw (b = cos(roll) ~ 1e-16: atan2 rounds
    # to RN(pi/2) for b < 1.7e-16 |a|)
    for k in range(-3, 4):
        for sign in (1.0, -1.0):
            for m in range(-3 * span, 3 * span + 1):
                qs.append(_from_euler([sign * (math.pi / 2 + k * 1.1e-16), 0.0, 0.1 * m]))
    s = math.sqrt(0.5)
    for i in range(-2, 3):
        for j in range(-2, 3):
            qs.append([_ulps(s, i), 0.0, 0.0, _ulps(s, j)])
    # pitch near asin(0.99999), stepped so that sarg = sin(pitch) moves by about an ulp
    p = math.asin(0.99999)
    for i in range(-3 * span, 3 * span + 1):
        h = (p + i * 2.5e-14) / 2
        for yaw in (0.0, 0.4):
            for sgn in (1.0, -1.0):
                qs.append(_from_euler([0.0, sgn * 2 * h, yaw]))
    qs = np.array(qs)
    keep = []
    for q in qs:
        sarg, a, b = literal_args(q)
        if abs(b) < 1e-14 or abs(abs(sarg) - 0.99999) < 1e-14:
            keep.append(q)
    return np.array(keep)
