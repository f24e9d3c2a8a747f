"""The drone <-> drone contact restatement (oracle/bullet_mb.py drone_contact; parity unpinned
against pybullet): geometry known answers and the solve's invariants, on the CPU."""
import math

import numpy as np

from oracle.bullet_mb import (LINEAR_SLOP, breaking_threshold, drone_contact, drone_contacts, pair_geometry, plane_space)
from oracle.bullet_math import quat_from_euler, quat_to_mat
from oracle.params import derived

P = derived("cf2x")
R_, HH, ZO = P["collision_r"], P["collision_h"] / 2, P["collision_z_offset"]
M, I = P["m"], np.array([P["ixx"], P["iyy"], P["izz"]])
DT = 1 / 240
EZ = np.array([0.0, 0.0, 1.0])


def test_pair_geometry_known_answers():
    # side by side, level: the rims face each other along the centre line
    n, pb, d = pair_geometry(np.array([0.2, 0, 1.0]), EZ, np.array([0.0, 0, 1.0]), EZ, R_, HH)
    assert abs(d - (0.2 - 2 * R_)) < 1e-15 and np.allclose(n, [1, 0, 0]) and np.allclose(pb, [R_, 0, 1.0])
    # stacked, coaxial: the caps face each other
    n, pb, d = pair_geometry(np.array([0.0, 0, 1.05]), EZ, np.array([0.0, 0, 1.0]), EZ, R_, HH)
    assert abs(d - (0.05 - 2 * HH)) < 1e-15 and np.allclose(n, [0, 0, 1])
    # overlapping side by side: depth along the centre line, the point in both cylinders
    n, pb, d = pair_geometry(np.array([0.115, 0, 1.0]), EZ, np.array([0.0, 0, 1.0]), EZ, R_, HH)
    assert abs(d + (2 * R_ - 0.115)) < 1e-15 and np.allclose(n, [1, 0, 0]) and abs(pb[2] - 1.0) < 1e-15
    # overlapping stacked with an offset: the axis is the direction of least overlap
    n, pb, d = pair_geometry(np.array([0.03, 0, 1.02]), EZ, np.array([0.0, 0, 1.0]), EZ, R_, HH)
    assert np.allclose(n, [0, 0, 1]) and abs(d + (2 * HH - 0.02)) < 1e-15


def test_plane_space_matches_the_plane_rows():
    t1, t2 = plane_space(EZ)
    assert np.array_equal(t1, [0.0, -1.0, 0.0]) and np.array_equal(t2, [1.0, 0.0, 0.0])
    rng = np.random.default_rng(0)
    for _ in range(50):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        t1, t2 = plane_space(n)
        assert abs(t1 @ n) < 1e-15 and abs(t2 @ n) < 1e-15 and abs(t1 @ t2) < 1e-15
        assert abs(np.linalg.norm(t1) - 1) < 1e-15 and abs(np.linalg.norm(t2) - 1) < 1e-15


def _solve(pos, rpys, vel, omg):
    rot = np.array([quat_to_mat(quat_from_euler(np.array(r, dtype=np.float64))) for r in rpys])
    return drone_contact(np.array(pos, float), rot, np.array(vel, float), np.array(omg, float), M, I, DT, R_, HH, ZO)


def test_head_on_stops_and_conserves_momentum():
    pos = [[0, 0, 1.0], [0.121, 0.0, 1.0]]
    vel = [[1.0, 0, 0], [-1.0, 0, 0]]
    v, w = _solve(pos, [(0, 0, 0)] * 2, vel, np.zeros((2, 3)))
    assert np.allclose(v.sum(0), 0, atol=1e-14)
    gap = 0.121 - 2 * R_
    # speculative row: the closing speed is cut to what closes the gap (+ the slop) in one step
    assert abs((v[1, 0] - v[0, 0]) * -DT - (gap + LINEAR_SLOP)) < 1e-12
    assert np.abs(w).max() < 1e-12


def test_off_centre_impulse_conserves_linear_and_angular_momentum():
    rng = np.random.default_rng(3)
    for _ in range(20):
        pos = [[0, 0, 1.0], [0.115 + rng.uniform(0, 0.004), rng.uniform(-0.02, 0.02), 1.0 + rng.uniform(-0.01, 0.01)]]
        rpys = [rng.uniform(-0.3, 0.3, 3), rng.uniform(-0.3, 0.3, 3)]
        vel = [rng.uniform(0, 1, 3) * [1, 0.2, 0.2], -rng.uniform(0, 1, 3) * [1, 0.2, 0.2]]
        omg = rng.uniform(-2, 2, (2, 3))
        v, w = _solve(pos, rpys, vel, omg)
        np.testing.assert_allclose(v.sum(0), np.sum(vel, 0), atol=1e-12)
        rot = [quat_to_mat(quat_from_euler(r)) for r in rpys]
        ang = lambda vv, ww: sum(M * np.cross(pos[i], vv[i]) + rot[i] @ (I * (rot[i].T @ ww[i])) for i in range(2))
        # normal impulses act along one line (exact); a friction impulse acts at A's and B's points,
        # |p_A - p_B| = |dist| <= 5 mm apart (as Bullet's), so it moves L by <= dist * mu * m |dv|
        np.testing.assert_allclose(ang(v, w), ang(np.array(vel), omg), atol=5e-3 * 0.25 * M * 2.0)


def test_far_and_separating_pairs_unchanged():
    pos = [[0, 0, 1.0], [0.3, 0, 1.0]]
    vel = [[0.5, 0, 0], [-0.5, 0, 0]]
    v, w = _solve(pos, [(0, 0, 0)] * 2, vel, np.zeros((2, 3)))
    assert np.array_equal(v, vel) and not w.any()
    pos = [[0, 0, 1.0], [0.1205, 0, 1.0]]          # in contact range, moving apart: zero impulse
    vel = [[-0.5, 0, 0], [0.5, 0, 0]]
    v, w = _solve(pos, [(0, 0, 0)] * 2, vel, np.zeros((2, 3)))
    assert np.array_equal(v, vel)


def test_contact_order_and_slot_cap():
    # five drones stacked tightly: 4 adjacent contacts (+ none at two levels apart), in (i, j) order
    pos = np.array([[0, 0, 1.0 + 0.0245 * k] for k in range(5)])
    rot = np.array([np.eye(3)] * 5)
    cons = drone_contacts(pos, rot, R_, HH, ZO)
    assert [(c[0], c[1]) for c in cons] == [(0, 1), (1, 2), (2, 3), (3, 4)]
    # a three-drone cluster all within the threshold: 3 pairs fit the 3 slots; four mutually
    # touching drones (6 pairs) keep the first 4
    tri = np.array([[0, 0, 1.0], [0.12, 0, 1.0], [0.06, 0.1039, 1.0]])
    assert len(drone_contacts(tri, rot[:3], R_, HH, ZO)) == 3
    quad = np.array([[0, 0, 1.0], [0.0, 0, 1.0245], [0.0, 0, 1.049], [0.0, 0, 1.0735]])
    quad[:, 0] += [0, 0.001, 0.002, 0.003]
    cons = drone_contacts(quad, rot[:4], R_, HH, ZO)
    assert len(cons) == 3 or len(cons) == 4
    assert breaking_threshold(R_, HH) < 0.002
    assert math.isfinite(cons[0][4])
