"""The drone <-> drone contact restatement (oracle/bullet_mb.py drone_contact; parity unpinned
against pybullet): geometry known answers and the solve's invariants, on the CPU."""
import math

import numpy as np

from oracle.bullet_mb import (CORE_MARGINS, LINEAR_SLOP, breaking_threshold, cyl_project, drone_contact, drone_contacts, pair_geometry,
                              pair_near, plane_space)
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


def _rot(rpys):
    return np.array([quat_to_mat(quat_from_euler(np.array(r, dtype=np.float64))) for r in rpys])


def _pairs(cons):
    """the (i, j) sequence of a contact list, one entry per pair (its points are consecutive)"""
    out = []
    for c in cons:
        if not out or out[-1] != (c[0], c[1]):
            out.append((c[0], c[1]))
    return out


def test_contact_order_and_no_cap():
    # five drones stacked tightly: 4 adjacent contacts (+ none at two levels apart), in (i, j) order;
    # each a cap-to-cap contact: four points, Bullet's manifold capacity - the face manifold's four
    # with the closest point (the cap centre) in the slot btPersistentManifold::sortCachedPoints
    # frees: slot 0 (the lens tip (s - r) u; areas 4 r^4, 4 r^4, r^4, r^4, the first of the tie)
    pos = np.array([[0, 0, 1.0 + 0.0245 * k] for k in range(5)])
    rot = np.array([np.eye(3)] * 5)
    cons = drone_contacts(pos, rot, R_, HH, ZO)
    assert _pairs(cons) == [(0, 1), (1, 2), (2, 3), (3, 4)]
    assert len(cons) == 4 * 4 and all(abs(c[4] - (0.0245 - 2 * HH)) < 1e-15 for c in cons)
    for k in range(4):
        centre = cons[4 * k][3]
        assert abs(centre[0]) < 1e-15 and abs(centre[1]) < 1e-15      # the cap centre took slot 0
        for c in cons[4 * k + 1:4 * k + 4]:
            assert math.hypot(c[3][0], c[3][1]) > 0.9 * (R_ - CORE_MARGINS[0])   # three rim points kept
    # four drones, six contacts (more than the env's D): a touching triangle with a fourth drone
    # resting on all three - every pair is kept
    tri = [[0, 0, 1.0], [0.1195, 0, 1.0], [0.05975, 0.1035, 1.0]]
    top = np.mean(tri, axis=0) + [0, 0, 2 * HH - 0.0005]
    quad = np.array(tri + [top])
    cons = drone_contacts(quad, rot[:4], R_, HH, ZO)
    assert _pairs(cons) == [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    # eight drones as a 2 x 2 x 2 stack: 12 face / side contacts plus the rims of the layers' diagonals
    cube = np.array([[0.1195 * (k & 1), 0.1195 * ((k >> 1) & 1), 1.0 + (2 * HH - 0.0005) * (k >> 2)] for k in range(8)])
    cons = drone_contacts(cube, np.array([np.eye(3)] * 8), R_, HH, ZO)
    assert len(_pairs(cons)) >= 12 and all(c[4] < breaking_threshold(R_, HH) for c in cons)
    assert breaking_threshold(R_, HH) < 0.002
    per = {}
    for c in cons:
        per[(c[0], c[1])] = per.get((c[0], c[1]), 0) + 1
    assert max(per.values()) == 4                      # never more than Bullet's MANIFOLD_CACHE_SIZE


def test_manifold_replace_rule():
    """bullet_mb.manifold_replace restates btPersistentManifold::sortCachedPoints: a cached point
    deeper than the new one is never replaced, otherwise the slot whose replacement spans the
    largest quad (|(new - c_a) x (c_b - c_c)|^2, Bullet's pairing) wins, the first of a tie."""
    from oracle.bullet_mb import manifold_replace, pair_manifold
    sq = [np.array(p, dtype=float) for p in ((-1, 0, 0), (1, 0, 0), (0, 1, 0), (0, -1, 0))]
    # the new point at the centre, all equally deep: res = (4, 4, 1, 1) -> slot 0 (tie: the first)
    assert manifold_replace(np.zeros(3), 0.0, [(p, 0.0) for p in sq]) == 0
    # rounding-level depth differences do not protect a slot (MANIFOLD_DEPTH_TIE)
    assert manifold_replace(np.zeros(3), 0.0, [(sq[0], -1e-13)] + [(p, 0.0) for p in sq[1:]]) == 0
    # a truly deeper slot 0 is kept: the best of the others (res1 = 4) replaced
    assert manifold_replace(np.zeros(3), 0.0, [(sq[0], -1e-3)] + [(p, 0.0) for p in sq[1:]]) == 1
    # a new point far out along +x spans the largest quad in place of slot 1 (res1 = |(new - c0) x (c3 - c2)|^2)
    assert manifold_replace(np.array([3.0, 0, 0]), 0.0, [(p, 0.0) for p in sq]) == 1
    # fewer than four face points: the closest point first, then the face points (no replacement)
    n = np.array([0, 0, 1.0])
    got = pair_manifold(np.zeros(3), 0.0, n, [(sq[0], 0.0), (sq[1], 0.0)])
    assert len(got) == 3 and got[0][1] == 0.0 and np.array_equal(got[1][0], sq[0])


def test_face_manifold_points():
    """A cap-to-cap contact's face manifold (bullet_mb.face_points): four points spanning the overlap
    of the two caps, each at its own distance; side-by-side and rim contacts have none."""
    from oracle.bullet_mb import CORE_MARGINS, face_points
    mg = CORE_MARGINS[0]
    r = R_ - mg
    # level, offset 0.03 in x, 0.5 mm apart: tips at x = 0.03 - r and r, corners at x = 0.015
    cb, ca = np.array([0.0, 0, 1.0]), np.array([0.03, 0, 1.0 + 2 * HH + 0.0005])
    pts = face_points(ca, EZ, cb, EZ, EZ, R_, HH, mg)
    w = math.sqrt(r * r - 0.015 ** 2)
    want = [[0.03 - r, 0, 0], [r, 0, 0], [0.015, w, 0], [0.015, -w, 0]]
    for (pb, d), xy in zip(pts, want):
        assert abs(d - 0.0005) < 1e-15 and np.allclose(pb, cb + [xy[0], xy[1], HH], atol=1e-15)
    # A tilted by 0.02 rad about y: the points' distances follow A's cap plane
    rot = quat_to_mat(quat_from_euler(np.array([0.0, 0.02, 0.0])))
    pts = face_points(ca, rot[:, 2], cb, EZ, EZ, R_, HH, mg)
    ds = [d for _, d in pts]
    assert ds[0] > ds[2] > ds[1] and abs(ds[2] - ds[3]) < 1e-15
    # side by side: the caps do not face each other
    assert face_points(np.array([0.12, 0, 1.0]), EZ, cb, EZ, np.array([1.0, 0, 0]), R_, HH, mg) == []


def test_six_contacts_in_a_four_drone_pile_conserve_momentum():
    tri = [[0, 0, 1.0], [0.1195, 0, 1.0], [0.05975, 0.1035, 1.0]]
    top = np.mean(tri, axis=0) + [0, 0, 2 * HH - 0.0005]
    pos = np.array(tri + [top])
    rng = np.random.default_rng(7)
    vel = rng.uniform(-0.5, 0.5, (4, 3))
    vel[3] = [0, 0, -0.8]
    omg = rng.uniform(-1, 1, (4, 3))
    v, w = _solve(pos, [(0, 0, 0)] * 4, vel, omg)
    np.testing.assert_allclose(v.sum(0), vel.sum(0), atol=1e-12)
    assert v[3, 2] > -0.8 + 0.1                 # the top drone is held up by the three below


def test_broadphase_never_drops_a_contact():
    """pair_near's separating-axis reject bounds the distance from below: every pair it rejects
    is farther apart than the breaking threshold (random poses around contact range)."""
    rng = np.random.default_rng(11)
    brk = breaking_threshold(R_, HH)
    rejected = 0
    for _ in range(3000):
        ci = np.zeros(3)
        cj = rng.normal(size=3) * [0.08, 0.08, 0.03]
        ai, aj = _rot([rng.uniform(-0.6, 0.6, 3), rng.uniform(-0.6, 0.6, 3)])[:, :, 2]
        if pair_near(ci, ai, cj, aj, R_, HH, brk):
            continue
        rejected += 1
        # the true distance by many plain alternating-projection rounds (monotone, from above)
        y = np.zeros(3)
        for _ in range(400):
            y = cyl_project(np.zeros(3), aj, R_, HH, cyl_project(ci - cj, ai, R_, HH, y))
        d = np.linalg.norm(cyl_project(ci - cj, ai, R_, HH, y) - y)
        assert d > brk - 1e-6
    assert rejected > 100


def test_narrowphase_is_continuous_and_converged():
    """The narrowphase's distance is the cores' exact distance: against the certified bracket of
    tests/tools/np_exact.py (SLSQP upper bound, separating-axis lower bound, agreeing to 1e-9) on
    random, stacked, side-by-side, rim-to-rim and flat (tilts < 1 deg) near-contact pairs, within
    1e-5 m on every pair (p99 1e-8 m: the round-4 narrowphase was ~2 mm long at the median on
    stacked discs); every overlap of the cores is detected (distance <= CORE_SEP).  And a 1e-12
    change of the poses moves the contact by no more than 1e-10."""
    from tests.tools.np_accuracy import errors, pair_sets
    ca, cb = np.array([0.0, 0.0, 1.0]), np.array([0.121, 0.002, 1.001])
    aa, ab = _rot([(0.1, 0.2, 0.0), (-0.15, 0.05, 0.3)])[:, :, 2]
    n0, pb0, d0 = pair_geometry(ca, aa, cb, ab, R_, HH)
    n1, pb1, d1 = pair_geometry(ca + 1e-12, aa, cb, ab, R_, HH)
    assert abs(d1 - d0) < 1e-10 and np.abs(pb1 - pb0).max() < 1e-10
    allerr = []
    for name, pairs in pair_sets(40, np.random.default_rng(5)).items():
        e, _, (ok, ov) = errors(pairs)
        print(f"\n[narrowphase] {name}: {len(e)} separated, error max {e.max():.1e} min {e.min():.1e} m, "
              f"overlaps {ok}/{ov}")
        assert ok == ov
        assert e.min() > -1e-12          # a feasible pair: never below the exact distance
        allerr.append(e)
    e = np.concatenate(allerr)
    assert len(e) > 100 and e.max() <= 1e-5 and np.percentile(e, 99) <= 1e-5


def test_stacked_on_the_plane_island_solve():
    """A level drone dropped onto another resting on the plane: the island solve (the bottom
    drone's plane rows in the pair's Gauss-Seidel loop, as Bullet solves an island,
    ``BaseAviary.py:370``) holds the top one on top - round 4's pair-then-plane split let it sink
    ~1 cm into the bottom one.  Pinned: the top drone rests on the bottom one within the slop + 1 mm
    (gap >= 2 HH - 1e-5 - 1e-3 at every substep), the bottom drone stays on the plane, both come to
    rest level."""
    from oracle.ref_aviary import RefAviary
    env = RefAviary(num_drones=2, task="none", integrator="bullet", drones_per_env=2)
    raw = np.zeros((2, 20))
    raw[0, 0:3] = [0, 0, -ZO + HH - 1e-5]              # bottom drone on the plane
    raw[1, 0:3] = [0.01, 0, raw[0, 2] + 2 * HH + 0.001]
    raw[:, 6] = 1.0
    raw[1, 9] = -0.3
    env.set_raw_state(raw)
    out = env.integrate(np.zeros((240, 2, 4)))
    gap = out[:, 1, 2] - out[:, 0, 2]
    print(f"\n[stack] gap min {gap.min():.5f} m (touching: {2 * HH:.4f}), end {gap[-1]:.5f}, "
          f"max tilt {np.abs(out[:, :, 7:9]).max():.2e} rad")
    assert gap.min() >= 2 * HH - LINEAR_SLOP - 1e-3     # resting on top: no sinking into the bottom drone
    assert abs(out[-1, 0, 2] - raw[0, 2]) < 2e-3          # the bottom drone stays on the plane
    assert np.abs(out[-1, :, 10:13]).max() < 0.1          # both (nearly) at rest after 1 s
