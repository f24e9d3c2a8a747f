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

Ground-plane contact (``p.loadURDF("plane.urdf")``, ``:484``; the drone <-> plane collision filter
at ``:500-503`` is commented out, so the pair collides) is restated as ``plane_contact`` below:
Bullet's multibody contact constraints solved by projected Gauss-Seidel inside
``btMultiBodyConstraintSolver`` between the velocity update and ``integrateTransforms``.  The
contact set is this restatement's own (see ``plane_contact``).  Drone <-> drone collisions
(cylinder vs cylinder, MultiHoverAviary's drones, ``:486-491``) are restated as ``drone_contact``:
one contact per pair (every pair in contact, no cap) from the margin-shrunk cores' closest points
(FISTA-accelerated alternating projection from B's centre), solved with the same rows between two moving bodies before the plane solve.  Bit-level rounding of Bullet's own
operation order (the world <-> base round trips of the link forces, the 6x6 inverse of the
articulated inertia) is not reproduced either; the restatement is exact in exact arithmetic.

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
                   lin_damp=LIN_DAMP, ang_damp=ANG_DAMP, max_vel=MAX_COORD_VEL, cylinder=None):
    """One ``stepSimulation`` of a free base.

    ``f_base`` / ``t_base``: force and torque in the base frame (the link forces moved to the
    base COM); ``f_world``: world-frame base force (gravity).  ``cylinder`` = (radius,
    half_height, z_offset) of the collision cylinder turns on the ground-plane contact
    (``plane_contact``); None = free flight.  Returns the new (pos, q_s, vel_w, omega_w)."""
    q_wb, rot, vel_new, omega_new = multibody_velocity(pos, q_s, vel_w, omega_w, f_base, t_base, f_world, m,
                                                       inertia, dt, lin_damp, ang_damp, max_vel)
    return multibody_finish(pos, q_wb, rot, vel_new, omega_new, m, inertia, dt, cylinder)


def multibody_velocity(pos, q_s, vel_w, omega_w, f_base, t_base, f_world, m, inertia, dt,
                       lin_damp=LIN_DAMP, ang_damp=ANG_DAMP, max_vel=MAX_COORD_VEL):
    """The unconstrained half of ``multibody_step`` (solveExternalForces).  Returns (q_wb, rot,
    vel_new, omega_new) for ``multibody_finish``; envs of several drones run it for every drone,
    then ``drone_contact`` over the env, then ``multibody_finish`` per drone."""
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
    return q_wb, rot, vel_new, omega_new


def multibody_finish(pos, q_wb, rot, vel_new, omega_new, m, inertia, dt, cylinder=None):
    """The constrained half of ``multibody_step``: the ground-plane contact (solveConstraints)
    and integrateTransforms.  Returns the new (pos, q_s, vel_w, omega_w)."""
    if cylinder is not None:                                 # solveConstraints, before integrateTransforms
        vel_new, omega_new = plane_contact(pos, rot.T, vel_new, omega_new, m, inertia, dt, *cylinder)
    pos_new = np.asarray(pos, dtype=np.float64) + dt * vel_new
    q_s_new = qconj(base_quat_update(q_wb, omega_new, dt))
    return pos_new, q_s_new, vel_new, omega_new


# ---------------------------------------------------------------------------- ground-plane contact
# pybullet's world settings (PhysicsServerCommandProcessor::createEmptyDynamicsWorld) and Bullet3
# defaults the contact restatement uses; third-party values restated from Bullet3 knowledge
# (parity unpinned, see the module doc).
CONTACT_ERP = 0.08          # btContactSolverInfo::m_erp2 as pybullet sets it (contactERP)
LINEAR_SLOP = 1e-5          # m_linearSlop as pybullet sets it
SOLVER_ITERS = 50           # m_numIterations as pybullet sets it (numSolverIterations)
RESIDUAL_THRESHOLD = 1e-7   # m_leastSquaresResidualThreshold as pybullet sets it
FRICTION = 0.5 * 1.0        # combined friction = drone (btCollisionObject default 0.5, the URDFs
                            # carry no <contact>) x plane.urdf lateral_friction 1; restitution 0
URDF_MARGIN = 0.001         # gUrdfDefaultCollisionMargin (collision-shape margin of URDF shapes)
BREAKING_FACTOR = 0.02      # gContactBreakingThreshold, relative to the shape's angular-motion disc
PLANE_HALF = 15.0           # plane.urdf collision box 30 x 30 x 10 at z = -5: top face z = 0


def breaking_threshold(radius, half_height):
    """btCollisionDispatcher (CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD) takes the smaller of the
    two shapes' getContactBreakingThreshold(0.02) = 0.02 * getAngularMotionDisc(); the drone's
    cylinder is the smaller: disc = |AABB half extents| incl. margin, centred at the origin."""
    r, h = radius + URDF_MARGIN, half_height + URDF_MARGIN
    return BREAKING_FACTOR * math.sqrt(r * r + r * r + h * h)


def contact_points(radius, half_height, z_offset, rot_bw):
    """Body-frame contact candidates: the four rim points at body azimuth 0, 90, 180, 270 deg of
    the cap whose outward normal points down (btCylinderShapeZ's support rule: ``v.z < 0`` ->
    the -z cap, with v = R^T (0, 0, -1)).  Bullet's own manifold holds <= 4 points refreshed
    from GJK/EPA and its contact cache; this fixed four-point set is the restatement's
    deterministic stand-in for a resting / landing cylinder."""
    zc = -half_height if -rot_bw[2, 2] < 0.0 else half_height
    zc = zc + z_offset
    return [np.array([radius, 0.0, zc]), np.array([0.0, radius, zc]),
            np.array([-radius, 0.0, zc]), np.array([0.0, -radius, zc])]


def plane_contact(pos, rot_bw, vel_w, omega_w, m, inertia, dt, radius, half_height, z_offset):
    """Contact of the collision cylinder with the ground plane for one ``stepSimulation``.

    Follows btMultiBodyConstraintSolver for a free base against a static body:
    * contact geometry from the pose at the start of the step (collision detection runs before
      the solve), velocities after the unconstrained update (solveExternalForces);
    * a candidate point joins when its signed distance to the plane is below the breaking
      threshold and it lies over the plane box's top face;
    * rows per point: the normal (+z) and two friction directions (btPlaneSpace1(+z) =
      (0,-1,0), (1,0,0); SOLVER_USE_2_FRICTION_DIRECTIONS with the implicit friction cone);
      Jacobians in the base frame, M^-1 = diag(1/m, 1/I);
    * normal rhs: separated points (penetration = distance + slop > 0) are speculative,
      velocityError = -v_n - penetration/dt; penetrating points add the ERP position error
      -penetration * erp / dt; restitution 0, cfm 0; impulse >= 0;
    * friction rhs: -v_t; the pair (t1, t2) is projected onto the cone |lambda_t| <=
      mu * lambda_n, and solved only while the point's normal impulse is positive;
    * each iteration solves every normal row, then every friction pair; the solver stops when
      the largest squared row residual (normal: delta * jacDiag, friction pair: delta1 + delta2)
      is <= the threshold, or after the iteration cap;
    * no warm start (the restatement keeps no manifold between steps).
    Returns the new world (vel, omega)."""
    rot_bw = np.asarray(rot_bw, dtype=np.float64)
    pos = np.asarray(pos, dtype=np.float64)
    brk = breaking_threshold(radius, half_height)
    n_b = rot_bw[2, :].copy()                 # base-frame directions of world +z, (0,-1,0), (1,0,0)
    t1_b = -rot_bw[1, :]
    t2_b = rot_bw[0, :].copy()
    pts = []
    for r in contact_points(radius, half_height, z_offset, rot_bw):
        dist = pos[2] + n_b @ r
        wx = pos[0] + rot_bw[0, :] @ r
        wy = pos[1] + rot_bw[1, :] @ r
        if dist < brk and abs(wx) <= PLANE_HALF and abs(wy) <= PLANE_HALF:
            pts.append((r, dist))
    if not pts:
        return vel_w, omega_w
    inertia = np.asarray(inertia, dtype=np.float64)
    inv_m = 1.0 / m
    inv_i = 1.0 / inertia
    v_b = rot_bw.T @ np.asarray(vel_w, dtype=np.float64)
    w_b = rot_bw.T @ np.asarray(omega_w, dtype=np.float64)

    def row(r, d):
        a = np.array([r[1] * d[2] - r[2] * d[1], r[2] * d[0] - r[0] * d[2], r[0] * d[1] - r[1] * d[0]])
        jd = inv_m + ((a[0] * (a[0] * inv_i[0]) + a[1] * (a[1] * inv_i[1])) + a[2] * (a[2] * inv_i[2]))
        rel = ((d[0] * v_b[0] + d[1] * v_b[1]) + d[2] * v_b[2]) + ((a[0] * w_b[0] + a[1] * w_b[1]) + a[2] * w_b[2])
        return a, jd, 1.0 / jd, rel

    rows = []
    for r, dist in pts:
        a_n, jd_n, jdi_n, rel_n = row(r, n_b)
        pen = dist + LINEAR_SLOP
        if pen > 0:
            rhs_n = (-rel_n - pen / dt) * jdi_n
        else:
            rhs_n = (-pen * CONTACT_ERP / dt - rel_n) * jdi_n
        a_1, _, jdi_1, rel_1 = row(r, t1_b)
        a_2, _, jdi_2, rel_2 = row(r, t2_b)
        rows.append(dict(a=(a_n, a_1, a_2), jd_n=jd_n, jdi=(jdi_n, jdi_1, jdi_2),
                         rhs=(rhs_n, -rel_1 * jdi_1, -rel_2 * jdi_2), lam=[0.0, 0.0, 0.0]))
    dvl = np.zeros(3)
    dva = np.zeros(3)

    def jdv(d, a):
        return ((d[0] * dvl[0] + d[1] * dvl[1]) + d[2] * dvl[2]) + ((a[0] * dva[0] + a[1] * dva[1]) + a[2] * dva[2])

    def apply(d, a, delta):
        for j in range(3):
            dvl[j] = dvl[j] + d[j] * (inv_m * delta)
            dva[j] = dva[j] + (a[j] * inv_i[j]) * delta

    for _ in range(SOLVER_ITERS):
        res = 0.0
        for c in rows:                                        # normal rows
            delta = c["rhs"][0] - c["jdi"][0] * jdv(n_b, c["a"][0])
            s = c["lam"][0] + delta
            if s < 0.0:
                delta = -c["lam"][0]
                s = 0.0
            c["lam"][0] = s
            apply(n_b, c["a"][0], delta)
            res = max(res, (delta * c["jd_n"]) ** 2)
        for c in rows:                                        # friction pairs (implicit cone)
            ln = c["lam"][0]
            if not ln > 0.0:
                continue
            lim = FRICTION * ln
            d1 = c["rhs"][1] - c["jdi"][1] * jdv(t1_b, c["a"][1])
            d2 = c["rhs"][2] - c["jdi"][2] * jdv(t2_b, c["a"][2])
            s1 = c["lam"][1] + d1
            s2 = c["lam"][2] + d2
            m2 = s1 * s1 + s2 * s2
            if m2 > lim * lim:
                f = lim / math.sqrt(m2)
                s1 = s1 * f
                s2 = s2 * f
            d1 = s1 - c["lam"][1]
            d2 = s2 - c["lam"][2]
            c["lam"][1] = s1
            c["lam"][2] = s2
            apply(t1_b, c["a"][1], d1)
            apply(t2_b, c["a"][2], d2)
            res = max(res, (d1 + d2) ** 2)
        if res <= RESIDUAL_THRESHOLD:
            break
    return (np.asarray(vel_w, dtype=np.float64) + rot_bw @ dvl,
            np.asarray(omega_w, dtype=np.float64) + rot_bw @ dva)


# ---------------------------------------------------------------------------- drone <-> drone contact
# MultiHoverAviary's drones are colliding Bullet bodies (BaseAviary.py:486-491, stepped together
# by :369-370).  Bullet finds a cylinder pair's contact with GJK / EPA and keeps it in a persistent
# manifold; this restatement's own deterministic contact set (parity unpinned, like the plane's):
# one point per pair per step from the closest points of the two cylinders' margin-shrunk cores,
# found by a fixed number of FISTA-accelerated alternating-projection rounds from B's centre.
# (Continuing a pair from its previous substep's point, as Bullet's persistent manifold does with
# its points, was measured and rejected: on flat faces every point of the overlap is a fixed point
# of the projections, so the single contact point drifts with the bodies and tips a drone resting
# on another one over - DESIGN.md §2.3.)
FRICTION_DD = 0.5 * 0.5     # drone x drone combined friction (btCollisionObject default 0.5 each)
PAIR_COLD = 8               # accelerated alternating-projection rounds from B's centre
CORE_MARGINS = (0.001, 0.003, 0.006, 0.011)   # core shrink per level (the first = the URDF margin)
CORE_SEP = 1e-4             # core distance below which a level has no well-conditioned normal
SAT_SLACK = 1e-9            # the broadphase's separating-axis reject keeps this much against rounding
SIMDSQRT12 = 0.7071067811865475244008443621048490


def fista_momentum(k):
    """FISTA's momentum weights beta_0..beta_{k-1}: t_0 = 1, t_{i+1} = (1 + sqrt(1 + 4 t_i^2)) / 2,
    beta_i = (t_i - 1) / t_{i+1} (beta_0 = 0)."""
    out, t = [], 1.0
    for _ in range(k):
        tn = (1.0 + math.sqrt(1.0 + 4.0 * t * t)) / 2.0
        out.append((t - 1.0) / tn)
        t = tn
    return tuple(out)


PAIR_BETA = fista_momentum(PAIR_COLD)


def plane_space(n):
    """btPlaneSpace1: the two friction directions of a contact normal."""
    if abs(n[2]) > SIMDSQRT12:
        a = n[1] * n[1] + n[2] * n[2]
        k = 1.0 / math.sqrt(a)
        p = np.array([0.0, -n[2] * k, n[1] * k])
        q = np.array([a * k, -n[0] * p[2], n[0] * p[1]])
    else:
        a = n[0] * n[0] + n[1] * n[1]
        k = 1.0 / math.sqrt(a)
        p = np.array([-n[1] * k, n[0] * k, 0.0])
        q = np.array([-n[2] * p[1], n[2] * p[0], a * k])
    return p, q


def cyl_project(c, a, radius, half_height, x):
    """Closest point of the solid cylinder (centre c, unit axis a) to x."""
    d = x - c
    t = float(d @ a)
    tc = min(max(t, -half_height), half_height)
    rad = d - t * a
    rho2 = float(rad @ rad)
    if rho2 > radius * radius:
        rad = rad * (radius / math.sqrt(rho2))
    return c + tc * a + rad


def cyl_extent(u, a, radius, half_height):
    """Half-width of the cylinder (unit axis a) along the unit direction u."""
    ua = float(u @ a)
    return half_height * abs(ua) + radius * math.sqrt(max(0.0, 1.0 - ua * ua))


def pair_near(ci, ai, cj, aj, radius, half_height, brk):
    """Broadphase of the pair (i, j): bounding spheres within the breaking threshold, and no
    separating axis among the two cylinder axes and the centre line with a separation above it
    (+ SAT_SLACK).  Separation along any axis bounds the distance from below, so the reject
    never drops a pair whose distance is below the threshold."""
    bs = math.sqrt(radius * radius + half_height * half_height)
    reach = 2.0 * bs + brk
    e = ci - cj
    e2 = float(e @ e)
    if not e2 < reach * reach:
        return False
    lim = brk + SAT_SLACK
    ab = float(ai @ aj)
    tilt = half_height * abs(ab) + radius * math.sqrt(max(0.0, 1.0 - ab * ab))
    if abs(float(e @ ai)) - (half_height + tilt) > lim:
        return False
    if abs(float(e @ aj)) - (half_height + tilt) > lim:
        return False
    if e2 > 0.0:
        ln = math.sqrt(e2)
        ua, ub = float(e @ ai) / ln, float(e @ aj) / ln
        ext = cyl_extent_cos(ua, radius, half_height) + cyl_extent_cos(ub, radius, half_height)
        if ln - ext > lim:
            return False
    return True


def cyl_extent_cos(ua, radius, half_height):
    """cyl_extent for a direction whose cosine with the axis is ua."""
    return half_height * abs(ua) + radius * math.sqrt(max(0.0, 1.0 - ua * ua))


def pair_geometry(ca, aa, cb, ab, radius, half_height):
    """One contact of cylinders A and B: (normal on B pointing to A, point on B, distance;
    negative = penetration).  Bullet's margin scheme:
    the closest points of the CORE cylinders (radius and half-height shrunk by a margin m) give
    the normal and the distance core_distance - 2 m; the point on B's surface is B's core point +
    m n.  Core points by PAIR_COLD rounds of alternating projection in B-centred coordinates from
    B's centre with FISTA momentum (y' = P_B(P_A(z)), z = y' + beta (y' - y)) - a fixed count, no
    convergence test, so the result is a continuous function of the poses (16 plain rounds, round
    3's choice, left up to 2 mm of distance error on tilted face-to-face pairs where the plain
    rounds creep at cos^2 of the faces' angle; 8 accelerated ones reach the same accuracy, 16 ten
    times better) - then the point of A's core closest to B's.  A level whose cores come within CORE_SEP of each
    other (overlapping or nearly so: no well-conditioned normal) passes to the next, thicker
    margin (CORE_MARGINS: penetrations up to ~2 cm).  Deeper overlaps: the axis of least overlap
    among the centre line and the two cylinder axes, at the point the last level reached (Bullet
    runs EPA here)."""
    cl = ca - cb
    zero = np.zeros(3)
    y = zero
    for mg in CORE_MARGINS:
        r, h = radius - mg, half_height - mg
        y = zero.copy()
        z = zero.copy()
        for beta in PAIR_BETA:
            yn = cyl_project(zero, ab, r, h, cyl_project(cl, aa, r, h, z))
            z = yn + beta * (yn - y)
            y = yn
        pa = cyl_project(cl, aa, r, h, y)
        dv = pa - y
        d2 = float(dv @ dv)
        if d2 > CORE_SEP * CORE_SEP:
            dc = math.sqrt(d2)
            n = dv / dc
            return n, cb + (y + n * mg), dc - 2.0 * mg
    cands = []
    c2 = float(cl @ cl)
    if c2 > 1e-24:
        cands.append(cl / math.sqrt(c2))
    cands += [aa, ab]
    best, best_ov = None, None
    for u in cands:
        u = -u if float(u @ cl) < 0.0 else u
        ov = cyl_extent(u, aa, radius, half_height) + cyl_extent(u, ab, radius, half_height) - float(u @ cl)
        if best is None or ov < best_ov:
            best, best_ov = u, ov
    return best, cb + y, -best_ov


def drone_contacts(pos, rot_bw, radius, half_height, z_offset):
    """The env's contacts in solve order: pairs (i, j), i < j, lexicographic, that pass the
    broadphase (``pair_near``) and whose distance is below the breaking threshold - every such
    pair, however many (up to D (D - 1) / 2; round 3 kept at most D)."""
    D = pos.shape[0]
    brk = breaking_threshold(radius, half_height)
    axes = [rot_bw[i][:, 2].copy() for i in range(D)]
    cent = [pos[i] + axes[i] * z_offset for i in range(D)]
    out = []
    for i in range(D):
        for j in range(i + 1, D):
            if not pair_near(cent[i], axes[i], cent[j], axes[j], radius, half_height, brk):
                continue
            n, pb, dist = pair_geometry(cent[i], axes[i], cent[j], axes[j], radius, half_height)
            if dist < brk:
                out.append((i, j, n, pb, dist))
    return out


def drone_contact(pos, rot_bw, vel_w, omega_w, m, inertia, dt, radius, half_height, z_offset):
    """Drone <-> drone contact of one env for one ``stepSimulation``: the rows of
    ``plane_contact`` between two moving bodies, solved before it (between the unconstrained
    velocity update and the ground-plane solve).  Known deviation: Bullet solves the pair and
    plane rows of an island in one Gauss-Seidel loop; here the pair solve runs first and each
    drone's plane solve after it, so a drone resting on another that rests on the plane settles
    over substeps rather than within one solve (tests/test_oracle_drone_contact.py pins the
    stacked-on-the-plane case).

    ``pos`` [D, 3] start-of-step positions, ``rot_bw`` [D, 3, 3] body -> world, ``vel_w`` /
    ``omega_w`` [D, 3] after the unconstrained update.  Per contact (A = i, B = j, normal n from B
    to A, point on B ``pb``, point on A ``pb + n dist``): rows along n and btPlaneSpace1(n) with
    arms from each COM, effective mass 2/m + a_A.I_A^-1 a_A + a_B.I_B^-1 a_B (world inverse
    inertia R diag(1/I) R^T), the plane's rhs rules (speculative / ERP, slop) and friction cone
    (FRICTION_DD); Gauss-Seidel over the env's normal rows, then its friction pairs, in contact
    order, until the largest squared residual <= RESIDUAL_THRESHOLD or SOLVER_ITERS.  Returns
    the new (vel, omega) [D, 3]."""
    pos = np.asarray(pos, dtype=np.float64)
    vel = np.array(vel_w, dtype=np.float64)
    omg = np.array(omega_w, dtype=np.float64)
    cons = drone_contacts(pos, rot_bw, radius, half_height, z_offset)
    if not cons:
        return vel, omg
    D = pos.shape[0]
    im = 1.0 / m
    inv_i = 1.0 / np.asarray(inertia, dtype=np.float64)
    iw = [rot_bw[i] @ np.diag(inv_i) @ rot_bw[i].T for i in range(D)]
    rows = []
    for (i, j, n, pb, dist) in cons:
        pa = pb + n * dist
        ra, rb = pa - pos[i], pb - pos[j]
        t1, t2 = plane_space(n)
        row = dict(i=i, j=j, d=(n, t1, t2), aa=[], ab=[], ga=[], gb=[], jdi=[], rhs=[], lam=[0.0, 0.0, 0.0])
        for k, d in enumerate((n, t1, t2)):
            aa, ab = np.cross(ra, d), np.cross(rb, d)
            ga, gb = iw[i] @ aa, iw[j] @ ab
            jd = (2.0 * im + float(aa @ ga)) + float(ab @ gb)
            rel = float(d @ (vel[i] - vel[j])) + float(aa @ omg[i]) - float(ab @ omg[j])
            if k == 0:
                pen = dist + LINEAR_SLOP
                rhs = (-rel - pen / dt) / jd if pen > 0 else (-pen * CONTACT_ERP / dt - rel) / jd
                row["jdn"] = jd
            else:
                rhs = -rel / jd
            row["aa"].append(aa); row["ab"].append(ab); row["ga"].append(ga); row["gb"].append(gb)
            row["jdi"].append(1.0 / jd); row["rhs"].append(rhs)
        rows.append(row)
    dl = np.zeros((D, 3))
    da = np.zeros((D, 3))

    def jv(c, k):
        i, j = c["i"], c["j"]
        return float(c["d"][k] @ (dl[i] - dl[j])) + float(c["aa"][k] @ da[i]) - float(c["ab"][k] @ da[j])

    def apply(c, k, delta):
        i, j = c["i"], c["j"]
        dl[i] += c["d"][k] * (im * delta)
        da[i] += c["ga"][k] * delta
        dl[j] -= c["d"][k] * (im * delta)
        da[j] -= c["gb"][k] * delta

    for _ in range(SOLVER_ITERS):
        res = 0.0
        for c in rows:                                        # normal rows
            delta = c["rhs"][0] - c["jdi"][0] * jv(c, 0)
            s = c["lam"][0] + delta
            if s < 0.0:
                delta = -c["lam"][0]
                s = 0.0
            c["lam"][0] = s
            apply(c, 0, delta)
            res = max(res, (delta * c["jdn"]) ** 2)
        for c in rows:                                        # friction pairs (implicit cone)
            ln = c["lam"][0]
            if not ln > 0.0:
                continue
            lim = FRICTION_DD * ln
            s1 = c["lam"][1] + (c["rhs"][1] - c["jdi"][1] * jv(c, 1))
            s2 = c["lam"][2] + (c["rhs"][2] - c["jdi"][2] * jv(c, 2))
            m2 = s1 * s1 + s2 * s2
            if m2 > lim * lim:
                f = lim / math.sqrt(m2)
                s1 = s1 * f
                s2 = s2 * f
            d1 = s1 - c["lam"][1]
            d2 = s2 - c["lam"][2]
            c["lam"][1] = s1
            c["lam"][2] = s2
            apply(c, 1, d1)
            apply(c, 2, d2)
            res = max(res, (d1 + d2) ** 2)
        if res <= RESIDUAL_THRESHOLD:
            break
    touched = sorted({c["i"] for c in rows} | {c["j"] for c in rows})
    for i in touched:
        vel[i] = vel[i] + dl[i]
        omg[i] = omg[i] + da[i]
    return vel, omg
