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
one contact per pair (every pair in contact, no cap) from the margin-shrunk cores' converged closest
points, solved with the same rows between two moving bodies before the plane solve.  Bit-level rounding of Bullet's own
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
# test instrumentation: when a list, every drone <-> drone solve appends its iteration count
# (SOLVER_ITERS + 1 = stopped by the cap without reaching RESIDUAL_THRESHOLD)
SOLVE_LOG = None
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
# by :369-370).  Bullet finds a cylinder pair's contact with GJK / EPA (to a distance tolerance) and
# keeps it in a persistent manifold; this restatement's own deterministic contact set (parity
# unpinned, like the plane's): one point per pair per step, the CONVERGED closest points of the two
# cylinders' margin-shrunk cores (``core_pair``: every feature pair the closest points can lie on,
# each minimised to rounding - DESIGN.md §2.3).
# (Continuing a pair from its previous substep's point, as Bullet's persistent manifold does with
# its points, was measured and rejected in round 3: on flat faces every point of the overlap is a
# closest point, so the single contact point drifted with the bodies and tipped a drone resting on
# another one over - DESIGN.md §2.3.)
FRICTION_DD = 0.5 * 0.5     # drone x drone combined friction (btCollisionObject default 0.5 each)
CORE_MARGINS = (0.001, 0.003, 0.006, 0.011)   # core shrink per level (the first = the URDF margin)
CORE_SEP = 1e-4             # core distance below which a level has no well-conditioned normal
SAT_SLACK = 1e-9            # the broadphase's separating-axis reject keeps this much against rounding
SIMDSQRT12 = 0.7071067811865475244008443621048490
RIM_SAMPLES = 16            # the azimuth grid (k * 22.5 deg in btPlaneSpace1 of the axis): the first trust radius
RIM_STARTS = tuple(range(16))   # the Newton starts on it: every grid azimuth
RIM_ITERS = 5               # trust-region Newton steps from each start azimuth.  Round 6: 16 starts x 5
                            # steps (6 evaluations a chain) instead of 4 x 8 (9): on the GPU a pair's chains
                            # run side by side, one per lane, so a chain's length is the latency.  Against the
                            # certified exact distance: max 3.4e-6 m over 1 095 random near pairs (4 x 8:
                            # 2.0e-6; 8 x 5: 5.3e-5, 8 x 6: 1.4e-5), tests/test_oracle_drone_contact.py
RIM_ACCEPT = 1e-10          # a step must lower the squared distance by this fraction (rounding-proof)
RIM_SAME = 1e-4             # starts whose squared distances agree to this fraction count as one minimum (sized
                            # for the f32 kernel's rounding, so both precisions pick the same start)
PAIR_TIE = 1e-7             # candidates within this of the closest count as tied: the first wins (m); sized
                            # for the f32 kernel (a level side-by-side pair ties its lateral line and both rims)
# k * 22.5 deg: the first quadrant's (cos, sin) rotated by quarter turns, negations as 0 - x (no -0.0),
# exactly as gpd_kernels.h np_rim_task forms them
_C1, _S1 = 0.92387953251128674, 0.38268343236508978      # cos / sin 22.5 deg
_QC, _QS = (1.0, _C1, SIMDSQRT12, _S1), (0.0, _S1, SIMDSQRT12, _C1)
RIM_COS = tuple((_QC[q], 0.0 - _QS[q], 0.0 - _QC[q], _QS[q])[k] for k in range(4) for q in range(4))
RIM_SIN = tuple((_QS[q], _QC[q], 0.0 - _QS[q], 0.0 - _QC[q])[k] for k in range(4) for q in range(4))


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


def axial_project(x, r, h):
    """Closest point of the solid cylinder (centre 0, axis z, radius r, half-height h) to x."""
    rho2 = x[0] * x[0] + x[1] * x[1]
    f = r / math.sqrt(rho2) if rho2 > r * r else 1.0
    return np.array([x[0] * f, x[1] * f, min(max(x[2], -h), h)])


def _rim_eval(C, e1, e2, c, s, r, h):
    """Rim point P = C + r (c e1 + s e2) (c^2 + s^2 = 1) against the axial cylinder: the squared
    distance f, and with phi the rim angle, f'/2 = e.P' and f''/2 = ((I - J) P').P' + e.P'' (e = P -
    proj(P), J = the projection's Jacobian: the radial scaling (r/rho)(I - rr^T) in xy outside the
    radius, 0 in z beyond the caps)."""
    u = c * e1 + s * e2
    d1 = r * (c * e2 - s * e1)                       # P'
    P = C + r * u
    rho2 = P[0] * P[0] + P[1] * P[1]
    Q = axial_project(P, r, h)
    e = P - Q
    f = float(e @ e)
    g = float(e @ d1)
    m0 = m1 = m2 = 0.0
    if rho2 > r * r:
        rho = math.sqrt(rho2)
        k = r / rho
        rt = (P[0] * d1[0] + P[1] * d1[1]) / rho2
        m0 = d1[0] - k * (d1[0] - rt * P[0])
        m1 = d1[1] - k * (d1[1] - rt * P[1])
    if abs(P[2]) > h:
        m2 = d1[2]
    hh = (m0 * d1[0] + m1 * d1[1] + m2 * d1[2]) - r * float(e @ u)    # P'' = -r u
    return f, g, hh, P, Q


def rim_newton(C, e1, e2, r, h, c, s):
    """RIM_ITERS trust-region Newton steps on the rim angle from the rim point (c, s): tangent step
    c' = c - d s, s' = s + d c, renormalised, d = -f'/f'' clamped to the radius (-radius . sign(f')
    where f'' <= 0); a step is kept only when it lowers the squared distance by the fraction
    RIM_ACCEPT - rounding noise never moves the point - and the radius doubles, up to 1 rad, else
    it shrinks to |d| / 4.  Returns (f, P, Q)."""
    f, g, hh, P, Q = _rim_eval(C, e1, e2, c, s, r, h)
    rad = math.pi / RIM_SAMPLES
    for _ in range(RIM_ITERS):
        d = -g / hh if hh > 0.0 else -math.copysign(rad, g)
        d = min(max(d, -rad), rad)
        c2, s2 = c - d * s, s + d * c
        k = 1.0 / math.sqrt(c2 * c2 + s2 * s2)
        c2, s2 = c2 * k, s2 * k
        f2, g2, hh2, P2, Q2 = _rim_eval(C, e1, e2, c2, s2, r, h)
        if f2 < f * (1.0 - RIM_ACCEPT):
            c, s, f, g, hh, P, Q = c2, s2, f2, g2, hh2, P2, Q2
            rad = min(2.0 * rad, 1.0)
        else:
            rad = abs(d) * 0.25
    return f, P, Q


def rim_closest(C, e1, e2, r, h):
    """The point of the rim circle (centre C, orthonormal in-plane basis e1, e2, radius r) closest to
    the axial cylinder (centre 0, axis z, radius r, half-height h), and that cylinder's point.
    The rim's distance is not convex in the angle (two local minima on nearly parallel stacked
    faces, a kink where the rim point crosses the other cylinder's edge), so Newton runs from each of
    the RIM_STARTS azimuths (rim_newton) and the lowest start whose squared distance is within the
    relative RIM_SAME of the smallest wins: chains that reached one minimum agree on f to rounding
    but on the point only to ~sqrt(RIM_ACCEPT) (a flat minimum), so a plain argmin would pick its
    chain by rounding noise.  On the GPU the 4 x 16 starts of a pair run on 64 lanes at once."""
    out = [rim_newton(C, e1, e2, r, h, RIM_COS[k], RIM_SIN[k]) for k in RIM_STARTS]
    fmin = min(o[0] for o in out)
    k = next(i for i, o in enumerate(out) if o[0] <= fmin * (1.0 + RIM_SAME))
    return out[k][1], out[k][2]


def segment_closest(L, A, h):
    """Closest points of the axis segments L + s A and t z, s, t in [-h, h] (A, z unit)."""
    b = float(A[2])
    dd = float(A @ L)
    e = float(L[2])
    den = 1.0 - b * b
    s = (b * e - dd) / den if den > 1e-12 else 0.0
    s = min(max(s, -h), h)
    t = min(max(b * s + e, -h), h)
    s = min(max(b * t - dd, -h), h)
    return L + s * A, np.array([0.0, 0.0, t])


def axial_extent(az, r, h):
    """Half-width along a unit direction of the axial cylinder (axis z), az the direction's z."""
    return h * abs(az) + r * math.sqrt(max(0.0, 1.0 - az * az))


def core_pair(L, A, r, h):
    """Closest points (x on A, y on B) of two solid cylinders of radius r and half-height h in B's
    frame: B centred at 0 with axis z, A centred at L with unit axis A.  The closest points of two
    separated cylinders lie on a rim of one of them (against any feature of the other), or on both
    lateral surfaces (the axes' closest points interior); every other feature pair (face-face,
    face-lateral) shares its distance with a rim point.  So the distance is the smallest of:
      0/1. the near caps' centres against the other cylinder (level stacks: the centred point);
      2.   the lateral surfaces along the axes' closest points (closed form; level side-by-side
           pairs: the point at mid-height);
      3/4. the rims of the caps facing the other cylinder, against it (rim_closest; B's rim in A's
           frame, btPlaneSpace1 of A);
      5/6. the far caps' rims;
    each candidate a feasible pair (an upper bound); the first, in that order, within PAIR_TIE of the
    closest is taken.  When the other cylinder lies wholly beyond a near cap's plane
    (its extent along the cap normal), that cylinder's far rim and lateral surface are farther than
    its near rim point by point, and candidates 2 and 5 (A) / 6 (B) are skipped - the stacked case.
    Accuracy against the certified exact distance (tests/tools/np_exact.py): <= 3e-6 m on random,
    side-by-side, rim-to-rim, stacked and flat pairs (tests/test_oracle_drone_contact.py).
    Overlapping cores give a distance <= CORE_SEP (a rim or a cap centre inside the other core)."""
    ap, aq = plane_space(A)
    Ma = np.stack([ap, aq, A])                        # B's frame -> A's frame
    Lb = Ma @ (-L)                                    # B's centre and axis in A's frame
    Bz = Ma[:, 2].copy()
    bp, bq = plane_space(Bz)
    la = float(L @ A)
    sa = -1.0 if la > 0.0 else 1.0                    # A's cap facing B
    sb = 1.0 if L[2] >= 0.0 else -1.0                 # B's cap facing A
    # B wholly beyond A's near cap plane / A wholly beyond B's
    far_a = -sa * la - h < axial_extent(sa * A[2], r, h)
    far_b = sb * L[2] - h < axial_extent(A[2], r, h)
    xa = L + sa * h * A
    cands = [(xa, axial_project(xa, r, h))]
    yb = Lb + sb * h * Bz                             # in A's frame
    cands.append((Ma.T @ axial_project(yb, r, h) + L, Ma.T @ yb + L))
    if far_a and far_b:
        pa, pb = segment_closest(L, A, h)
        w = pa - pb
        wn = math.sqrt(float(w @ w))
        if wn > 1e-12:
            u = w / wn
            cands.append((cyl_project(L, A, r, h, pa - r * u), axial_project(pb + r * u, r, h)))
    for sg, sgb, ok_a, ok_b in ((sa, sb, True, True), (-sa, -sb, far_a, far_b)):
        if ok_a:
            cands.append(rim_closest(L + sg * h * A, ap, aq, r, h))
        if ok_b:
            yb, xa_ = rim_closest(Lb + sgb * h * Bz, bp, bq, r, h)
            cands.append((Ma.T @ xa_ + L, Ma.T @ yb + L))
    ds = [math.sqrt(float((x - y) @ (x - y))) for x, y in cands]
    lim = min(ds) + PAIR_TIE
    k = next(i for i, d in enumerate(ds) if d <= lim)      # the first candidate within the tie of the closest
    return cands[k][0], cands[k][1], ds[k]


def pair_geometry(ca, aa, cb, ab, radius, half_height, with_margin=False):
    """One contact of cylinders A and B: (normal on B pointing to A, point on B, distance;
    negative = penetration).  Bullet's margin scheme: the closest points of the CORE cylinders
    (radius and half-height shrunk by a margin m) give the normal and the distance core_distance -
    2 m; the point on B's surface is B's core point + m n.  Core points by ``core_pair`` in B's frame
    (btPlaneSpace1(aB), aB), converged to rounding.  A level whose cores come within CORE_SEP of each
    other (overlapping or nearly so: no well-conditioned normal) passes to the next, thicker margin
    (CORE_MARGINS: penetrations up to ~2 cm).  Deeper overlaps: the axis of least overlap among the
    centre line and the two cylinder axes, at the point the last level reached (Bullet runs EPA
    here).  ``with_margin``: also return the margin of the level that gave the contact (None for the
    least-overlap fallback)."""
    bp, bq = plane_space(ab)
    Mb = np.stack([bp, bq, ab])                       # world -> B's frame
    cl = ca - cb
    L = Mb @ cl
    A = Mb @ aa
    y = np.zeros(3)
    for mg in CORE_MARGINS:
        x, y, dc = core_pair(L, A, radius - mg, half_height - mg)
        if dc > CORE_SEP:
            n = Mb.T @ ((x - y) / dc)
            out = (n, cb + (Mb.T @ y + n * mg), dc - 2.0 * mg)
            return out + (mg,) if with_margin else out
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
    out = (best, cb + Mb.T @ y, -best_ov)
    return out + (None,) if with_margin else out


FACE_COS = SIMDSQRT12       # both near caps' normals within 45 deg of the contact normal: a face contact


def face_points(ca, aa, cb, ab, n, radius, half_height, mg):
    """The face manifold of a cap-to-cap contact: four points spanning the overlap of the two near
    caps, as (point on B, distance) - a deterministic stand-in for the up-to-4-point persistent
    manifold Bullet builds over frames (btPersistentManifold, MANIFOLD_CACHE_SIZE 4) for two
    resting faces, as ``contact_points`` is for the plane.  With one point per pair (the exact
    closest point, at a rim as soon as the faces tilt) a drone resting on another rocks from rim
    to rim and sinks ~6 mm into it (tests/test_oracle_drone_contact.py).
    A face contact: the cores' caps facing each other (A's cap nearer B, outward normal nu_A =
    +-a_A, and B's, nu_B) with n.nu_B >= FACE_COS and -n.nu_A >= FACE_COS.  In the plane normal to
    n the two cap discs (radius r of the core at margin mg) overlap in a lens; its four extreme
    points: the two tips on the line of the cap centres (from B's centre cB: (s - r) u and r u, u
    the unit centre offset, s its length; u = btPlaneSpace1(n)'s first direction for coaxial caps)
    and the two corners (s/2) u +- sqrt(r^2 - s^2/4) (n x u).  Each point p is carried along n to
    B's cap plane (y) and to A's (x); its distance is (x - y).n - 2 mg and its point on B y + mg n.
    No points when the caps do not overlap (s >= 2 r)."""
    r, h = radius - mg, half_height - mg
    sa = 1.0 if float((cb - ca) @ aa) >= 0.0 else -1.0
    sb = 1.0 if float((ca - cb) @ ab) >= 0.0 else -1.0
    cA, nuA = ca + sa * h * aa, sa * aa
    cB, nuB = cb + sb * h * ab, sb * ab
    nb, na = float(n @ nuB), -float(n @ nuA)
    if not (nb >= FACE_COS and na >= FACE_COS):
        return []
    c_ab = cA - cB
    dl = c_ab - float(c_ab @ n) * n                    # the centre offset in the plane normal to n
    s2 = float(dl @ dl)
    if not s2 < 4.0 * r * r:
        return []
    s = math.sqrt(s2)
    u = dl / s if s > 1e-9 else plane_space(n)[0]
    v = np.cross(n, u)
    w = math.sqrt(max(r * r - 0.25 * s2, 0.0))
    out = []
    for p in ((s - r) * u, r * u, (0.5 * s) * u + w * v, (0.5 * s) * u - w * v):
        tb = -float(p @ nuB) / nb                      # along n from cB + p to B's cap plane
        ta = float((c_ab - p) @ nuA) / -na             # ... to A's cap plane ((cA - cB - p).nuA / n.nuA)
        out.append((cB + p + (tb + mg) * n, (ta - tb) - 2.0 * mg))
    return out


MANIFOLD_CACHE_SIZE = 4     # btPersistentManifold's point capacity
MANIFOLD_DEPTH_TIE = 1e-6   # a cached point counts as deeper than the new one only beyond this (m)
MANIFOLD_AREA_TIE = 1e-4    # areas within this fraction of the largest count as tied: the first wins


def manifold_replace(new_a, new_d, cache):
    """btPersistentManifold::sortCachedPoints: the cache slot a new point replaces when the cache
    is full.  ``new_a``: the new point on A, ``new_d`` its distance; ``cache``: 4 (point on A,
    distance).  The deepest point (KEEP_DEEPEST_POINT: a cached point deeper than the new one) is
    never replaced; for every other slot the "area" |(new - c_a) x (c_b - c_c)|^2 of the quad with
    that slot replaced (Bullet's pairing of the cached points), and the slot of the largest wins
    (btVector4::closestAxis4: the first maximum).  The two comparisons carry ties
    (MANIFOLD_DEPTH_TIE, MANIFOLD_AREA_TIE): a symmetric manifold (a level stack: every point at the
    same distance, two equal areas) must not be decided by rounding, so the GPU's f64 and f32
    builds take the same slot as this restatement."""
    maxpen, imax = new_d, -1
    for i, (_, d) in enumerate(cache):
        if d < maxpen - MANIFOLD_DEPTH_TIE:
            maxpen, imax = d, i
    c = [np.asarray(a, dtype=np.float64) for a, _ in cache]
    pairs = ((1, 3, 2), (0, 3, 2), (0, 3, 1), (0, 2, 1))     # res_k = |(new - c_a) x (c_b - c_c)|^2
    res = []
    for k, (a, b, cc) in enumerate(pairs):
        if k == imax:
            res.append(0.0)
            continue
        x = np.cross(new_a - c[a], c[b] - c[cc])
        res.append(float(x @ x))
    top = max(res)
    return next(k for k, v in enumerate(res) if v >= top * (1.0 - MANIFOLD_AREA_TIE))


def pair_manifold(pb, dist, n, face):
    """A contact pair's points, at most MANIFOLD_CACHE_SIZE like Bullet's manifold: the closest
    point (pb, dist) and the face points ``face`` (already below the breaking threshold).  With
    four face points the closest point takes the slot ``manifold_replace`` picks (Bullet adding a
    point to a full cache); with fewer, the closest point comes first and the face points follow.
    Round 5 kept all five: the closest point of a level stack is the cap centre, inside the lens the
    face points span, so every face contact had five nearly dependent normal rows - one more than
    Bullet can hold - and where Gauss-Seidel stopped depended on rounding."""
    if len(face) < MANIFOLD_CACHE_SIZE:
        return [(pb, dist)] + list(face)
    k = manifold_replace(pb + n * dist, dist, [(p + n * d, d) for p, d in face])
    out = list(face)
    out[k] = (pb, dist)
    return out


def drone_contacts(pos, rot_bw, radius, half_height, z_offset):
    """The env's contacts in solve order: pairs (i, j), i < j, lexicographic, that pass the
    broadphase (``pair_near``) and whose distance is below the breaking threshold - every such
    pair, however many (up to D (D - 1) / 2; round 3 kept at most D).  Per pair: the closest
    points (``pair_geometry``) and, for a cap-to-cap contact, its face manifold (``face_points``)
    points below the breaking threshold - at most four points per pair (``pair_manifold``) - as
    contacts of the same pair (i, j, n, pb, dist)."""
    D = pos.shape[0]
    brk = breaking_threshold(radius, half_height)
    axes = [rot_bw[i][:, 2].copy() for i in range(D)]
    cent = [pos[i] + axes[i] * z_offset for i in range(D)]
    out = []
    for i in range(D):
        for j in range(i + 1, D):
            if not pair_near(cent[i], axes[i], cent[j], axes[j], radius, half_height, brk):
                continue
            n, pb, dist, mg = pair_geometry(cent[i], axes[i], cent[j], axes[j], radius, half_height, with_margin=True)
            if dist < brk:
                face = [] if mg is None else \
                    [(p, d) for p, d in face_points(cent[i], axes[i], cent[j], axes[j], n, radius, half_height, mg)
                     if d < brk]
                for p, d in pair_manifold(pb, dist, n, face):
                    out.append((i, j, n, p, d))
    return out


def _plane_rows_world(pos, rot_bw, vel, omg, im, iw, dt, radius, half_height, z_offset):
    """``plane_contact``'s rows of one drone in world coordinates (directions +z, (0,-1,0), (1,0,0);
    arms R r; angular Jacobians r x d; I_w^-1 = R diag(1/I) R^T): the same rows as its base-frame
    form up to rounding, for an island solve that also holds pair rows."""
    brk = breaking_threshold(radius, half_height)
    dirs = (np.array([0.0, 0.0, 1.0]), np.array([0.0, -1.0, 0.0]), np.array([1.0, 0.0, 0.0]))
    rows = []
    for r in contact_points(radius, half_height, z_offset, rot_bw):
        rw = rot_bw @ r
        dist = pos[2] + rw[2]
        if not (dist < brk and abs(pos[0] + rw[0]) <= PLANE_HALF and abs(pos[1] + rw[1]) <= PLANE_HALF):
            continue
        row = dict(a=[], g=[], jdi=[], rhs=[], lam=[0.0, 0.0, 0.0])
        for k, d in enumerate(dirs):
            a = np.cross(rw, d)
            g = iw @ a
            jd = im + float(a @ g)
            rel = float(d @ vel) + float(a @ omg)
            if k == 0:
                pen = dist + LINEAR_SLOP
                rhs = (-rel - pen / dt) / jd if pen > 0 else (-pen * CONTACT_ERP / dt - rel) / jd
                row["jdn"] = jd
            else:
                rhs = -rel / jd
            row["a"].append(a); row["g"].append(g); row["jdi"].append(1.0 / jd); row["rhs"].append(rhs)
        rows.append(row)
    return rows


def drone_contact(pos, rot_bw, vel_w, omega_w, m, inertia, dt, radius, half_height, z_offset, plane=False):
    """Drone <-> drone contact of one env for one ``stepSimulation`` (between the unconstrained
    velocity update and the position update).

    ``pos`` [D, 3] start-of-step positions, ``rot_bw`` [D, 3, 3] body -> world, ``vel_w`` /
    ``omega_w`` [D, 3] after the unconstrained update.  Per contact (A = i, B = j, normal n from B
    to A, point on B ``pb``, point on A ``pb + n dist``): rows along n and btPlaneSpace1(n) with
    arms from each COM, effective mass 2/m + a_A.I_A^-1 a_A + a_B.I_B^-1 a_B (world inverse
    inertia R diag(1/I) R^T), the plane's rhs rules (speculative / ERP, slop) and friction cone
    (FRICTION_DD).

    ``plane=True`` (the ground plane is on): the island solve.  Bullet solves the rows of all
    bodies an island's contacts connect in one Gauss-Seidel loop; here every drone that is in a
    pair contact AND touches the plane (``plane_contact``'s points) brings its plane rows into the
    env's loop, and its own plane solve is skipped (the caller uses the returned set).  Per
    iteration: the plane normal rows of those drones (drone order, point order), the pair normal
    rows (contact order), the plane friction pairs, the pair friction pairs; the env stops at its
    largest squared residual <= RESIDUAL_THRESHOLD or after SOLVER_ITERS (the env's islands share
    the stopping rule).  Round 4; before it the pair solve ran first and each drone's plane solve
    after it, so a drone resting on another that rests on the plane sank ~1 cm into it.
    ``plane=False``: pair rows only.  Returns (vel, omega) [D, 3], and with ``plane=True`` also the
    set of drones whose plane rows were solved here."""
    pos = np.asarray(pos, dtype=np.float64)
    vel = np.array(vel_w, dtype=np.float64)
    omg = np.array(omega_w, dtype=np.float64)
    cons = drone_contacts(pos, rot_bw, radius, half_height, z_offset)
    if not cons:
        return (vel, omg, set()) if plane else (vel, omg)
    D = pos.shape[0]
    im = 1.0 / m
    inv_i = 1.0 / np.asarray(inertia, dtype=np.float64)
    iw = [rot_bw[i] @ np.diag(inv_i) @ rot_bw[i].T for i in range(D)]
    touched = sorted({c[0] for c in cons} | {c[1] for c in cons})
    prows = {}
    if plane:
        for i in touched:
            r = _plane_rows_world(pos[i], rot_bw[i], vel[i], omg[i], im, iw[i], dt, radius, half_height, z_offset)
            if r:
                prows[i] = r
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
    pdirs = (np.array([0.0, 0.0, 1.0]), np.array([0.0, -1.0, 0.0]), np.array([1.0, 0.0, 0.0]))

    def jv(c, k):
        i, j = c["i"], c["j"]
        return float(c["d"][k] @ (dl[i] - dl[j])) + float(c["aa"][k] @ da[i]) - float(c["ab"][k] @ da[j])

    def apply(c, k, delta):
        i, j = c["i"], c["j"]
        dl[i] += c["d"][k] * (im * delta)
        da[i] += c["ga"][k] * delta
        dl[j] -= c["d"][k] * (im * delta)
        da[j] -= c["gb"][k] * delta

    def pjv(i, c, k):
        return float(pdirs[k] @ dl[i]) + float(c["a"][k] @ da[i])

    def papply(i, c, k, delta):
        dl[i] += pdirs[k] * (im * delta)
        da[i] += c["g"][k] * delta

    def cone(s1, s2, lim):
        m2 = s1 * s1 + s2 * s2
        if m2 > lim * lim:
            f = lim / math.sqrt(m2)
            return s1 * f, s2 * f
        return s1, s2

    used = SOLVER_ITERS + 1
    for it in range(SOLVER_ITERS):
        res = 0.0
        for i, pr in prows.items():                           # plane normal rows
            for c in pr:
                delta = c["rhs"][0] - c["jdi"][0] * pjv(i, c, 0)
                s_ = c["lam"][0] + delta
                if s_ < 0.0:
                    delta = -c["lam"][0]
                    s_ = 0.0
                c["lam"][0] = s_
                papply(i, c, 0, delta)
                res = max(res, (delta * c["jdn"]) ** 2)
        for c in rows:                                        # pair normal rows
            delta = c["rhs"][0] - c["jdi"][0] * jv(c, 0)
            s_ = c["lam"][0] + delta
            if s_ < 0.0:
                delta = -c["lam"][0]
                s_ = 0.0
            c["lam"][0] = s_
            apply(c, 0, delta)
            res = max(res, (delta * c["jdn"]) ** 2)
        for i, pr in prows.items():                           # plane friction pairs
            for c in pr:
                ln = c["lam"][0]
                if not ln > 0.0:
                    continue
                s1 = c["lam"][1] + (c["rhs"][1] - c["jdi"][1] * pjv(i, c, 1))
                s2 = c["lam"][2] + (c["rhs"][2] - c["jdi"][2] * pjv(i, c, 2))
                s1, s2 = cone(s1, s2, FRICTION * ln)
                d1 = s1 - c["lam"][1]
                d2 = s2 - c["lam"][2]
                c["lam"][1] = s1
                c["lam"][2] = s2
                papply(i, c, 1, d1)
                papply(i, c, 2, d2)
                res = max(res, (d1 + d2) ** 2)
        for c in rows:                                        # pair friction pairs (implicit cone)
            ln = c["lam"][0]
            if not ln > 0.0:
                continue
            s1 = c["lam"][1] + (c["rhs"][1] - c["jdi"][1] * jv(c, 1))
            s2 = c["lam"][2] + (c["rhs"][2] - c["jdi"][2] * jv(c, 2))
            s1, s2 = cone(s1, s2, FRICTION_DD * ln)
            d1 = s1 - c["lam"][1]
            d2 = s2 - c["lam"][2]
            c["lam"][1] = s1
            c["lam"][2] = s2
            apply(c, 1, d1)
            apply(c, 2, d2)
            res = max(res, (d1 + d2) ** 2)
        if res <= RESIDUAL_THRESHOLD:
            used = it + 1
            break
    if SOLVE_LOG is not None:
        SOLVE_LOG.append(used)
    for i in touched:
        vel[i] = vel[i] + dl[i]
        omg[i] = omg[i] + da[i]
    return (vel, omg, set(prows)) if plane else (vel, omg)
