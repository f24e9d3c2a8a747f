"""Certified exact distance of two solid cylinders (test infrastructure: numpy + scipy).

The drone <-> drone narrowphase (oracle/bullet_mb.py pair_geometry) is checked against the cores'
exact closest points.  Alternating projection is not a usable reference: on nearly parallel faces
it creeps by (local gap x tilt) per round, so even 4 000 rounds leave millimetres on discs tilted by
~0.01 rad.  This module brackets the distance from both sides instead:
  * upper bound: SLSQP on min |x - y|^2 over x in A, y in B (a convex QCQP), started from the
    product's own pair and from alternating projection; any feasible pair bounds the distance from
    above;
  * lower bound: the separation along a direction u, u.(cA - cB) - ext_A(u) - ext_B(u), maximised
    over the unit sphere (Nelder-Mead in the tangent plane of the primal normal); any u bounds the
    distance from below (separating-axis theorem).
A pair is certified when the two bounds agree to `tol`.  Usage: ``exact_distance(...)``."""
import math

import numpy as np
from scipy.optimize import minimize


def _proj(c, a, r, h, x):
    d = x - c
    t = float(d @ a)
    tc = min(max(t, -h), h)
    rad = d - t * a
    rho2 = float(rad @ rad)
    if rho2 > r * r:
        rad = rad * (r / math.sqrt(rho2))
    return c + tc * a + rad


def extent(u, a, r, h):
    ua = float(u @ a)
    return h * abs(ua) + r * math.sqrt(max(0.0, 1.0 - ua * ua))


def separation(u, cl, aa, ab, r, h):
    """Lower bound on the distance of A (centre cl, axis aa) and B (centre 0, axis ab) along the unit u."""
    return float(u @ cl) - extent(u, aa, r, h) - extent(u, ab, r, h)


def exact_distance(cl, aa, ab, r, h, starts=(), tol=1e-9):
    """(upper, lower) bounds of the distance of cylinders A (centre cl, unit axis aa) and B (centre 0,
    unit axis ab), both of radius r and half-height h.  `starts`: extra (x, y) feasible pairs."""
    cl = np.asarray(cl, float)
    aa = np.asarray(aa, float)
    ab = np.asarray(ab, float)
    zero = np.zeros(3)
    y = zero
    for _ in range(200):
        y = _proj(zero, ab, r, h, _proj(cl, aa, r, h, y))
    cand = [(_proj(cl, aa, r, h, y), y)] + [(np.asarray(x, float), np.asarray(yy, float)) for x, yy in starts]

    def f(z):
        d = z[:3] - z[3:]
        return float(d @ d), 2 * np.concatenate([d, -d])

    def cons():
        out = []
        for c, a, sl in ((cl, aa, slice(0, 3)), (zero, ab, slice(3, 6))):
            def ax_lo(z, c=c, a=a, sl=sl):
                return float((z[sl] - c) @ a) + h

            def ax_hi(z, c=c, a=a, sl=sl):
                return h - float((z[sl] - c) @ a)

            def rad(z, c=c, a=a, sl=sl):
                d = z[sl] - c
                p = d - float(d @ a) * a
                return r * r - float(p @ p)
            out += [dict(type="ineq", fun=ax_lo), dict(type="ineq", fun=ax_hi), dict(type="ineq", fun=rad)]
        return out
    cs = cons()
    best_up, best_n = math.inf, None
    for x0, y0 in cand:
        up0 = float(np.linalg.norm(x0 - y0))
        if up0 < best_up:
            best_up, best_n = up0, (x0 - y0)
        res = minimize(f, np.concatenate([x0, y0]), jac=True, constraints=cs, method="SLSQP",
                       options=dict(ftol=1e-24, maxiter=400))
        z = res.x
        # snap to feasibility (SLSQP may sit 1e-12 outside), then the pair is a true upper bound
        xs, ys = _proj(cl, aa, r, h, z[:3]), _proj(zero, ab, r, h, z[3:])
        up = float(np.linalg.norm(xs - ys))
        if up < best_up:
            best_up, best_n = up, xs - ys
    if best_up < 1e-12:
        return best_up, -math.inf                     # overlapping: no separating direction
    n = best_n / np.linalg.norm(best_n)
    # directions around n: u = normalise(n + p e1 + q e2), e1, e2 orthonormal to n (no pole)
    e1 = np.cross(n, [1.0, 0.0, 0.0] if abs(n[0]) < 0.6 else [0.0, 1.0, 0.0])
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(n, e1)

    def u_of(p):
        u = n + p[0] * e1 + p[1] * e2
        return u / np.linalg.norm(u)
    low = separation(n, cl, aa, ab, r, h)
    p0 = np.zeros(2)
    for scale in (1e-2, 1e-4, 1e-6, 1e-8):
        res = minimize(lambda p: -separation(u_of(p), cl, aa, ab, r, h), p0, method="Nelder-Mead",
                       options=dict(xatol=scale * 1e-3, fatol=1e-17,
                                    initial_simplex=[p0, p0 + [scale, 0.0], p0 + [0.0, scale]]))
        if -res.fun > low:
            low = -res.fun
            p0 = res.x
    return best_up, low
