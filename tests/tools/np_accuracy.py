"""Accuracy of the drone-contact narrowphase (oracle/bullet_mb.py pair_geometry's FISTA-accelerated
alternating projection) against the exact closest points of the cores (4 000 plain rounds), on random
near-contact pairs and on stacked, nearly parallel discs - the study behind DESIGN.md §2.3 / §11
(test infrastructure: numpy, the oracle's constants).  Usage: python tests/tools/np_accuracy.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.bullet_mb import CORE_MARGINS, fista_momentum  # noqa: E402

R, H = 0.06, 0.0125   # cf2x.urdf collision cylinder


def proj(c, a, r, h, x):
    d = x - c
    t = np.sum(d * a, 1, keepdims=True)
    tc = np.clip(t, -h, h)
    rad = d - t * a
    rho2 = np.sum(rad * rad, 1, keepdims=True)
    f = np.where(rho2 > r * r, r / np.sqrt(np.maximum(rho2, 1e-300)), 1.0)
    return c + tc * a + rad * f


def study(name, cl, aa, ab, k_list=(4, 6, 8)):
    mg = CORE_MARGINS[0]
    r, h = R - mg, H - mg
    n = cl.shape[0]
    zero = np.zeros((n, 3))
    y = zero.copy()
    for _ in range(4000):
        y = proj(zero, ab, r, h, proj(cl, aa, r, h, y))
    dex = np.linalg.norm(proj(cl, aa, r, h, y) - y, axis=1)
    ok = dex > 1e-4
    for k in k_list:
        y = zero.copy()
        z = zero.copy()
        for b in fista_momentum(k):
            yn = proj(zero, ab, r, h, proj(cl, aa, r, h, z))
            z = yn + b * (yn - y)
            y = yn
        e = (np.linalg.norm(proj(cl, aa, r, h, y) - y, axis=1) - dex)[ok]
        print(f"{name}: {ok.sum()} separated pairs, {k} rounds: distance error p50 {np.percentile(e, 50):.1e} "
              f"p90 {np.percentile(e, 90):.1e} p99 {np.percentile(e, 99):.1e} max {e.max():.1e} m", flush=True)


def main():
    rng = np.random.default_rng(0)
    n = 20000

    def tilted(m, deg):
        t = np.radians(rng.random(m) * deg)
        ph = rng.random(m) * 2 * np.pi
        return np.stack([np.sin(t) * np.cos(ph), np.sin(t) * np.sin(ph), np.cos(t)], 1)
    # random near-contact pairs (half near-upright, half any axis)
    aa, ab = tilted(n, 20), tilted(n, 20)
    aa[: n // 2] = rng.normal(size=(n // 2, 3))
    aa[: n // 2] /= np.linalg.norm(aa[: n // 2], axis=1, keepdims=True)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    ext = lambda v, a: H * np.abs(np.sum(v * a, 1)) + R * np.sqrt(np.maximum(0, 1 - np.sum(v * a, 1) ** 2))
    cl = u * (ext(u, aa) + ext(u, ab) + rng.uniform(-0.006, 0.004, n))[:, None]
    study("random pairs", cl, aa, ab)
    # stacked discs: A above B, small lateral offsets, nearly parallel axes
    aa, ab = tilted(n, 10), tilted(n, 10)
    cl = np.stack([rng.uniform(-0.06, 0.06, n), rng.uniform(-0.06, 0.06, n), 2 * H + rng.uniform(-0.002, 0.004, n)], 1)
    study("stacked discs", cl, aa, ab)


if __name__ == "__main__":
    main()
