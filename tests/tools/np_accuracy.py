"""Accuracy of the drone-contact narrowphase (oracle/bullet_mb.py core_pair) against the certified
exact distance of the cores (tests/tools/np_exact.py: SLSQP upper bound, separating-axis lower bound),
on five sets of near-contact pairs - the study behind DESIGN.md §2.3 (test infrastructure: numpy,
scipy, the oracle's constants).  Usage: python tests/tools/np_accuracy.py [pairs per set] [seed]"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.bullet_mb import CORE_MARGINS, core_pair, plane_space  # noqa: E402
from tests.tools.np_exact import exact_distance  # noqa: E402

R, H = 0.06, 0.0125   # cf2x.urdf collision cylinder
MG = CORE_MARGINS[0]
RC, HC = R - MG, H - MG


def pair_sets(n, rng):
    """{name: [(cA - cB, axis A, axis B)]}: random near-contact pairs (half any axis); stacked discs
    (A over B, nearly parallel axes, small offsets); side by side; rim to rim (stacked with offsets
    near 2 R); flat (stacked, tilts below 1 degree)."""
    def tilted(deg):
        t = math.radians(rng.random() * deg)
        ph = rng.random() * 2 * math.pi
        return np.array([math.sin(t) * math.cos(ph), math.sin(t) * math.sin(ph), math.cos(t)])

    def any_axis():
        v = rng.normal(size=3)
        return v / np.linalg.norm(v)

    def ext(u, a):
        ua = float(u @ a)
        return H * abs(ua) + R * math.sqrt(max(0.0, 1.0 - ua * ua))
    out = {k: [] for k in ("random", "stacked", "side", "rimrim", "flat")}
    for i in range(n):
        aa, ab = (any_axis() if i % 2 else tilted(20)), tilted(20)
        u = any_axis()
        out["random"].append((u * (ext(u, aa) + ext(u, ab) + rng.uniform(-0.006, 0.004)), aa, ab))
        aa, ab = tilted(10), tilted(10)
        out["stacked"].append((np.array([rng.uniform(-.06, .06), rng.uniform(-.06, .06),
                                         2 * H + rng.uniform(-0.002, 0.004)]), aa, ab))
        aa, ab = tilted(10), tilted(10)
        ph, d = rng.random() * 2 * math.pi, 2 * R + rng.uniform(-0.002, 0.004)
        out["side"].append((np.array([d * math.cos(ph), d * math.sin(ph), rng.uniform(-0.02, 0.02)]), aa, ab))
        aa, ab = tilted(15), tilted(15)
        ph, d = rng.random() * 2 * math.pi, rng.uniform(0.09, 0.125)
        out["rimrim"].append((np.array([d * math.cos(ph), d * math.sin(ph), 2 * H + rng.uniform(-0.004, 0.004)]), aa, ab))
        aa, ab = tilted(1), tilted(1)
        out["flat"].append((np.array([rng.uniform(-.1, .1), rng.uniform(-.1, .1),
                                      2 * H + rng.uniform(-0.0005, 0.002)]), aa, ab))
    return out


def core_distance(cl, aa, ab):
    """core_pair's distance for a world-frame pair (B at the origin), in B's btPlaneSpace1 frame."""
    bp, bq = plane_space(ab)
    Mb = np.stack([bp, bq, ab])
    return core_pair(Mb @ cl, Mb @ aa, RC, HC)[2]


def errors(pairs):
    """(errors of separated pairs vs the exact distance, exact distances, overlaps detected / total)."""
    err, ex, ov, ovok = [], [], 0, 0
    for cl, aa, ab in pairs:
        up, lo = exact_distance(cl, aa, ab, RC, HC)
        d = core_distance(cl, aa, ab)
        if up < 1e-9:
            ov += 1
            ovok += d <= 1e-4
            continue
        if up - lo > 1e-9:
            continue                      # not certified (never seen on these sets)
        err.append(d - up)
        ex.append(up)
    return np.array(err), np.array(ex), (ovok, ov)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    for name, pairs in pair_sets(n, rng).items():
        e, _, (ok, ov) = errors(pairs)
        print(f"{name}: {len(e)} separated pairs: distance error p50 {np.percentile(e, 50):.1e} p99 "
              f"{np.percentile(e, 99):.1e} max {e.max():.1e} min {e.min():.1e} m; overlaps detected {ok}/{ov}",
              flush=True)


if __name__ == "__main__":
    main()
