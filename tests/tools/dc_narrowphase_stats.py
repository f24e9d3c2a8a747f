"""CPU: what the drone <-> drone narrowphase costs on the RL example's env (2-drone MultiHover,
Physics.PYB, U[-1,1] RPM actions, auto-reset), counted in the numpy oracle: near pairs per
env-substep, margin levels tried and alternating-projection rounds per level, and how long a pair
stays in contact (persistent contacts are what hold the slowest GPU wave: 8 solves per step).
Usage: python tests/tools/dc_narrowphase_stats.py [envs] [steps] [drones]"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle.bullet_mb as mb  # noqa: E402
from tests.oracle_runs import run_vec  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 240
D = int(sys.argv[3]) if len(sys.argv) > 3 else 2

calls = []
orig_proj = mb.cyl_project
rounds = [0]


def proj(*a):
    rounds[0] += 1
    return orig_proj(*a)


orig_geom = mb.pair_geometry


def geom(ca, aa, cb, ab, radius, half_height):
    rounds[0] = 0
    levels = [0]
    orig_sep = mb.CORE_SEP
    out = orig_geom(ca, aa, cb, ab, radius, half_height)
    calls.append((rounds[0] // 2, out[2]))
    return out


mb.cyl_project = proj
mb.pair_geometry = geom
rng = np.random.default_rng(0)
acts = rng.uniform(-1, 1, (T, E, D, 4)).astype(np.float32)
run_vec(acts, E, drones_per_env=D, act="rpm", task="multihover", integrator="bullet")
r = np.array([c[0] for c in calls])
d = np.array([c[1] for c in calls])
print(f"{E} envs x {D} drones, {T} steps: {len(calls)} narrowphase calls ({len(calls) / (E * T * 8):.4f} per env-substep)")
print(f"  projection rounds per call (all levels): mean {r.mean():.2f}  hist {dict(sorted(collections.Counter(r).items()))}")
print(f"  contacts (dist < brk): {(d < mb.breaking_threshold(0.06, 0.0125)).mean():.3f} of calls; dist quantiles "
      f"{np.quantile(d, [0, 0.1, 0.5, 0.9, 1]).round(5).tolist()}")
