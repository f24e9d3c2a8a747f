"""Diagnostic: per-column obs differences, GPU f64 step() vs oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tests.oracle_runs import run_vec
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
rng = np.random.default_rng(4)
E, T, A = 16, 80, 4
acts = np.clip(rng.normal(0, 0.1, (T, E, 1, A)), -1, 1).astype(np.float32)
acts[:, :4] = rng.uniform(-1, 1, (T, 4, 1, A)).astype(np.float32)
obs_r, rew_r, te_r, tr_r, tobs_r = run_vec(acts, E)
for prec in ("f64", "f32"):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision=prec, device="cuda:0")
    worst = []
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        o = o.cpu().numpy()
        d = np.abs(o - obs_r[t])
        e, _, c = np.unravel_index(np.argmax(d), d.shape)
        worst.append((d.max(), t, e, c, o[e, 0, c], obs_r[t][e, 0, c], bool(te_r[t][e] or tr_r[t][e])))
    worst.sort(reverse=True)
    print(prec, "top diffs (absdiff, step, env, col, gpu, ref, done):")
    for w in worst[:8]:
        print("  ", w)
