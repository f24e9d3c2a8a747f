"""Diagnostic: where does the PID-path obs differ from the oracle (act/physics from argv)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tests.oracle_runs import run_vec
from tests.test_gpu_pid import _actions
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
act, physics = sys.argv[1], sys.argv[2]
rng = np.random.default_rng(11)
E, T = 12, 60
acts = _actions(rng, act, T, E)
envs = []
obs_r, rew_r, te_r, tr_r, _ = run_vec(acts, E, act=act, wrench="geom" if physics == "pyb" else "dyn", envs=envs)
sim = BatchedAviarySim(device="cuda:0", n_envs=E, task="hover", precision="f64", act=ActionType(act), physics=Physics(physics))
for t in range(T):
    o = sim.step(torch.from_numpy(acts[t]).cuda())[0].cpu().numpy()
    d = np.abs(o - obs_r[t])
    bad = np.argwhere(d > 1e-6 + 1e-5 * np.abs(obs_r[t]))
    if len(bad):
        for e, _, col in bad[:6]:
            print(f"t={t} env={e} col={col} gpu={o[e,0,col]!r} ref={obs_r[t][e,0,col]!r} done={te_r[t,e] or tr_r[t,e]} act={acts[t,e,0]}")
    print(t, "maxdiff", d.max(), flush=True)
