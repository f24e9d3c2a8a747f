"""examples/learn.py's PPO update, eager vs graphed (GraphedMinibatch), in lockstep from the same
weights on the same real rollout batch (seed 0, single-drone HoverAviary, Physics.PYB): the largest
parameter difference after each minibatch step, split by how large the Adam update of that
parameter was - to tell rounding (1e-7) from a systematic difference.
Usage (GPU box): python scripts/graph_vs_eager.py"""
import copy
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import learn  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
E, T = 4096, 64
env = learn.make_env(False, E, learn.DEFAULT_ACT, learn.Physics.PYB, dev, 0)
D, A = env.num_drones, env.sim.act_width
n_obs, n_act = D * env.sim.obs_width, D * A
pol_a = learn.ActorCritic(n_obs, n_act).to(dev)
pol_b = copy.deepcopy(pol_a)
# one rollout with pol_a (the training loop's first iteration)
obs = env.reset().reshape(E, -1)
bo, ba, bl, bv, br, bd = [], [], [], [], [], []
with torch.no_grad():
    for t in range(T):
        d = pol_a.dist(obs)
        a = d.sample()
        v = pol_a.value(obs)
        o2, r, done, info = env.step(a.clamp(-1, 1))
        bo.append(obs); ba.append(a); bl.append(d.log_prob(a).sum(-1)); bv.append(v); br.append(r); bd.append(done.float())
        obs = o2.reshape(E, -1)
    last_v = pol_a.value(obs)
    adv = torch.zeros(T, E, device=dev)
    g = torch.zeros(E, device=dev)
    for t in reversed(range(T)):
        nv = last_v if t == T - 1 else bv[t + 1]
        nt = 1.0 - bd[t]
        delta = br[t] + 0.99 * nv * nt - bv[t]
        g = delta + 0.99 * 0.95 * nt * g
        adv[t] = g
    ret = adv + torch.stack(bv)
N = T * E
b_obs, b_act = torch.stack(bo).reshape(N, -1), torch.stack(ba).reshape(N, -1)
b_logp, b_adv, b_ret = torch.stack(bl).reshape(N), adv.reshape(N), ret.reshape(N)
mb, clip, vf, mgn = 16384, 0.2, 0.5, 0.5
opt_a = torch.optim.Adam(pol_a.parameters(), lr=3e-4, eps=1e-5)
opt_b = torch.optim.Adam(pol_b.parameters(), lr=3e-4, eps=1e-5, capturable=True)
gstep = learn.GraphedMinibatch(pol_b, opt_b, mb, n_obs, n_act, clip, vf, mgn, dev)
assert all(torch.equal(p, q) for p, q in zip(pol_a.parameters(), pol_b.parameters()))
rows = []
step = 0
for ep in range(10):
    perm = torch.randperm(N, device=dev)
    for s in range(0, N, mb):
        idx = perm[s:s + mb]
        p0 = [p.detach().clone() for p in pol_a.parameters()]
        d = pol_a.dist(b_obs[idx])
        ratio = (d.log_prob(b_act[idx]).sum(-1) - b_logp[idx]).exp()
        ma = (b_adv[idx] - b_adv[idx].mean()) / (b_adv[idx].std() + 1e-8)
        pg = -torch.min(ratio * ma, ratio.clamp(1 - clip, 1 + clip) * ma).mean()
        loss = pg + vf * ((pol_a.value(b_obs[idx]) - b_ret[idx]) ** 2).mean()
        opt_a.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(pol_a.parameters(), mgn)
        opt_a.step()
        gstep.step(b_obs[idx], b_act[idx], b_logp[idx], b_adv[idx], b_ret[idx])
        step += 1
        if step in (1, 2, 4, 8, 16, 32, 64, 100, 160):
            dif = max(float((p - q).abs().max()) for p, q in zip(pol_a.parameters(), pol_b.parameters()))
            mv = max(float(p.abs().max()) for p in pol_a.parameters())
            upd = max(float((p - p0_).abs().max()) for p, p0_ in zip(pol_a.parameters(), p0))
            rows.append({"step": step, "max_param_diff": dif, "max_param": mv, "last_update_max": upd,
                         "loss_eager": float(loss)})
            print(json.dumps(rows[-1]), flush=True)
env.close()
