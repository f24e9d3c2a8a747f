"""examples/learn.py on the MI355X path: PPO on thousands of batched HoverAviary /
MultiHoverAviary envs, everything resident in HBM.

The reference (``gym_pybullet_drones/examples/learn.py:52-103``) trains stable-baselines3 PPO
('MlpPolicy') on ``make_vec_env(HoverAviary, env_kwargs=dict(obs=KIN, act=ONE_D_RPM), n_envs=1)``
and stops at an evaluation return of 474.15 (single agent) / 949.5 (two agents).  SB3 is not
installed in this image, so this script carries a compact PPO with SB3's defaults (separate
64-64 tanh actor and critic, state-independent log-std, GAE(0.99, 0.95), clip 0.2, 10 epochs,
advantage normalisation, TimeLimit bootstrapping from ``terminal_observation``) over the same
env surface: ``make_vec_env(..., output="torch")`` returns observations, rewards and done
masks as device tensors, so the whole loop (policy, env step, GAE, update) stays on the GPU.

    python examples/learn.py                     # HoverAviary, 4096 envs, ONE_D_RPM, Physics.PYB
    python examples/learn.py --multiagent true   # MultiHoverAviary, 2 drones
    python examples/learn.py --physics dyn       # the explicit DYN integrator instead
    python examples/learn.py --gpus 8 --n_envs 32768   # envs sharded over 8 GPUs, learner on rank 0
    python examples/learn.py --gpus 8 --n_envs 32768 --learner per-rank   # a learner per GPU, gradient all-reduce

Physics defaults to the env classes' default, Physics.PYB (the reference's learn.py does not
pass one), i.e. the restated Bullet multibody step.

Evaluation follows the reference's EvalCallback(deterministic=True): the mean action of the
policy on a fresh single env, the return of one full episode (the env and the policy are
deterministic, so EvalCallback's 5 episodes are 5 copies of it), after every PPO update - the
reference's eval_freq=1000 with n_envs=1 evaluates about twice per 2048-step update
(``examples/learn.py:84-91`` there); round 4 evaluated after every second update.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_pybullet_drones_routing_amd.enums import ActionType, ObservationType, Physics  # noqa: E402
from gym_pybullet_drones_routing_amd.envs import HoverAviary, MultiHoverAviary, make_vec_env  # noqa: E402
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

DEFAULT_OBS = ObservationType('kin')
DEFAULT_ACT = ActionType('one_d_rpm')
DEFAULT_AGENTS = 2


def mlp(n_in, n_out, out_gain):
    layers = [nn.Linear(n_in, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, n_out)]
    for i, l in enumerate(m for m in layers if isinstance(m, nn.Linear)):
        nn.init.orthogonal_(l.weight, gain=out_gain if i == 2 else math.sqrt(2))
        nn.init.zeros_(l.bias)
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    """SB3 MlpPolicy for a Box action space: separate pi / vf networks [64, 64] tanh."""

    def __init__(self, n_obs, n_act):
        super().__init__()
        self.pi = mlp(n_obs, n_act, 0.01)
        self.vf = mlp(n_obs, 1, 1.0)
        self.log_std = nn.Parameter(torch.zeros(n_act))

    def dist(self, obs):
        return torch.distributions.Normal(self.pi(obs), self.log_std.exp())

    def value(self, obs):
        return self.vf(obs).squeeze(-1)


def evaluate(policy, multiagent, device, act, physics=Physics.PYB):
    """EvalCallback(deterministic=True, n_eval_episodes=1): one episode of a fresh env."""
    D = DEFAULT_AGENTS if multiagent else 1
    sim = BatchedAviarySim(n_envs=1, drones_per_env=D, task="multihover" if multiagent else "hover",
                           act=act, physics=physics, autoreset=False, device=device)
    obs = sim.reset().clone()
    ret, steps = 0.0, 0
    with torch.no_grad():
        while True:
            a = policy.pi(obs.reshape(1, -1)).clamp(-1, 1).reshape(1, D, -1).contiguous()
            o, r, te, tr = sim.step(a, terminal_obs=False)
            ret += float(r[0])
            steps += 1
            if bool(te[0]) or bool(tr[0]):
                break
            obs = o.clone()
    sim.close()
    return ret, steps


def _collective(fn, t, *args):
    """Run a torch.distributed collective on `t` in place; gloo (the rehearsal backend) gets a host
    copy of a device tensor."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        fn(h, *args)
        t.copy_(h)
    else:
        fn(t, *args)
    return t


def sync_grads(params, world):
    """Per-rank learners (SURVEY §8(e)'s alternative to the single learner): average the
    gradients over the ranks with ONE all-reduce of a flat bucket (the 64-64 actor / critic pair
    is ~10^4 parameters, ~40 KB: one latency-bound RCCL call per minibatch).  Every rank then
    holds the same gradients, so the same clip and Adam step keep the parameters identical."""
    import torch.distributed as dist
    params = [p for p in params if p.grad is not None]
    flat = torch.cat([p.grad.reshape(-1) for p in params])
    _collective(dist.all_reduce, flat)
    flat.div_(world)
    off = 0
    for p in params:
        n = p.grad.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n


def broadcast_params(module):
    """Rank 0's initial parameters on every rank (one flat broadcast)."""
    import torch.distributed as dist
    ps = list(module.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in ps])
    _collective(dist.broadcast, flat, 0)
    off = 0
    with torch.no_grad():
        for p in ps:
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()


def make_env(multiagent, n_envs, act, physics, device, seed=0, distributed=False):
    env_cls = MultiHoverAviary if multiagent else HoverAviary
    kw = dict(obs=DEFAULT_OBS, act=act, physics=Physics(physics))
    if multiagent:
        kw["num_drones"] = DEFAULT_AGENTS
    # store policy 2 (write-through rows): between the policy's kernels the step measured 6.12 vs
    # 6.40 us (bench.py rollout leg, profiles/r4/rollout_policy/); the back-to-back default is 3
    extra = {}
    if distributed:
        import torch.distributed as dist
        # RCCL: the hand-off (scatter, shard step, pack, gather, unpack) replays one hipGraph per step
        extra["graph"] = dist.is_initialized() and dist.get_backend() == "nccl"
    return make_vec_env(env_cls, env_kwargs=kw, n_envs=n_envs, seed=seed, output="torch", device=device,
                        distributed=distributed, tuning={"store_policy": 2}, **extra)


class GraphedMinibatch:
    """One PPO minibatch step (forward, clipped surrogate + value loss, backward, grad-norm clip,
    Adam) captured in a hipGraph: the ~100 small kernels of the eager step replay without a host
    launch each (world == 1; the per-rank learners' all-reduce stays eager).  The minibatch is
    gathered into static buffers outside the graph.  Capture needs the optimizer's state and the
    allocator's warm-up: a few eager steps on a side stream, after which the policy's parameters
    and the optimizer's state are restored to their values from before them (in place: the graph
    holds those tensors), so the training is the same as the eager loop's."""

    def __init__(self, policy, opt, mb, n_obs, n_act, clip, vf_coef, max_grad_norm, device):
        self.policy, self.opt = policy, opt
        self.obs = torch.zeros((mb, n_obs), device=device)
        self.act = torch.zeros((mb, n_act), device=device)
        self.logp = torch.zeros(mb, device=device)
        self.adv = torch.zeros(mb, device=device)
        self.ret = torch.zeros(mb, device=device)
        self.clip, self.vf_coef, self.max_grad_norm = clip, vf_coef, max_grad_norm
        params0 = [p.detach().clone() for p in policy.parameters()]
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _ in range(3):
                opt.zero_grad(set_to_none=True)
                self._body()
        torch.cuda.current_stream(device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self._body()
        with torch.no_grad():                        # undo the warm-up steps, in place
            for p, p0 in zip(policy.parameters(), params0):
                p.copy_(p0)
            for st in opt.state.values():
                for k, t in st.items():
                    if torch.is_tensor(t):
                        t.zero_()                    # Adam's moments and step count start at zero

    def _body(self):
        # Normal(mu, exp(log_std)).log_prob, written out as torch.distributions computes it (its
        # argument validation would read a device flag on the host: not capturable)
        mu = self.policy.pi(self.obs)
        scale = self.policy.log_std.exp()
        logp = (-((self.act - mu) ** 2) / (2 * scale ** 2) - scale.log() - math.log(math.sqrt(2 * math.pi))).sum(-1)
        ratio = (logp - self.logp).exp()
        ma = (self.adv - self.adv.mean()) / (self.adv.std() + 1e-8)
        pg = -torch.min(ratio * ma, ratio.clamp(1 - self.clip, 1 + self.clip) * ma).mean()
        vl = ((self.policy.value(self.obs) - self.ret) ** 2).mean()
        loss = pg + self.vf_coef * vl
        loss.backward()
        nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
        self.opt.step()

    def step(self, obs, act, logp, adv, ret):
        self.obs.copy_(obs)
        self.act.copy_(act)
        self.logp.copy_(logp)
        self.adv.copy_(adv)
        self.ret.copy_(ret)
        self.graph.replay()


class FusedRollout:
    """The rollout on the HIP path: per env.step ONE fused policy kernel (actor + critic forward,
    Normal sample, clip, the buffer rows, and the previous step's time-limit bootstrap;
    ``policy.MlpPolicyKernel``) and ONE env step, the whole n_steps sequence captured in one
    hipGraph and replayed every PPO iteration (the parameters are read in place, so the optimizer's
    in-place updates reach the graph); then the last value and GAE (``gpd_policy_gae``, bit-identical
    to the torch loop of ``train``).  The same quantities as the eager loop, drawn from a Philox
    stream instead of torch's generator.

    ``env``: an ``AviaryVecEnv`` (the step is ``gpd_step`` on its sim) or, on RCCL, a
    ``ShardedAviaryVecEnv`` (the step is the learner hand-off: action scatter, every rank's shard
    step, record gather and unpack, ``shard.LearnerHandoff``; the other ranks capture and replay the
    same n_steps hand-off steps on the learner's ROLLOUT command, so the collectives pair up)."""

    def __init__(self, policy, env, n_steps, gamma, gae_lambda, seed, bufs):
        from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
        # the Philox row-group counters sized for the whole batch before anything is captured
        self.k = MlpPolicyKernel(policy, seed=seed, max_rows=max(1, int(env.num_envs)))
        self.env, self.T, self.gamma, self.lam = env, n_steps, gamma, gae_lambda
        h = getattr(env, "handoff", None)
        self.h = h
        if h is not None:            # the learner's global batch, rebuilt in place by every hand-off step
            E = env.num_envs
            n_obs = h.obs[0].numel()
            self.obs, self.tobs = h.obs.view(E, n_obs), h.terminal_rows.view(E, n_obs)
            self.act = h.global_actions
            self.flags = lambda: (h.reward, h.terminated, h.truncated, self.tobs)
            self.step_fn = lambda: h.step_body(h.global_actions)
            dev = h.device
        else:
            sim = env.sim
            E = sim.n_envs
            n_obs = sim.drones_per_env * sim.obs_width
            self.obs = sim.obs.view(E, n_obs)             # sim-owned, rewritten in place by every step
            self.tobs = sim.terminal_obs.view(E, n_obs)
            self.act = torch.zeros((E, sim.drones_per_env, sim.act_width), device=sim.device)
            self.flags = lambda: (sim.reward, sim.terminated, sim.truncated, self.tobs)
            self.step_fn = lambda: sim.step(self.act, terminal_obs=True)
            dev = sim.device
        self.E = E
        self.b = bufs
        self.last_v = torch.zeros(E, device=dev)
        self.graph = None

    def _seq(self):
        b, k = self.b, self.k
        for t in range(self.T):
            prev = self.flags() if t else None
            k.step(self.obs, self.act.view(self.E, -1), b["obs"][t], b["act"][t], b["logp"][t],
                   b["val"][t], prev=prev, gamma=self.gamma, buf_rew=b["rew"][t - 1] if t else None,
                   buf_done=b["done"][t - 1] if t else None)
            self.step_fn()
        k.step(self.obs, buf_val=self.last_v, prev=self.flags(),
               gamma=self.gamma, buf_rew=b["rew"][self.T - 1], buf_done=b["done"][self.T - 1])
        k.gae(b["rew"], b["val"], b["done"], self.last_v, self.gamma, self.lam, b["adv"], b["ret"])

    def run(self):
        if self.h is not None:
            self.env.rollout(self.T, self._seq)      # the ROLLOUT command: every rank replays its graph
            return
        if self.graph is None:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._seq()
        self.graph.replay()


def train(multiagent=False, n_envs=4096, n_steps=64, total_timesteps=int(3e7), lr=3e-4, epochs=10,
          minibatch=16384, gamma=0.99, gae_lambda=0.95, clip=0.2, vf_coef=0.5, max_grad_norm=0.5,
          eval_every=1, seed=0, device="cuda:0", act=DEFAULT_ACT, target_reward=None, max_seconds=None,
          log=print, physics=Physics.PYB, env=None, world=1, rank=0, graph=False, fused=False):
    """PPO on the batched env.  ``env``: an already built torch-output VecEnv (e.g. the
    multi-GPU ``ShardedAviaryVecEnv``); by default one ``AviaryVecEnv`` on ``device``.
    world > 1: per-rank learners under torch.distributed — this rank trains on its own
    ``n_envs`` envs with ``minibatch / world`` samples per minibatch, gradients are averaged over
    the ranks (sync_grads), rank 0 evaluates and decides when every rank stops; ``timesteps``
    and the history count all ranks' samples.  ``graph``: the minibatch steps as one captured
    hipGraph (``GraphedMinibatch``; world == 1 and full minibatches only).  ``fused``: the rollout
    as ``FusedRollout`` (one policy kernel + one gpd_step per env.step, one hipGraph per rollout;
    a single-GPU ``AviaryVecEnv``)."""
    import torch.distributed as dist
    torch.manual_seed(seed)
    physics = Physics(physics)
    if env is None:
        env = make_env(multiagent, n_envs, act, physics, device, seed)
    if target_reward is None:   # learn.py:80-83
        if act == ActionType.ONE_D_RPM:
            target_reward = 474.15 if not multiagent else 949.5
        else:
            target_reward = 467. if not multiagent else 920.
    log(f"[INFO] Action space: {env.action_space}")
    log(f"[INFO] Observation space: {env.observation_space}")
    D, A = env.num_drones, env.sim.act_width
    n_obs, n_act = D * env.sim.obs_width, D * A
    policy = ActorCritic(n_obs, n_act).to(device)
    if world > 1:
        broadcast_params(policy)
        torch.manual_seed(seed + 1000003 * rank)   # each rank samples its own actions / minibatches
        minibatch = max(1, minibatch // world)
    graph = graph and world == 1 and torch.device(device).type == "cuda"
    opt = torch.optim.Adam(policy.parameters(), lr=lr, eps=1e-5, capturable=graph)
    gstep = GraphedMinibatch(policy, opt, minibatch, n_obs, n_act, clip, vf_coef, max_grad_norm, device) if graph else None
    E = n_envs
    buf_obs = torch.zeros((n_steps, E, n_obs), device=device)
    buf_act = torch.zeros((n_steps, E, n_act), device=device)
    buf_logp = torch.zeros((n_steps, E), device=device)
    buf_val = torch.zeros((n_steps, E), device=device)
    buf_rew = torch.zeros((n_steps, E), device=device)
    buf_done = torch.zeros((n_steps, E), device=device)
    obs = env.reset().reshape(E, -1)
    fr = None
    if fused:
        if getattr(env, "handoff", None) is not None and not getattr(env, "graphed", False):
            raise ValueError("fused=True over sharded envs needs the RCCL hand-off (ShardedAviaryVecEnv(graph=True))")
        adv_buf, ret_buf = torch.zeros((n_steps, E), device=device), torch.zeros((n_steps, E), device=device)
        fr = FusedRollout(policy, env, n_steps, gamma, gae_lambda, seed,
                          {"obs": buf_obs, "act": buf_act, "logp": buf_logp, "val": buf_val, "rew": buf_rew,
                           "done": buf_done, "adv": adv_buf, "ret": ret_buf})
    history = []
    t0 = time.time()
    timesteps, it = 0, 0
    best = -1e9
    while timesteps < total_timesteps:
        t_roll = time.time()
        if fr is not None:
            with torch.no_grad():
                fr.run()
            adv, ret = fr.b["adv"], fr.b["ret"]
        else:
            with torch.no_grad():
                for t in range(n_steps):
                    d = policy.dist(obs)
                    a = d.sample()
                    v = policy.value(obs)
                    o2, r, done, info = env.step(a.clamp(-1, 1))            # SB3 clips to the Box
                    o2 = o2.reshape(E, -1)
                    trunc = info["TimeLimit.truncated"]
                    if bool(trunc.any()):                                 # bootstrap time limits
                        tv = policy.value(info["terminal_observation"].reshape(E, -1))
                        r = r + gamma * tv * trunc.float()
                    buf_obs[t], buf_act[t], buf_logp[t], buf_val[t] = obs, a, d.log_prob(a).sum(-1), v
                    buf_rew[t], buf_done[t] = r, done.float()
                    obs = o2
                last_v = policy.value(obs)
                adv = torch.zeros_like(buf_rew)
                g = torch.zeros(E, device=device)
                for t in reversed(range(n_steps)):
                    nv = last_v if t == n_steps - 1 else buf_val[t + 1]
                    nonterm = 1.0 - buf_done[t]
                    delta = buf_rew[t] + gamma * nv * nonterm - buf_val[t]
                    g = delta + gamma * gae_lambda * nonterm * g
                    adv[t] = g
                ret = adv + buf_val
        t_upd = time.time()
        N = n_steps * E
        b_obs, b_act, b_logp = buf_obs.reshape(N, -1), buf_act.reshape(N, -1), buf_logp.reshape(N)
        b_adv, b_ret, b_val = adv.reshape(N), ret.reshape(N), buf_val.reshape(N)
        for _ in range(epochs):
            perm = torch.randperm(N, device=device)
            for s in range(0, N, minibatch):
                idx = perm[s:s + minibatch]
                if gstep is not None and idx.numel() == minibatch:
                    gstep.step(b_obs[idx], b_act[idx], b_logp[idx], b_adv[idx], b_ret[idx])
                    continue
                d = policy.dist(b_obs[idx])
                logp = d.log_prob(b_act[idx]).sum(-1)
                ratio = (logp - b_logp[idx]).exp()
                ma = b_adv[idx]
                ma = (ma - ma.mean()) / (ma.std() + 1e-8)
                pg = -torch.min(ratio * ma, ratio.clamp(1 - clip, 1 + clip) * ma).mean()
                vl = ((policy.value(b_obs[idx]) - b_ret[idx]) ** 2).mean()
                loss = pg + vf_coef * vl
                opt.zero_grad(set_to_none=True)
                loss.backward()
                if world > 1:
                    sync_grads(policy.parameters(), world)
                nn.utils.clip_grad_norm_(policy.parameters(), max_grad_norm)
                opt.step()
        timesteps += N * world
        it += 1
        mean_rew = buf_rew.mean()
        if world > 1:
            mean_rew = _collective(dist.all_reduce, mean_rew.reshape(1)) / world
        rec = {"iter": it, "timesteps": timesteps, "mean_step_reward": float(mean_rew),
               "rollout_s": round(t_upd - t_roll, 3), "update_s": round(time.time() - t_upd, 3),
               "wall_s": round(time.time() - t0, 1)}
        if it % eval_every == 0 and rank == 0:
            er, el = evaluate(policy, multiagent, device, act, physics)
            rec.update(eval_return=er, eval_len=el)
            best = max(best, er)
        history.append(rec)
        if rank == 0:
            log(json.dumps(rec))
        reached = rec.get("eval_return", -1e9) >= target_reward
        stop = reached or bool(max_seconds and time.time() - t0 > max_seconds)
        if world > 1:   # rank 0's decision for every rank
            flag = torch.tensor([1 if stop else 0, 1 if reached else 0], device=device)
            _collective(dist.broadcast, flag, 0)
            stop, reached = bool(flag[0]), bool(flag[1])
        if reached and rank == 0:
            log(f"[INFO] reward threshold {target_reward} reached after {timesteps} timesteps")
        if stop:
            break
    env.close()
    return policy, history, best, target_reward


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="PPO on batched HoverAviary / MultiHoverAviary (MI355X)")
    p.add_argument("--multiagent", default="false")
    p.add_argument("--n_envs", type=int, default=4096, help="envs over all GPUs")
    p.add_argument("--total_timesteps", type=float, default=2e8)
    p.add_argument("--max_seconds", type=float, default=None)
    p.add_argument("--physics", default="pyb", help="Physics value (default: pyb, the env classes' default)")
    p.add_argument("--output", default=None, help="JSON file for the training history")
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs: the envs are sharded over one rank per GPU, the learner runs on rank 0 "
                        "(without WORLD_SIZE in the env, learn.py starts the ranks itself)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL over xGMI); gloo only to rehearse several ranks on one GPU")
    p.add_argument("--seed", type=int, default=0, help="torch seed of the policy, the sampling and the envs")
    p.add_argument("--graph", action="store_true",
                   help="replay each PPO minibatch step as one captured hipGraph (faster update; same "
                        "arithmetic up to rounding, so a different training trajectory than the default "
                        "eager loop, which reproduces the recorded runs step for step)")
    p.add_argument("--rollout", default="fused", choices=["fused", "eager"],
                   help="fused: one policy kernel + one env step (gpd_step, or the RCCL learner hand-off over the "
                        "ranks) per env.step, the rollout replayed as one hipGraph (FusedRollout); eager: the "
                        "torch policy step by step (the loop that reproduces the recorded round-4/5 runs)")
    p.add_argument("--learner", default="rank0", choices=["rank0", "per-rank"],
                   help="rank0: one learner on the gathered batch (ShardedAviaryVecEnv); per-rank: a learner "
                        "per GPU on its own env shard, gradients all-reduced")
    return p.parse_args(argv)


def run(a):
    """One rank: shard of the envs; rank 0 also runs PPO on the gathered batch (--learner rank0),
    or every rank runs PPO on its own shard with averaged gradients (--learner per-rank)."""
    import torch.distributed as dist
    multi = str(a.multiagent).lower() in ("1", "true", "yes")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local % torch.cuda.device_count() if a.dist_backend == "gloo" else local
    device = torch.device(f"cuda:{dev_index}")
    torch.cuda.set_device(device)
    env = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        if a.learner == "per-rank":
            from gym_pybullet_drones_routing_amd.shard import env_shard
            _, n_local = env_shard(a.n_envs, rank, world)
            policy, hist, best, target = train(multiagent=multi, n_envs=n_local,
                                               total_timesteps=int(a.total_timesteps), max_seconds=a.max_seconds,
                                               physics=Physics(a.physics), device=device, world=world, rank=rank,
                                               log=print if rank == 0 else (lambda *x: None))
            if rank == 0:
                out = {"multiagent": multi, "physics": a.physics, "n_envs": a.n_envs, "gpus": world,
                       "learner": "per-rank", "target_reward": target, "best_eval_return": best,
                       "reached": best >= target, "history": hist}
                print(json.dumps({k: v for k, v in out.items() if k != "history"}), flush=True)
                if a.output:
                    with open(a.output, "w") as f:
                        json.dump(out, f, indent=1)
            dist.destroy_process_group()
            return
        env = make_env(multi, a.n_envs, DEFAULT_ACT, Physics(a.physics), device, distributed=True)
        if rank != 0:
            env.serve()
            dist.destroy_process_group()
            return
    fused = a.rollout == "fused" and (world == 1 or getattr(env, "graphed", False))
    policy, hist, best, target = train(multiagent=multi, n_envs=a.n_envs, total_timesteps=int(a.total_timesteps),
                                       max_seconds=a.max_seconds, physics=Physics(a.physics), device=device, env=env,
                                       graph=a.graph, seed=a.seed, fused=fused)
    out = {"multiagent": multi, "physics": a.physics, "n_envs": a.n_envs, "gpus": world, "target_reward": target,
           "rollout": "fused" if fused else "eager",
           "best_eval_return": best, "reached": best >= target, "history": hist}
    print(json.dumps({k: v for k, v in out.items() if k != "history"}), flush=True)
    if a.output:
        with open(a.output, "w") as f:
            json.dump(out, f, indent=1)
    if world > 1:
        dist.destroy_process_group()


def _rank_entry(rank, world, port, argv):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run(parse_args(argv))


def main():
    a = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != a.gpus:
        raise SystemExit(f"learn.py: WORLD_SIZE={env_world} but --gpus {a.gpus}")
    if env_world is not None or a.gpus <= 1:
        run(a)
        return
    # --gpus N without a launcher: N rank processes, started before anything touches the GPU
    import socket
    import torch.multiprocessing as mp
    if a.dist_backend == "nccl" and torch.cuda.device_count() < a.gpus:
        raise SystemExit(f"learn.py: --gpus {a.gpus} needs {a.gpus} GPUs for RCCL (--dist-backend gloo rehearses)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_entry, args=(r, a.gpus, port, sys.argv[1:])) for r in range(a.gpus)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    if any(p.exitcode != 0 for p in procs):
        raise SystemExit(f"learn.py: rank exit codes {[p.exitcode for p in procs]}")


if __name__ == "__main__":
    main()
