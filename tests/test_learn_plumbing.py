"""examples/learn.py plumbing: the GPU-resident PPO drives the batched
VecEnv surface end to end.  The full run (reward threshold 474.15 / 949.5) is recorded in
profiles/learn_r1.json; here two short iterations check that rollout, TimeLimit bootstrapping,
GAE, the update and the deterministic evaluation episode all run on the device."""
import math
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("multi", [False, True])
def test_ppo_two_iterations(multi):
    import learn
    logs = []
    policy, hist, best, target = learn.train(multiagent=multi, n_envs=256, n_steps=16, total_timesteps=2 * 256 * 16,
                                             minibatch=1024, epochs=2, eval_every=1, log=logs.append)
    assert len(hist) == 2
    assert target == (949.5 if multi else 474.15)
    for h in hist:
        assert math.isfinite(h["mean_step_reward"]) and h["eval_len"] >= 1
    assert any("Observation space" in l for l in logs if isinstance(l, str))


def _sharded_worker(rank, world, port, q):
    import datetime

    import torch
    import torch.distributed as dist
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        import learn
        from gym_pybullet_drones_routing_amd.enums import Physics
        env = learn.make_env(False, 128, learn.DEFAULT_ACT, Physics.PYB, "cuda:0", distributed=True)
        assert env.sim.n_envs == 64
        if rank == 0:
            _, hist, _, _ = learn.train(n_envs=128, n_steps=8, total_timesteps=2 * 128 * 8, minibatch=512, epochs=2,
                                        eval_every=1, log=lambda *a: None, device=torch.device("cuda:0"), env=env)
            env.close()
            q.put(hist)
        else:
            env.serve()
    finally:
        dist.destroy_process_group()


def test_ppo_sharded_two_ranks_matches_single_process():
    """examples/learn.py --gpus 2 (config 5 plumbing): the learner on rank 0 drives two env shards
    through ShardedAviaryVecEnv (command broadcast, action scatter, output-pack all-gather; gloo,
    both ranks on this GPU).  The training history equals one process stepping all 128 envs:
    the gathered batch is bit-identical, so the seeded PPO run is too."""
    import socket

    import torch.multiprocessing as mp
    import learn
    from tests.test_gpu_dist import _collect
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    hist2 = _collect(q, procs)
    _, hist1, _, _ = learn.train(n_envs=128, n_steps=8, total_timesteps=2 * 128 * 8, minibatch=512, epochs=2,
                                 eval_every=1, log=lambda *a: None)
    assert len(hist1) == len(hist2) == 2
    for a, b in zip(hist1, hist2):
        assert a["timesteps"] == b["timesteps"]
        assert math.isclose(a["mean_step_reward"], b["mean_step_reward"], rel_tol=1e-6)
        assert math.isclose(a["eval_return"], b["eval_return"], rel_tol=1e-5) and a["eval_len"] == b["eval_len"]


def _per_rank_worker(rank, world, port, q, ack):
    import datetime

    import torch
    import torch.distributed as dist
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        import learn
        pol, hist, best, _ = learn.train(n_envs=64, n_steps=8, total_timesteps=2 * 128 * 8, minibatch=512, epochs=2,
                                         eval_every=1, log=lambda *a: None, device=torch.device("cuda:0"),
                                         world=world, rank=rank)
        flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu()
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        if rank == 0:
            q.put((hist, best, all(torch.equal(allp[0], x) for x in allp[1:])))
            ack.wait(60)
    finally:
        dist.destroy_process_group()


def test_ppo_per_rank_learners_two_ranks():
    """examples/learn.py --gpus 2 --learner per-rank (SURVEY §8(e)'s alternative): every rank
    steps its own 64-env shard and trains on it, gradients averaged by one all-reduce per
    minibatch (gloo, both ranks on this GPU).  Both ranks end with identical weights, the history
    counts both ranks' samples, and rank 0 evaluates."""
    import socket

    import torch.multiprocessing as mp
    from tests.test_gpu_dist import _collect
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ack = ctx.Event()
    procs = [ctx.Process(target=_per_rank_worker, args=(r, 2, port, q, ack)) for r in range(2)]
    for p in procs:
        p.start()
    hist, best, same = _collect(q, procs, ack=ack)
    assert same
    assert [h["timesteps"] for h in hist] == [2 * 64 * 8, 2 * 2 * 64 * 8]
    assert all(math.isfinite(h["mean_step_reward"]) and h["eval_len"] >= 1 for h in hist)
    assert math.isfinite(best)


def test_graphed_minibatch_matches_eager():
    """learn.GraphedMinibatch (the PPO minibatch step replayed as one hipGraph) starts from the
    policy's own weights after its capture warm-up, and five replays track five eager steps (the
    train() loop's eager form, torch.distributions and a non-capturable Adam) to f32 rounding."""
    import copy

    import learn
    import torch
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    n_obs, n_act, mb, clip, vf_coef, mgn = 12, 4, 256, 0.2, 0.5, 0.5
    pol_a = learn.ActorCritic(n_obs, n_act).to(dev)
    pol_b = copy.deepcopy(pol_a)
    opt_a = torch.optim.Adam(pol_a.parameters(), lr=3e-4, eps=1e-5)
    opt_b = torch.optim.Adam(pol_b.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    gstep = learn.GraphedMinibatch(pol_b, opt_b, mb, n_obs, n_act, clip, vf_coef, mgn, dev)
    for pa, pb in zip(pol_a.parameters(), pol_b.parameters()):
        assert torch.equal(pa, pb)
    g = torch.Generator(device=dev).manual_seed(3)
    for _ in range(5):
        obs = torch.randn(mb, n_obs, device=dev, generator=g)
        act = torch.randn(mb, n_act, device=dev, generator=g)
        logp_old = torch.randn(mb, device=dev, generator=g) - 4.0
        adv = torch.randn(mb, device=dev, generator=g)
        ret = torch.randn(mb, device=dev, generator=g)
        d = pol_a.dist(obs)
        ratio = (d.log_prob(act).sum(-1) - logp_old).exp()
        ma = (adv - adv.mean()) / (adv.std() + 1e-8)
        pg = -torch.min(ratio * ma, ratio.clamp(1 - clip, 1 + clip) * ma).mean()
        loss = pg + vf_coef * ((pol_a.value(obs) - ret) ** 2).mean()
        opt_a.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(pol_a.parameters(), mgn)
        opt_a.step()
        gstep.step(obs, act, logp_old, adv, ret)
    torch.cuda.synchronize()
    for pa, pb in zip(pol_a.parameters(), pol_b.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("multi", [False, True])
def test_ppo_two_iterations_fused(multi):
    """learn.train(fused=True): the rollout as one hipGraph of (policy kernel + gpd_step) x n_steps,
    then the last value and GAE kernels, replayed each PPO iteration."""
    import learn
    policy, hist, best, target = learn.train(multiagent=multi, n_envs=256, n_steps=16, total_timesteps=3 * 256 * 16,
                                             minibatch=1024, epochs=2, eval_every=1, log=lambda *a: None, fused=True)
    assert len(hist) == 3
    for h in hist:
        assert math.isfinite(h["mean_step_reward"]) and h["eval_len"] >= 1


@pytest.mark.parametrize("multi", [False, True])
def test_fused_rollout_matches_torch_rollout(multi):
    """FusedRollout against train()'s eager torch rollout fed the kernel's own sampled actions
    (Philox draws, not torch's generator): the env trajectory, observations and done flags are
    bit-identical; values, log-probabilities, bootstrapped rewards, advantages and returns agree to
    f32 rounding of the MLP (the kernel sums the 64-wide dot products in another order)."""
    import learn
    import torch
    from gym_pybullet_drones_routing_amd.enums import Physics
    dev = torch.device("cuda:0")
    E, T, gamma, lam = 256, 80, 0.99, 0.95
    env = learn.make_env(multi, E, learn.DEFAULT_ACT, Physics.PYB, dev)
    sim = env.sim
    n_obs, n_act = sim.drones_per_env * sim.obs_width, sim.drones_per_env * sim.act_width
    torch.manual_seed(1)
    pol = learn.ActorCritic(n_obs, n_act).to(dev)
    with torch.no_grad():
        pol.log_std.fill_(0.3)
        pol.pi[4].bias.fill_(1.5)                   # climbing at +5 % thrust: z > 2 truncates after ~60 steps
    env.reset()
    blob, pack0 = sim.save_state(), sim.out_pack.clone()
    bufs = {n: torch.zeros((T, E) + s, device=dev) for n, s in
            (("obs", (n_obs,)), ("act", (n_act,)), ("logp", ()), ("val", ()), ("rew", ()), ("done", ()),
             ("adv", ()), ("ret", ()))}
    fr = learn.FusedRollout(pol, env, T, gamma, lam, 7, bufs)
    with torch.no_grad():
        fr._seq()                                   # eager launches (the graph is tested in test_gpu_policy)
    torch.cuda.synchronize()
    sim.load_state(blob)
    sim.out_pack.copy_(pack0)
    obs = sim.obs.view(E, n_obs).clone()
    ref = {n: torch.zeros_like(b) for n, b in bufs.items()}
    with torch.no_grad():
        for t in range(T):
            d = pol.dist(obs)
            a = bufs["act"][t]                      # the kernel's draw
            v = pol.value(obs)
            o2, r, done, info = env.step(a.clamp(-1, 1))
            trunc = info["TimeLimit.truncated"]
            tv = pol.value(info["terminal_observation"].reshape(E, -1))
            r = r + gamma * tv * trunc.float()
            ref["obs"][t], ref["logp"][t], ref["val"][t] = obs, d.log_prob(a).sum(-1), v
            ref["rew"][t], ref["done"][t] = r, done.float()
            obs = o2.reshape(E, -1)
        last_v = pol.value(obs)
        g = torch.zeros(E, device=dev)
        for t in reversed(range(T)):
            nv = last_v if t == T - 1 else ref["val"][t + 1]
            nonterm = 1.0 - ref["done"][t]
            delta = ref["rew"][t] + gamma * nv * nonterm - ref["val"][t]
            g = delta + gamma * lam * nonterm * g
            ref["adv"][t] = g
        ref["ret"] = ref["adv"] + ref["val"]
    assert float(ref["done"].sum()) > 0
    assert torch.equal(bufs["obs"], ref["obs"]) and torch.equal(bufs["done"], ref["done"])
    for n in ("val", "logp", "rew"):
        torch.testing.assert_close(bufs[n], ref[n], rtol=1e-5, atol=1e-5, msg=n)
    for n in ("adv", "ret"):
        torch.testing.assert_close(bufs[n], ref[n], rtol=1e-4, atol=1e-4, msg=n)
    env.close()
