"""World-size-2 gloo test of the multi-GPU path (gym_pybullet_drones_routing_amd.shard) on CPU.

Each rank steps its env shard (the C oracle stands in for the per-GPU HIP sim, since this
suite has no GPU) and all-gathers the observations; the gathered batch must equal one process
stepping all envs, and the max-over-ranks timing helper must return the global max."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _OracleShard:
    """Adapter: C oracle with the sim's step() signature, returning torch tensors."""

    def __init__(self, n_envs):
        from oracle.c_oracle import COracle
        self.o = COracle(n_envs=n_envs, task="hover", threads=1)

    def step(self, actions):
        obs, rew, te, tr = self.o.step(actions.numpy())
        return (torch.from_numpy(obs.copy()), torch.from_numpy(rew.copy()),
                torch.from_numpy(te.astype(np.uint8)), torch.from_numpy(tr.astype(np.uint8)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, E, T, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gym_pybullet_drones_routing_amd.shard import ShardedStepper, env_shard, max_over_ranks
        start, count = env_shard(E, rank, world)
        stepper = ShardedStepper(_OracleShard(count), E)
        rng = np.random.default_rng(0)
        acts = torch.from_numpy(rng.uniform(-1, 1, (T, E, 1, 4)).astype(np.float32))
        outs = []
        for t in range(T):
            obs, rew, te, tr = stepper.step(acts[t])
            outs.append((obs.numpy().copy(), rew.numpy().copy(), te.numpy().copy(), tr.numpy().copy()))
        mx = max_over_ranks(float(rank + 1))
        if rank == 0:
            q.put((outs, mx, start, count))
    finally:
        dist.destroy_process_group()


def test_sharded_step_and_gather_gloo():
    from oracle.c_oracle import COracle
    E, T, world = 8, 30, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, E, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs, mx, start, count = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (start, count) == (0, 4) and mx == 2.0
    ref = COracle(n_envs=E, task="hover", threads=1)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (T, E, 1, 4)).astype(np.float32)
    for t in range(T):
        o, r, te, tr = ref.step(acts[t])
        np.testing.assert_array_equal(outs[t][0], o)
        np.testing.assert_array_equal(outs[t][1], r)
        np.testing.assert_array_equal(outs[t][2].astype(bool), te)
        np.testing.assert_array_equal(outs[t][3].astype(bool), tr)


def test_env_shard_split():
    from gym_pybullet_drones_routing_amd.shard import env_shard
    assert [env_shard(32768, r, 8) for r in (0, 7)] == [(0, 4096), (28672, 4096)]
    with pytest.raises(ValueError):
        env_shard(10, 0, 3)


class _PackedOracleShard:
    """C oracle with the HIP sim's output pack (sim.pack_layout): what LearnerHandoff gathers."""

    def __init__(self, n_envs, drones_per_env=1, **kw):
        from gym_pybullet_drones_routing_amd.sim import pack_layout
        from oracle.c_oracle import COracle
        self.o = COracle(n_envs=n_envs, drones_per_env=drones_per_env, threads=1, **kw)
        self.n_envs, self.drones_per_env, self.obs_width = n_envs, drones_per_env, self.o.W
        self.act_width = self.o.A
        self.pack_layout = pack_layout(n_envs, drones_per_env, self.o.W)
        self.out_pack = torch.zeros((self.pack_layout["total"],), dtype=torch.uint8)

    def _put(self, name, arr):
        off, n = self.pack_layout[name]
        self.out_pack[off:off + n] = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1))

    def reset(self):
        self._put("obs", self.o.reset())

    def step(self, actions, terminal_obs=True):
        self.o.step(actions.numpy())
        for name in ("obs", "reward", "terminated", "truncated", "terminal_obs"):
            self._put(name, getattr(self.o, name))


def _handoff_worker(rank, world, port, E, T, q, mode, force, ack, cap=None, D=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gym_pybullet_drones_routing_amd.shard import LearnerHandoff, env_shard
        _, count = env_shard(E, rank, world)
        task = "hover" if D == 1 else "multihover"
        h = LearnerHandoff(_PackedOracleShard(count, drones_per_env=D, task=task), E, mode=mode,
                           force_collectives=force, terminal_capacity=cap)
        rng = np.random.default_rng(1)
        acts = rng.uniform(-1, 1, (T, E, D, 4)).astype(np.float32)
        acts[:, :2] *= 0.05                          # long-lived envs beside ones that end early
        o0 = h.reset()
        outs = [o0.numpy().copy() if o0 is not None else None]
        ptrs = None
        for t in range(T):
            # only the learner holds the action batch
            r = h.step(torch.from_numpy(acts[t]) if rank == 0 else None)
            receives = rank == 0 or mode == "all_gather"
            assert (r is None) == (not receives)
            if r is not None:                       # the hand-off's own buffers, allocated once
                p = [x.data_ptr() for x in r]
                assert ptrs is None or p == ptrs
                ptrs = p
            if rank == 0:
                outs.append(tuple(x.numpy().copy() for x in r))
        if rank == 0:
            q.put((outs, h.bytes_per_step(), h.stats()))
            ack.wait(120)          # stay alive until the parent has read the whole message
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,force,cap,D,E", [(2, "all_gather", False, None, 1, 8), (2, "gather", False, None, 1, 8),
                                                      (1, "all_gather", True, None, 1, 8), (1, "gather", True, None, 1, 8),
                                                      (1, "all_gather", False, None, 1, 8), (2, "gather", False, 1, 1, 8),
                                                      (2, "all_gather", False, 1, 1, 8), (2, "gather", False, None, 2, 8),
                                                      (2, "all_gather", False, 1, 2, 8), (2, "gather", False, None, 1, 6),
                                                      (2, "all_gather", False, None, 1, 6)])
def test_learner_handoff_gloo_matches_one_process(world, mode, force, cap, D, E):
    """Rank-0 learner scatters actions, shards step, the output-pack prefixes are gathered (or
    all-gathered) with the terminal rows' 12 state columns per drone (the history columns are the
    auto-reset obs's) - in the prefix's own record with the default capacity, in compacted blocks
    after it with a smaller one: the learner's batch (incl. terminal rows after auto-resets) equals
    one process stepping all envs, bit for bit, for single-drone and 2-drone MultiHover envs, and for
    shards of 3 envs (field offsets that are not multiples of 4 before alignment: ADVICE r5).
    World size 1 with and without forced collectives.  The returned tensors are the hand-off's own
    buffers, the same every step (allocated once).  With a
    terminal_capacity below the shard size (1 or 2 rows: the batch overflows it on many steps) no
    row is dropped: a second exchange carries the rest in the same step."""
    from oracle.c_oracle import COracle
    T = 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ack = ctx.Event()
    port = _free_port()
    procs = [ctx.Process(target=_handoff_worker, args=(r, world, port, E, T, q, mode, force, ack, cap, D))
             for r in range(world)]
    for p in procs:
        p.start()
    outs, (act_bytes, pack_bytes), stats = q.get(timeout=300)
    ack.set()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert act_bytes == E * D * 4 * 4 and pack_bytes == world * _prefix_bytes(E // world, D)
    ref = COracle(n_envs=E, drones_per_env=D, task="hover" if D == 1 else "multihover", threads=1)
    np.testing.assert_array_equal(outs[0], ref.reset())
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (T, E, D, 4)).astype(np.float32)
    acts[:, :2] *= 0.05
    n_done, n_over, extra_rows = 0, 0, 0
    per = E // world
    C = per if cap is None else cap
    for t in range(T):
        o, r, te, tr = ref.step(acts[t])
        obs, rew, gte, gtr, tobs = outs[t + 1]
        np.testing.assert_array_equal(obs, o)
        np.testing.assert_array_equal(rew, r)
        np.testing.assert_array_equal(gte.astype(bool), te)
        np.testing.assert_array_equal(gtr.astype(bool), tr)
        done = te | tr
        n_done += int(done.sum())
        # every finished env's terminal row arrives, whatever the capacity
        np.testing.assert_array_equal(tobs[done], ref.terminal_obs[done])
        assert not tobs[~done].any()                  # only finished envs' rows
        most = max(int(done[rk * per:(rk + 1) * per].sum()) for rk in range(world))
        n_over += most > C
        extra_rows += max(0, most - C)
    assert n_done > 0
    if cap is not None:
        assert n_over > 0 and stats["second_exchanges"] == n_over      # the overflow really happened
    # terminal bytes: a block of C rows of 12 state columns per rank and step, plus the second
    # exchanges' rows (sized by the largest finished count)
    assert stats["terminal_bytes_avg"] * T == world * (C * T + extra_rows) * D * 12 * 4


def _prefix_bytes(e, d=1):
    from gym_pybullet_drones_routing_amd.sim import pack_layout
    return pack_layout(e, d, 72)["prefix"]


def _learner_worker(rank, world, port, q, ack):
    """examples/learn.py --learner per-rank, the learner half: rank-local init (different seeds),
    broadcast_params, a rank-local loss, sync_grads, clip + Adam as train() does."""
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
        import learn
        torch.manual_seed(100 + rank)                    # deliberately different initialisations
        pol = learn.ActorCritic(6, 2)
        learn.broadcast_params(pol)
        flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
        opt = torch.optim.Adam(pol.parameters(), lr=1e-3, eps=1e-5)
        g = torch.Generator().manual_seed(7 + rank)      # rank-local batches
        out = []
        for _ in range(3):
            obs = torch.randn(32, 6, generator=g)
            act = torch.randn(32, 2, generator=g)
            loss = -pol.dist(obs).log_prob(act).sum(-1).mean() + (pol.value(obs) ** 2).mean()
            opt.zero_grad(set_to_none=True)
            loss.backward()
            local = torch.cat([p.grad.reshape(-1) for p in pol.parameters()])
            allg = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(allg, local)
            learn.sync_grads(pol.parameters(), world)
            synced = torch.cat([p.grad.reshape(-1) for p in pol.parameters()])
            out.append((torch.stack(allg).mean(0), synced))
            torch.nn.utils.clip_grad_norm_(pol.parameters(), 0.5)
            opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
        pars = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(pars, flat)
        f0 = [torch.zeros_like(flat0) for _ in range(world)]
        dist.all_gather(f0, flat0)
        if rank == 0:
            q.put((out, pars, f0))
            ack.wait(60)          # keep the queue's feeder alive until the parent has read it
        dist.barrier()            # neither rank tears the group down while the other still uses it
    finally:
        dist.destroy_process_group()


def test_per_rank_learners_stay_in_sync_gloo():
    """SURVEY §8(e)'s alternative hand-off: a PPO learner per rank.  After broadcast_params every
    rank starts from rank 0's weights; sync_grads leaves every rank with the mean of the ranks'
    gradients (one flat all-reduce), so the parameters stay identical through clip + Adam."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ack = ctx.Event()
    procs = [ctx.Process(target=_learner_worker, args=(r, world, port, q, ack)) for r in range(world)]
    for p in procs:
        p.start()
    out, pars, f0 = q.get(timeout=120)
    ack.set()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(f0[0], f0[1])
    for mean, synced in out:
        torch.testing.assert_close(synced, mean, rtol=1e-6, atol=1e-7)
    assert torch.equal(pars[0], pars[1])
    assert not torch.equal(pars[0], f0[0])             # the steps did move the weights
