"""Env sharding across the GPUs of one node (one process per GPU, torch.distributed / RCCL).

Envs are independent worlds: downwash couples drones only inside an env (the reference runs
one PyBullet client per env, ``BaseAviary.py:170``), so the path partitions with no exchange
at all.  Rank r owns the contiguous env block [r*E/G, (r+1)*E/G).  The only collectives are
the hand-off between a learner on rank 0 and the shards (BASELINE config 5):
``LearnerHandoff`` scatters the learner's action batch to the ranks, each rank steps its shard,
and one all-gather of every rank's output pack (obs, reward, terminated, truncated and, when
asked, the terminal rows) brings the step back, in rank order, exactly as a single process
stepping all E envs would have produced it (RCCL over xGMI on the GPU box; gloo in the CPU tests).
The caller being replaced is the reference's stepping loop, ``examples/learn.py:52-94``
(``make_vec_env(..., n_envs=...)`` + PPO), over independent worlds (``BaseAviary.py:170``).
"""
import torch
import torch.distributed as dist


def env_shard(global_envs, rank, world):
    """(first env, env count) of `rank`; the split must be even so all_gather needs no padding."""
    if global_envs % world != 0:
        raise ValueError(f"{global_envs} envs do not split evenly over {world} ranks")
    per = global_envs // world
    return rank * per, per


def rank_seed(base_seed, rank):
    """Per-rank synthetic-input seed (seed = 1000 + rank)."""
    return base_seed + rank


def max_over_ranks(value, device=None):
    """The max of a host float over all ranks (the bench's job time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None            # gloo reduces host tensors
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_batch(local, out=None):
    """All-gather a per-rank block [E_local, ...] into [world * E_local, ...] in rank order."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "gloo" and local.is_cuda:
        # gloo (CPU tests, single-GPU rehearsals): gather through host memory
        parts = [torch.empty_like(local, device="cpu") for _ in range(world)]
        dist.all_gather(parts, local.detach().cpu().contiguous())
        out.copy_(torch.cat(parts))
        return out
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


class ShardedStepper:
    """Steps this rank's env shard and hands the global batch to the learner.

    ``sim`` is any object with ``step(actions) -> (obs, reward, terminated, truncated)`` over the
    local shard (a ``BatchedAviarySim`` on the GPU box); actions arrive as the GLOBAL batch
    [E, ...] (what a learner broadcasts) and each rank slices its block."""

    def __init__(self, sim, global_envs):
        self.sim = sim
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.start, self.count = env_shard(global_envs, self.rank, self.world)
        self.global_envs = global_envs

    def step(self, global_actions, gather=True):
        local = global_actions[self.start:self.start + self.count]
        obs, rew, te, tr = self.sim.step(local)
        if not gather:
            return obs, rew, te, tr
        return (gather_batch(obs), gather_batch(rew), gather_batch(te), gather_batch(tr))


class LearnerHandoff:
    """Rank-0 learner <-> env shards, one step at a time.

    Every rank owns a ``sim`` (``BatchedAviarySim`` over its contiguous env block; any object
    with ``n_envs``, ``drones_per_env``, ``act_width``, ``step()``, ``reset()`` and the output
    pack ``out_pack`` / ``pack_layout`` of ``sim.BatchedAviarySim``).  Per step:

    1. ``scatter`` of the learner's actions [E, D, A] float32 -> each rank's [E/G, D, A]
       (E*D*A*4 bytes leave rank 0 in total);
    2. each rank steps its shard (the kernel writes straight into the output pack);
    3. one ``all_gather_into_tensor`` of the packs (the prefix without terminal rows when
       ``terminal_obs=False``): G * pack bytes land on every rank.

    ``step`` returns (obs [E, D, W], reward [E], terminated [E], truncated [E], terminal_obs or
    None) on the learner rank and None elsewhere.  With gloo (CPU tests, one-GPU rehearsals)
    the same collectives run through host memory."""

    def __init__(self, sim, global_envs, learner_rank=0, terminal_obs=True):
        self.sim = sim
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.learner = learner_rank
        self.start, self.count = env_shard(global_envs, self.rank, self.world)
        if sim.n_envs != self.count:
            raise ValueError(f"rank {self.rank} sim has {sim.n_envs} envs, its shard is {self.count}")
        self.global_envs = global_envs
        self.terminal_obs = terminal_obs
        L = sim.pack_layout
        self.layout = L
        self.nbytes = L["total"] if terminal_obs else L["prefix"]
        dev = sim.out_pack.device
        self._gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        self.pack_all = torch.empty((self.world * self.nbytes,), dtype=torch.uint8, device=dev)
        D, A = sim.drones_per_env, sim.act_width
        self.local_actions = torch.empty((self.count, D, A), dtype=torch.float32, device=dev)

    @property
    def is_learner(self):
        return self.rank == self.learner

    def bytes_per_step(self):
        """(action bytes scattered, pack bytes all-gathered onto every rank) per step."""
        return (self.global_envs * self.sim.drones_per_env * self.sim.act_width * 4,
                self.world * self.nbytes)

    def _scatter_actions(self, global_actions):
        if self.world == 1:
            self.local_actions.copy_(global_actions)
            return
        if self.is_learner:
            ga = global_actions.to(torch.float32).reshape((self.global_envs,) + tuple(self.local_actions.shape[1:]))
            parts = list(ga.chunk(self.world))
        else:
            parts = None
        if self._gloo:
            buf = torch.empty(self.local_actions.shape, dtype=torch.float32)
            dist.scatter(buf, [p.detach().cpu().contiguous() for p in parts] if parts else None, src=self.learner)
            self.local_actions.copy_(buf)
        else:
            dist.scatter(self.local_actions, [p.contiguous() for p in parts] if parts else None, src=self.learner)

    def _gather(self):
        local = self.sim.out_pack[:self.nbytes]
        if self.world == 1:
            self.pack_all.copy_(local)
        elif self._gloo:
            parts = [torch.empty((self.nbytes,), dtype=torch.uint8) for _ in range(self.world)]
            dist.all_gather(parts, local.cpu())
            self.pack_all.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(self.pack_all, local)

    def _views(self):
        """The learner's global batch, reassembled from the gathered packs (rank order)."""
        G, E, D = self.world, self.count, self.sim.drones_per_env
        W = self.sim.obs_width
        packs = self.pack_all.view(G, self.nbytes)

        def field(name, dtype, shape):
            off, n = self.layout[name]
            return packs[:, off:off + n].contiguous().view(dtype).reshape((G * E,) + shape)

        obs = field("obs", torch.float32, (D, W))
        rew = field("reward", torch.float32, ())
        te = field("terminated", torch.uint8, ())
        tr = field("truncated", torch.uint8, ())
        tobs = field("terminal_obs", torch.float32, (D, W)) if self.terminal_obs else None
        return obs, rew, te, tr, tobs

    def reset(self):
        """Reset every shard; the learner receives the global initial observation [E, D, W]."""
        self.sim.reset()
        self._gather()
        return self._views()[0] if self.is_learner else None

    def step(self, global_actions=None):
        """One env.step of every env of every rank driven by the learner's ``global_actions``."""
        self._scatter_actions(global_actions)
        self.sim.step(self.local_actions, terminal_obs=self.terminal_obs)
        self._gather()
        return self._views() if self.is_learner else None
