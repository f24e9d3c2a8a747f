"""Env sharding across the GPUs of one node (one process per GPU, torch.distributed / RCCL).

Envs are independent worlds: downwash couples drones only inside an env (the reference runs
one PyBullet client per env, ``BaseAviary.py:170``), so the path partitions with no exchange
at all.  Rank r owns the contiguous env block [r*E/G, (r+1)*E/G).  The only collective is the
optional hand-off of a step's observations / rewards / done flags to a learner:
``gather_batch`` all-gathers the per-rank blocks in rank order (RCCL all_gather over xGMI on
the GPU box; gloo in the CPU tests), giving every rank the batch exactly as a single process
stepping all E envs would have produced it.
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
