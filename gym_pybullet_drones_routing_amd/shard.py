"""Env sharding across the GPUs of one node (one process per GPU, torch.distributed / RCCL).

Envs are independent worlds: downwash couples drones only inside an env (the reference runs
one PyBullet client per env, ``BaseAviary.py:170``), so the path partitions with no exchange
at all.  Rank r owns the contiguous env block [r*E/G, (r+1)*E/G).  The only collectives are
the hand-off between a learner on rank 0 and the shards (BASELINE config 5):
``LearnerHandoff`` scatters the learner's action batch to the ranks, each rank steps its shard,
and a gather (one learner) or all-gather (data-parallel learners) of every rank's output-pack
prefix (obs, reward, terminated, truncated) plus the terminal rows of the envs that finished
brings the step back, in rank order, exactly as a single process stepping all E envs would
have produced it (RCCL over xGMI on the GPU box; gloo in the CPU tests).
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
    3. the pack PREFIX (obs | reward | terminated | truncated) of every rank goes to the learner:
       ``mode="gather"`` (one learner: ``dist.gather`` to rank 0, G x prefix bytes land there
       only) or ``mode="all_gather"`` (data-parallel learners: ``all_gather_into_tensor``, the
       batch lands on every rank);
    4. terminal rows (``terminal_obs=True``): only their 12 state columns travel.  The reference
       never clears the action buffer on reset (``BaseRLAviary`` has no ``reset`` override, SURVEY
       a13), so a finished env's terminal observation and its auto-reset observation share the 15
       history columns; the receiving ranks rebuild the terminal row from the gathered obs (48 B per
       drone instead of 288 B with RPM actions).  With the default capacity (the shard's env count)
       nothing is compacted: every env's state columns ride in the prefix's own record (ONE
       collective per step, E*D*48 extra bytes per rank) and the receivers keep the finished envs'
       rows; every size is fixed and nothing waits for the device (round 3 sized the exchange from
       the done counts, two host syncs per step, each longer than the ~5 us step).  A smaller
       ``terminal_capacity`` compacts the state columns of the envs that finished this step on the
       device (a prefix sum over the done flags, ``index_copy_``) into a block of that many rows,
       exchanged after the prefix; the receivers place row j of rank r at rank r's j-th finished
       env.  It never drops a row: an all-reduce of the largest finished count follows (read on the
       host - one synchronisation per step, the price of the smaller block), and when some rank
       finished more envs than the capacity a second exchange of exactly the missing rows runs in
       the same step.
    ``step`` returns (obs [E, D, W], reward [E], terminated [E], truncated [E], terminal_obs or
    None) - freshly allocated tensors, so a caller may keep them across steps - on the learner
    rank ("gather") or every rank ("all_gather"), None elsewhere.  Rows of ``terminal_obs`` whose
    env did not finish are zero.  ``force_collectives=True`` runs the collectives even in a
    one-rank group (the RCCL path on a one-GPU box; otherwise a one-rank hand-off is a local copy).
    With gloo (CPU tests, one-GPU rehearsals) the same exchange runs through host memory."""

    MODES = ("all_gather", "gather")
    STATE_COLS = 12    # KIN observation: pos, rpy, vel, ang_v (BaseRLAviary.py:313-316) before the history

    def __init__(self, sim, global_envs, learner_rank=0, terminal_obs=True, mode="all_gather",
                 force_collectives=False, terminal_capacity=None):
        if mode not in self.MODES:
            raise ValueError(f"mode must be one of {self.MODES}")
        self.sim = sim
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.learner = learner_rank
        self.mode = mode
        self.start, self.count = env_shard(global_envs, self.rank, self.world)
        if sim.n_envs != self.count:
            raise ValueError(f"rank {self.rank} sim has {sim.n_envs} envs, its shard is {self.count}")
        self.global_envs = global_envs
        self.terminal_obs = terminal_obs
        L = sim.pack_layout
        self.layout = L
        self.nbytes = L["prefix"]
        self.row_bytes = sim.drones_per_env * sim.obs_width * 4
        dev = sim.out_pack.device
        self.device = dev
        self._gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        self._coll = dist.is_initialized() and (self.world > 1 or force_collectives)
        D, A = sim.drones_per_env, sim.act_width
        self.local_actions = torch.empty((self.count, D, A), dtype=torch.float32, device=dev)
        C = self.count if terminal_capacity is None else int(terminal_capacity)
        if not 1 <= C <= self.count:
            raise ValueError(f"terminal_capacity must be in [1, {self.count}]")
        self.capacity = C
        W = sim.obs_width
        if W < self.STATE_COLS:
            raise ValueError(f"observation rows of width {W} have no {self.STATE_COLS} state columns")
        S = self.STATE_COLS
        # the default capacity (the whole shard) needs no compaction: every env's 12 state columns
        # ride in the same exchange as the pack prefix (one collective per step); a smaller capacity
        # compacts the finished envs' columns into a block (+ one scratch row that the envs still
        # running write to) exchanged on its own
        self._fused = terminal_obs and C == self.count
        self.sbytes = self.count * D * S * 4 if self._fused else 0
        self.rec = self.nbytes + self.sbytes          # bytes of one rank's record in the exchange
        self._send = torch.empty((self.rec,), dtype=torch.uint8, device=dev) if self._fused else None
        self.pack_all = torch.empty((self.world * self.rec,), dtype=torch.uint8, device=dev)
        if not self._fused:
            self._tblock = torch.zeros((self.count + 1, D * S), dtype=torch.float32, device=dev)
            self._trows = torch.zeros((self.world * C, D * S), dtype=torch.float32, device=dev)
        self.terminal_bytes = 0     # terminal-row bytes received by the learner so far (all steps)
        self.second_exchanges = 0   # steps that needed the overflow exchange (capacity < shard)
        self.finished = 0           # finished envs seen (receiving ranks; counted only with a capacity < shard)
        self.steps = 0

    @property
    def is_learner(self):
        return self.rank == self.learner

    @property
    def receives(self):
        return self.mode == "all_gather" or self.is_learner

    def bytes_per_step(self):
        """(action bytes scattered, prefix bytes landing per step: on every rank for
        "all_gather", on the learner for "gather")."""
        return (self.global_envs * self.sim.drones_per_env * self.sim.act_width * 4,
                self.world * self.nbytes)

    def stats(self):
        """Bytes per step of each part of the hand-off (learner side), averaged over the steps."""
        act_b, pre_b = self.bytes_per_step()
        return {"mode": self.mode, "action_bytes": act_b, "prefix_bytes": pre_b,
                "terminal_bytes_avg": self.terminal_bytes / max(1, self.steps),
                "terminal_row_bytes": self.sim.drones_per_env * self.STATE_COLS * 4,
                "terminal_capacity": self.capacity, "second_exchanges": self.second_exchanges,
                "lands_on": "every rank" if self.mode == "all_gather" else "learner"}

    # ------------------------------------------------------------------ collectives
    def _scatter_actions(self, global_actions):
        if not self._coll:
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

    def _gather_prefix(self, with_state=False):
        """The pack prefix of every rank (and with ``with_state`` its envs' terminal state columns,
        in the same record) -> ``pack_all`` on the receiving ranks."""
        if not with_state:
            self._exchange(self.sim.out_pack[:self.nbytes], self.pack_all[:self.world * self.nbytes])
            return
        E, D, W, S = self.count, self.sim.drones_per_env, self.sim.obs_width, self.STATE_COLS
        self._send[:self.nbytes].copy_(self.sim.out_pack[:self.nbytes])
        self._send[self.nbytes:].view(torch.float32).view(E, D, S).copy_(
            self._local("terminal_obs", torch.float32, (E, D, W))[:, :, :S])
        self._exchange(self._send, self.pack_all)

    def _field(self, name, dtype, shape, rec=None):
        """Field `name` of every rank's gathered pack, as ONE fresh tensor [G*E, ...]."""
        G, E = self.world, self.count
        rec = self.nbytes if rec is None else rec
        off, n = (self.nbytes, self.sbytes) if name == "state" else self.layout[name]
        out = torch.empty((G, n), dtype=torch.uint8, device=self.device)
        out.copy_(self.pack_all[:G * rec].view(G, rec)[:, off:off + n])
        return out.view(dtype).reshape((G * E,) + shape)

    def _local(self, name, dtype, shape):
        off, n = self.layout[name]
        return self.sim.out_pack[off:off + n].view(dtype).reshape(shape)

    def _exchange(self, local, out):
        """Every rank's block ``local`` [n, ...] -> ``out`` [G * n, ...] on the receiving ranks."""
        if not self._coll:
            out.copy_(local)
            return
        if self.mode == "all_gather":
            if self._gloo:
                host = [torch.empty(tuple(local.shape), dtype=local.dtype) for _ in range(self.world)]
                dist.all_gather(host, local.cpu())
                out.copy_(torch.cat(host))
            else:
                dist.all_gather_into_tensor(out, local.contiguous())
        else:
            if self._gloo:
                host = [torch.empty(tuple(local.shape), dtype=local.dtype) for _ in range(self.world)] \
                    if self.is_learner else None
                dist.gather(local.cpu(), host, dst=self.learner)
                if self.is_learner:
                    out.copy_(torch.cat(host))
            else:
                parts = list(out.view((self.world,) + tuple(local.shape)).unbind(0)) if self.is_learner else None
                dist.gather(local.contiguous(), parts, dst=self.learner)

    def _max_finished(self, ldone):
        """The largest finished-env count of any rank (an all-reduce, read on the host)."""
        n = ldone.sum().to(torch.int64).reshape(1)
        if self._coll:
            if self._gloo:
                n = n.cpu()
            dist.all_reduce(n, op=dist.ReduceOp.MAX)
        return int(n.item())

    def _terminal_rows(self, obs, te, tr):
        """Terminal rows of the envs that finished this step ([G*E, D, W], zero elsewhere) on the
        ranks that receive; None elsewhere, for a ``terminal_capacity`` below the shard size (the
        default capacity rides in the prefix's record, ``step``).  obs / te / tr: the gathered
        batch (receiving ranks)."""
        G, E, D, W = self.world, self.count, self.sim.drones_per_env, self.sim.obs_width
        C, S = self.capacity, self.STATE_COLS
        ldone = (self._local("terminated", torch.uint8, (E,)) | self._local("truncated", torch.uint8, (E,))).bool()
        lrows = self._local("terminal_obs", torch.float32, (E, D, W))[:, :, :S].reshape(E, D * S)
        # compaction: the j-th finished env's state columns -> block row j; the others -> the scratch row E
        j = torch.cumsum(ldone.to(torch.int64), 0) - 1
        self._tblock.index_copy_(0, torch.where(ldone, j, torch.full_like(j, E)), lrows)
        self._exchange(self._tblock[:C], self._trows)
        self.terminal_bytes += G * C * D * S * 4
        # rows past the block follow in a second exchange of exactly their count
        need = self._max_finished(ldone)
        if need > C:
            extra = torch.empty((G * (need - C), D * S), dtype=torch.float32, device=self.device)
            self._exchange(self._tblock[C:need], extra)
            self.terminal_bytes += G * (need - C) * D * S * 4
            self.second_exchanges += 1
        if not self.receives:
            return None
        done_all = (te | tr).bool().reshape(G, E)
        within = torch.cumsum(done_all.to(torch.int64), 1) - 1
        if need > C:
            rows_all = torch.cat([self._trows.view(G, C, D * S), extra.view(G, need - C, D * S)], 1).reshape(G * need, -1)
        else:
            rows_all, need = self._trows, C
        src = torch.arange(G, device=self.device)[:, None] * need + within.clamp(0, need - 1)
        rows = rows_all.index_select(0, src.reshape(-1)).view(G * E, D, S)
        full = torch.cat([rows, obs[:, :, S:]], 2)      # the history columns: the reset obs's (shared)
        out = torch.where(done_all.reshape(-1, 1, 1), full, torch.zeros((), dtype=full.dtype, device=self.device))
        return out

    def _views(self, rec=None):
        """The learner's global batch, reassembled from the gathered packs (rank order)."""
        D, W = self.sim.drones_per_env, self.sim.obs_width
        obs = self._field("obs", torch.float32, (D, W), rec)
        rew = self._field("reward", torch.float32, (), rec)
        te = self._field("terminated", torch.uint8, (), rec)
        tr = self._field("truncated", torch.uint8, (), rec)
        return obs, rew, te, tr

    def reset(self):
        """Reset every shard; the learner receives the global initial observation [E, D, W]."""
        self.sim.reset()
        self._gather_prefix()
        return self._field("obs", torch.float32, (self.sim.drones_per_env, self.sim.obs_width)) \
            if self.receives else None

    def step(self, global_actions=None):
        """One env.step of every env of every rank driven by the learner's ``global_actions``."""
        self._scatter_actions(global_actions)
        self.sim.step(self.local_actions, terminal_obs=self.terminal_obs)
        self.steps += 1
        if self._fused:
            # one exchange: pack prefix + every env's terminal state columns
            self._gather_prefix(with_state=True)
            G, D, S = self.world, self.sim.drones_per_env, self.STATE_COLS
            self.terminal_bytes += G * self.sbytes
            if not self.receives:
                return None
            obs, rew, te, tr = self._views(self.rec)
            state = self._field("state", torch.float32, (D, S), self.rec)
            done = (te | tr).bool().reshape(-1, 1, 1)
            full = torch.cat([state, obs[:, :, S:]], 2)  # the history columns: the reset obs's (shared)
            tobs = torch.where(done, full, torch.zeros((), dtype=full.dtype, device=self.device))
            return obs, rew, te, tr, tobs
        self._gather_prefix()
        if self.receives:
            obs, rew, te, tr = self._views()
        else:
            obs = te = tr = None
        tobs = self._terminal_rows(obs, te, tr) if self.terminal_obs else None
        if not self.receives:
            return None
        return obs, rew, te, tr, tobs
