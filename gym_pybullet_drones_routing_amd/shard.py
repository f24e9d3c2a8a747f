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
    with ``n_envs``, ``drones_per_env``, ``act_width``, ``obs_width``, ``step()``, ``reset()`` and
    the output pack ``out_pack`` / ``pack_layout`` of ``sim.BatchedAviarySim``).  Per step:

    1. the learner's actions [E, D, A] float32 go to the ranks' shards [E/G, D, A] with ONE
       ``all_to_all_single`` (the learner sends a block to every rank, the others send nothing);
    2. each rank steps its shard: the kernel writes obs, reward, the flags and the terminal rows
       straight into the output pack;
    3. ``gpd_handoff_pack`` copies the 12 state columns of the finished envs' terminal rows into the
       pack's ``terminal_state`` field, right behind the flags.  The reference never clears the
       action buffer on reset (``BaseRLAviary`` has no ``reset`` override), so a finished
       env's terminal row and its auto-reset row share the 15 history columns: only the 48 B of
       state per drone travel, not the 288 B row;
    4. ONE collective moves every rank's RECORD (obs | reward | terminated | truncated |
       terminal_state, a prefix of the pack: no copy on the sending side) into ``pack_all``:
       ``mode="gather"`` (one learner: ``all_to_all_single`` with every rank sending its record to
       the learner only - G records land there) or ``mode="all_gather"`` (data-parallel learners:
       ``all_gather_into_tensor``, the batch lands on every rank);
    5. ``gpd_handoff_unpack`` (one kernel) rebuilds the global batch in rank order on the receiving
       ranks: obs [E, D, W], reward [E], terminated / truncated [E] and terminal rows [E, D, W]
       (state columns + the reset row's history for finished envs, zero elsewhere).

    Every buffer is allocated once, in ``__init__``; every size is fixed; nothing waits for the
    device.  ``step`` returns the hand-off's own output tensors (obs, reward, terminated,
    truncated, terminal_obs or None) on the learner ("gather") or every rank ("all_gather"), None
    elsewhere; the next step overwrites them, like ``BatchedAviarySim.step``'s.

    ``capture()`` records steps 1-5 as ONE hipGraph (RCCL collectives are graph-capturable; every
    rank must call it, in the same order as its other collectives); afterwards ``step`` copies the
    actions into the static ``global_actions`` buffer and replays it.  Not with gloo (host
    staging) or a ``terminal_capacity`` below the shard size.

    ``terminal_capacity`` below the shard size (eager only): the record stops after the flags and
    the finished envs' state columns are compacted on the device (prefix sum over the done flags,
    ``index_copy_``) into a block of that many rows, exchanged after it; an all-reduce of the
    largest finished count follows, READ ON THE HOST (one synchronisation per step - this mode
    trades it for the bytes of the unfinished envs' columns) and, when some rank finished more
    envs than the capacity, a second exchange of exactly the missing rows runs in the same step:
    no row is ever dropped.  ``force_collectives=True`` runs the collectives even in a one-rank
    group (the RCCL path on a one-GPU box; otherwise a one-rank hand-off is a local copy).  With
    gloo (CPU tests, one-GPU rehearsals) the same collectives run through host memory.  CPU-resident
    shards (the C oracle standing in for the sim in the CPU tests) are packed and unpacked by the
    torch restatement of the two kernels (``_pack_host`` / ``_unpack_host``)."""

    MODES = ("all_gather", "gather")
    STATE_COLS = 12    # KIN observation: pos, rpy, vel, ang_v (BaseRLAviary.py:313-316) before the history

    def __init__(self, sim, global_envs, learner_rank=0, terminal_obs=True, mode="all_gather",
                 force_collectives=False, terminal_capacity=None, transport="rccl"):
        if mode not in self.MODES:
            raise ValueError(f"mode must be one of {self.MODES}")
        if transport not in ("rccl", "torch"):
            raise ValueError("transport must be 'rccl' (a raw RCCL communicator) or 'torch' (the process group)")
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
        G, E, D, W, A, S = self.world, self.count, sim.drones_per_env, sim.obs_width, sim.act_width, self.STATE_COLS
        if W < S:
            raise ValueError(f"observation rows of width {W} have no {S} state columns")
        L = sim.pack_layout
        self.layout = L
        self.nbytes = L["prefix"]
        dev = sim.out_pack.device
        self.device = dev
        self._host = dev.type == "cpu"
        self._gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        self._stage = self._gloo and not self._host       # gloo moves host tensors only
        self._coll = dist.is_initialized() and (self.world > 1 or force_collectives)
        # RCCL groups: the step's collectives go through a raw RCCL communicator (rccl.RcclComm:
        # ~1 us host calls, capturable) unless transport="torch"; gloo keeps the process group
        self._rc = None
        if self._coll and not self._gloo and transport == "rccl":
            from .rccl import RcclComm
            self._rc = RcclComm(dev)
        self.transport = "rccl" if self._rc is not None else ("gloo" if self._gloo else "torch")
        C = E if terminal_capacity is None else int(terminal_capacity)
        if not 1 <= C <= E:
            raise ValueError(f"terminal_capacity must be in [1, {E}]")
        self.capacity = C
        # with the default capacity every env's state columns ride in the record (one collective)
        self._fused = terminal_obs and C == E
        self.rec = L["record"] if self._fused else L["prefix_aligned"]
        self.sbytes = L["terminal_state"][1] if self._fused else 0
        if not self._host:
            from . import _lib
            self._lib = _lib.load()
            self._clayout = _lib.PackLayout()
            _lib.check("gpd_pack_layout_of", self._lib.gpd_pack_layout_of(E, D, W, self._clayout))
            for k in ("record", "prefix_aligned", "total"):
                if getattr(self._clayout, k) != L[k]:
                    raise RuntimeError(f"pack layout {k}: gpd_pack_layout_of {getattr(self._clayout, k)} != {L[k]}")
        # ---- every buffer, once
        f32, u8 = torch.float32, torch.uint8
        self.global_actions = torch.zeros((global_envs, D, A), dtype=f32, device=dev) if self.is_learner else None
        self.local_actions = torch.empty((E, D, A), dtype=f32, device=dev)
        self._empty_f32 = torch.empty((0,), dtype=f32, device=dev)
        self._empty_u8 = torch.empty((0,), dtype=u8, device=dev)
        self.pack_all = torch.empty((G * self.rec,) if self.receives else (0,), dtype=u8, device=dev)
        Eg = G * E
        self.obs = torch.empty((Eg, D, W), dtype=f32, device=dev) if self.receives else None
        self.reward = torch.empty((Eg,), dtype=f32, device=dev) if self.receives else None
        self.terminated = torch.empty((Eg,), dtype=u8, device=dev) if self.receives else None
        self.truncated = torch.empty((Eg,), dtype=u8, device=dev) if self.receives else None
        self.terminal_rows = torch.zeros((Eg, D, W), dtype=f32, device=dev) \
            if (self.receives and terminal_obs) else None
        self._record = sim.out_pack[:self.rec]
        if self._stage:
            self._h_send = torch.empty((self.rec,), dtype=u8).pin_memory()
            self._h_all = torch.empty(tuple(self.pack_all.shape), dtype=u8).pin_memory()
            self._h_local_act = torch.empty((E * D * A,), dtype=f32).pin_memory()
            self._h_global_act = torch.empty((global_envs * D * A,), dtype=f32).pin_memory() \
                if self.is_learner else self._empty_f32.cpu()
        if not self._fused and terminal_obs:
            self._tblock = torch.zeros((E + 1, D * S), dtype=f32, device=dev)
            self._trows = torch.zeros((G * C, D * S), dtype=f32, device=dev)
        # split sizes of the two all_to_all_single calls (elements along dim 0 of flat tensors)
        n_act = E * D * A
        self._act_in_splits = [n_act] * G if self.is_learner else [0] * G
        self._act_out_splits = [n_act if r == self.learner else 0 for r in range(G)]
        self._graph = None
        self.terminal_bytes = 0     # terminal-state bytes received by the learner so far (all steps)
        self.second_exchanges = 0   # steps that needed the overflow exchange (capacity < shard)
        self.steps = 0

    @property
    def is_learner(self):
        return self.rank == self.learner

    def close(self):
        """Release the captured graph and the RCCL communicator (collective on RCCL groups: every
        rank calls it).  The graph goes first: it holds the communicator's kernels."""
        self._graph = None
        if self._rc is not None:
            self._rc.destroy()
            self._rc = None

    @property
    def receives(self):
        return self.mode == "all_gather" or self.is_learner

    @property
    def host_sync_per_step(self):
        """True for a terminal_capacity below the shard size (the finished count is read on the host)."""
        return self.terminal_obs and not self._fused

    def bytes_per_step(self):
        """(action bytes scattered, prefix bytes landing per step: on every rank for
        "all_gather", on the learner for "gather")."""
        return (self.global_envs * self.sim.drones_per_env * self.sim.act_width * 4,
                self.world * self.nbytes)

    def stats(self):
        """Bytes per step of each part of the hand-off (learner side), averaged over the steps."""
        act_b, pre_b = self.bytes_per_step()
        return {"mode": self.mode, "transport": self.transport, "action_bytes": act_b, "prefix_bytes": pre_b,
                "record_bytes": self.rec, "terminal_bytes_avg": self.terminal_bytes / max(1, self.steps),
                "terminal_row_bytes": self.sim.drones_per_env * self.STATE_COLS * 4,
                "terminal_capacity": self.capacity, "second_exchanges": self.second_exchanges,
                "host_sync_per_step": self.host_sync_per_step, "graphed": self._graph is not None,
                "lands_on": "every rank" if self.mode == "all_gather" else "learner"}

    # ------------------------------------------------------------------ collectives
    def _scatter_actions(self, src):
        """The learner's [E_global, D, A] -> this rank's block (ONE all_to_all_single)."""
        if not self._coll:
            self.local_actions.copy_(src)
            return
        out = self.local_actions.view(-1)
        inp = src.reshape(-1) if self.is_learner else self._empty_f32
        if self._rc is not None:
            self._rc.scatter(inp if self.is_learner else None, out, self.learner)
            return
        if self._stage:
            if self.is_learner:
                self._h_global_act.copy_(inp)
            dist.all_to_all_single(self._h_local_act, self._h_global_act, self._act_out_splits, self._act_in_splits)
            out.copy_(self._h_local_act)
            return
        dist.all_to_all_single(out, inp, self._act_out_splits, self._act_in_splits)

    def _exchange(self, local, out, h_send=None, h_out=None):
        """Every rank's flat block ``local`` [n] -> ``out`` [G * n] on the receiving ranks (rank
        order): all_gather_into_tensor, or all_to_all_single with every rank sending to the learner."""
        if not self._coll:
            out.copy_(local)
            return
        n = local.numel()
        if self._stage:        # gloo and device tensors: through (pinned) host memory
            hs = h_send if h_send is not None else torch.empty((n,), dtype=local.dtype)
            ho = h_out if h_out is not None else torch.empty(tuple(out.shape), dtype=out.dtype)
            hs.copy_(local)
            self._collective(ho, hs, n)
            if self.receives:
                out.copy_(ho)
            return
        self._collective(out, local, n)

    def _collective(self, out, inp, n):
        G = self.world
        if self._rc is not None:
            if self.mode == "all_gather":
                self._rc.all_gather(inp, out)
            else:
                self._rc.gather(inp, out if self.is_learner else None, self.learner)
            return
        if self.mode == "gather" and not self.is_learner:
            out = inp.new_empty((0,))             # the learner receives; the others send only
        if self.mode == "all_gather":
            dist.all_gather_into_tensor(out, inp)
        else:
            dist.all_to_all_single(out, inp, [n] * G if self.is_learner else [0] * G,
                                   [n if r == self.learner else 0 for r in range(G)])

    # ------------------------------------------------------------------ pack / unpack
    def _pack(self):
        if self._host:
            _pack_host(self.sim.out_pack, self.layout, self.count, self.sim.drones_per_env, self.sim.obs_width)
            return
        from . import _lib
        _lib.check("gpd_handoff_pack", self._lib.gpd_handoff_pack(
            self.sim.out_pack.data_ptr(), self._clayout, _cur_stream(self.device)))

    def _unpack(self, with_tobs):
        tobs = self.terminal_rows if with_tobs else None
        if self._host:
            _unpack_host(self.pack_all, self.world, self.rec, self.layout, self.count, self.sim.drones_per_env,
                         self.sim.obs_width, self.obs, self.reward, self.terminated, self.truncated, tobs)
            return
        from . import _lib
        _lib.check("gpd_handoff_unpack", self._lib.gpd_handoff_unpack(
            self.pack_all.data_ptr(), self.world, self.rec, self._clayout, self.obs.data_ptr(),
            self.reward.data_ptr(), self.terminated.data_ptr(), self.truncated.data_ptr(),
            tobs.data_ptr() if tobs is not None else None, _cur_stream(self.device)))

    def _outputs(self):
        if not self.receives:
            return None
        return self.obs, self.reward, self.terminated, self.truncated, self.terminal_rows

    # ------------------------------------------------------------------ steps
    def reset(self):
        """Reset every shard; the learner receives the global initial observation [E, D, W]."""
        self.sim.reset()
        self._exchange(self._record, self.pack_all, *self._stage_bufs())
        if not self.receives:
            return None
        self._unpack(False)
        return self.obs

    def _stage_bufs(self):
        return (self._h_send, self._h_all) if self._stage else (None, None)

    def step_body(self, src):
        """Steps 1-5 of one hand-off step on the current stream (for a caller that captures them
        into its own graph, e.g. examples/learn.py's fused rollout); ``src``: the learner's
        [E, D, A] float32 actions (None elsewhere)."""
        self._step_body(src)

    def _step_body(self, src):
        self._scatter_actions(src)
        self.sim.step(self.local_actions, terminal_obs=self.terminal_obs)
        if self._fused:
            self._pack()
        self._exchange(self._record, self.pack_all, *self._stage_bufs())
        if self.receives:
            self._unpack(self._fused)

    def step(self, global_actions=None):
        """One env.step of every env of every rank driven by the learner's ``global_actions``
        [E, D, A] float32 (ignored on the other ranks)."""
        src = None
        if self.is_learner:
            if global_actions is None:
                raise ValueError("the learner rank must pass the global action batch")
            ga = global_actions
            ok = (isinstance(ga, torch.Tensor) and ga.dtype == torch.float32 and ga.device == self.device
                  and ga.is_contiguous() and ga.numel() == self.global_actions.numel())
            if self._graph is not None or not ok:
                if ga is not self.global_actions:
                    self.global_actions.copy_(torch.as_tensor(ga, dtype=torch.float32).reshape(self.global_actions.shape))
                src = self.global_actions
            else:
                src = ga
        self.steps += 1
        if self._fused:
            self.terminal_bytes += self.world * self.sbytes
        if self._graph is not None:
            self._graph.replay()
            return self._outputs()
        self._step_body(src)
        if self.terminal_obs and not self._fused:
            self._terminal_rows_compacted()
        return self._outputs()

    def capture(self, n_steps=1, install=True):
        """Record ``n_steps`` hand-off steps (action scatter, shard step, pack, exchange, unpack),
        all reading the static ``global_actions``, into ONE hipGraph and return it; with
        ``install`` (n_steps == 1) later ``step`` calls replay it.  Collective: every rank calls it at
        the same point.  Run at least one eager step first (it creates the RCCL communicator, which
        capture cannot).  A graph of several steps is what a caller with the policy inside the same
        graph (bench.py's rollout leg) or an open-loop benchmark replays."""
        if self._host or self._stage:
            raise ValueError("capture() needs device shards on RCCL (gloo stages through host memory)")
        if self.host_sync_per_step:
            raise ValueError("a terminal_capacity below the shard size reads the finished count on the host "
                             "every step: not capturable")
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.device(self.device), torch.cuda.graph(g):
            for _ in range(int(n_steps)):
                self._step_body(self.global_actions if self.is_learner else None)
        if install:
            if n_steps != 1:
                raise ValueError("step() replays a graph of exactly one step")
            self._graph = g
        return g

    # ------------------------------------------------------------------ capacity < shard (eager, synchronising)
    def _local(self, name, dtype, shape):
        off, n = self.layout[name]
        return self.sim.out_pack[off:off + n].view(dtype).reshape(shape)

    def _max_finished(self, ldone):
        """The largest finished-env count of any rank (an all-reduce, read on the host)."""
        n = ldone.sum().to(torch.int64).reshape(1)
        if self._coll:
            if self._gloo:
                n = n.cpu()
            dist.all_reduce(n, op=dist.ReduceOp.MAX)
        return int(n.item())

    def _terminal_rows_compacted(self):
        """Terminal rows of the envs that finished this step into ``terminal_rows`` (receiving
        ranks), for a ``terminal_capacity`` below the shard size."""
        G, E, D, W = self.world, self.count, self.sim.drones_per_env, self.sim.obs_width
        C, S = self.capacity, self.STATE_COLS
        ldone = (self._local("terminated", torch.uint8, (E,)) | self._local("truncated", torch.uint8, (E,))).bool()
        lrows = self._local("terminal_obs", torch.float32, (E, D, W))[:, :, :S].reshape(E, D * S)
        # compaction: the j-th finished env's state columns -> block row j; the others -> the scratch row E
        j = torch.cumsum(ldone.to(torch.int64), 0) - 1
        self._tblock.index_copy_(0, torch.where(ldone, j, torch.full_like(j, E)), lrows)
        self._exchange(self._tblock[:C].reshape(-1), self._trows.view(-1))
        self.terminal_bytes += G * C * D * S * 4
        # rows past the block follow in a second exchange of exactly their count
        need = self._max_finished(ldone)
        if need > C:
            extra = torch.empty((G * (need - C), D * S), dtype=torch.float32, device=self.device)
            self._exchange(self._tblock[C:need].reshape(-1), extra.view(-1))
            self.terminal_bytes += G * (need - C) * D * S * 4
            self.second_exchanges += 1
        if not self.receives:
            return
        done_all = (self.terminated | self.truncated).bool().reshape(G, E)
        within = torch.cumsum(done_all.to(torch.int64), 1) - 1
        if need > C:
            rows_all = torch.cat([self._trows.view(G, C, D * S), extra.view(G, need - C, D * S)], 1).reshape(G * need, -1)
        else:
            rows_all, need = self._trows, C
        src = torch.arange(G, device=self.device)[:, None] * need + within.clamp(0, need - 1)
        rows = rows_all.index_select(0, src.reshape(-1)).view(G * E, D, S)
        out = self.terminal_rows
        out[:, :, :S] = rows
        out[:, :, S:] = self.obs[:, :, S:]      # the history columns: the reset obs's (shared)
        out.masked_fill_(~done_all.reshape(-1, 1, 1), 0.0)


def _cur_stream(device):
    return torch.cuda.current_stream(device).cuda_stream


def _pack_host(pack, L, E, D, W):
    """``handoff_pack_kernel`` (csrc/gpd_handoff.h) on a CPU-resident pack (the CPU tests' oracle shards)."""
    S = LearnerHandoff.STATE_COLS
    done = (_view(pack, L, "terminated", torch.uint8, (E,)) | _view(pack, L, "truncated", torch.uint8, (E,))).bool()
    ts = _view(pack, L, "terminal_state", torch.float32, (E, D, S))
    tobs = _view(pack, L, "terminal_obs", torch.float32, (E, D, W))
    ts[done] = tobs[done][:, :, :S]


def _unpack_host(pack_all, G, stride, L, E, D, W, obs, reward, term, trunc, tobs):
    """``handoff_unpack_kernel`` (csrc/gpd_handoff.h) on CPU-resident records (the CPU tests)."""
    S = LearnerHandoff.STATE_COLS
    for g in range(G):
        rec = pack_all[g * stride:(g + 1) * stride]
        sl = slice(g * E, (g + 1) * E)
        o = _view(rec, L, "obs", torch.float32, (E, D, W))
        obs[sl] = o
        reward[sl] = _view(rec, L, "reward", torch.float32, (E,))
        te, tr = _view(rec, L, "terminated", torch.uint8, (E,)), _view(rec, L, "truncated", torch.uint8, (E,))
        term[sl], trunc[sl] = te, tr
        if tobs is not None:
            done = (te | tr).bool()
            t = tobs[sl]
            t.zero_()
            t[done, :, :S] = _view(rec, L, "terminal_state", torch.float32, (E, D, S))[done]
            t[done, :, S:] = o[done][:, :, S:]


def _view(buf, L, name, dtype, shape):
    off, n = L[name]
    return buf[off:off + n].view(dtype).view(shape)
