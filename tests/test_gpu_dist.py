"""Config-5 learner hand-off driving the HIP sims: two ranks on one GPU (gloo), each stepping
its own BatchedAviarySim shard through the C ABI, rank 0 scattering the actions and receiving
the all-gathered output packs.  The learner's batch must be bit-identical to ONE sim stepping
all envs (envs are independent worlds, BaseAviary.py:170; caller examples/learn.py:52-94)."""
import datetime
import os
import queue
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _actions(E, T, D, A, seed):
    rng = np.random.default_rng(seed)
    acts = rng.uniform(-1, 1, (T, E, D, A)).astype(np.float32)
    acts[:, : E // 2] *= np.float32(0.05)        # long-lived envs beside ones that end early
    return acts


def _worker(rank, world, port, kw, E, T, q, backend="gloo", mode="all_gather", ack=None, sync_check=False,
            graph_at=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    extra = {"device_id": torch.device("cuda:0")} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60), **extra)
    try:
        from gym_pybullet_drones_routing_amd.shard import LearnerHandoff, env_shard
        from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
        _, count = env_shard(E, rank, world)
        sim = BatchedAviarySim(n_envs=count, device="cuda:0", **kw)
        # a one-rank group runs the real collectives (RCCL on the one-GPU box), not the local copy
        h = LearnerHandoff(sim, E, mode=mode, force_collectives=True)
        if backend == "nccl":
            assert dist.get_backend() == "nccl"
        acts = _actions(E, T, sim.drones_per_env, sim.act_width, 5)
        acts_dev = torch.from_numpy(acts).cuda()
        o0 = h.reset()
        outs = [o0.cpu().numpy() if rank == 0 else None]
        keep = []
        for t in range(T):
            if graph_at is not None and t == graph_at:
                h.capture()                               # every later step replays one hipGraph
            if sync_check and t == 2:
                torch.cuda.synchronize()
                torch.cuda.set_sync_debug_mode("error")   # steady state: no host synchronisation at all
            r = h.step(acts_dev[t] if rank == 0 else None)
            if rank == 0:
                keep.append(tuple(x.clone() for x in r))  # the hand-off's buffers: the next step overwrites them
        torch.cuda.set_sync_debug_mode("default")
        for r in keep:
            outs.append(tuple(x.cpu().numpy() for x in r))
        h.close()
        sim.close()
        if rank == 0:
            q.put(outs)
            if ack is not None:
                ack.wait(120)      # stay alive until the parent has read the whole message
    finally:
        dist.destroy_process_group()


def _collect(q, procs, limit=150, ack=None):
    """Rank 0's result; fails as soon as a rank dies instead of waiting out the collective."""
    for _ in range(limit):
        try:
            outs = q.get(timeout=1)
            break
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead:
                for p in procs:
                    p.kill()
                raise AssertionError(f"a rank exited with {dead}")
    else:
        for p in procs:
            p.kill()
        raise AssertionError("ranks did not finish")
    if ack is not None:
        ack.set()                 # rank 0 may exit now that its message has been read
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return outs


def _run(kw, E, T, world, backend, mode, sync_check=False, graph_at=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ack = ctx.Event()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kw, E, T, q, backend, mode, ack, sync_check, graph_at))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        return _collect(q, procs, ack=ack)
    finally:
        ack.set()


def _check_against_one_sim(outs, kw, E, T):
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    sim = BatchedAviarySim(n_envs=E, device="cuda:0", **kw)
    acts = _actions(E, T, sim.drones_per_env, sim.act_width, 5)
    np.testing.assert_array_equal(outs[0], sim.reset().cpu().numpy())
    n_done = 0
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        obs, rew, gte, gtr, tobs = outs[t + 1]
        np.testing.assert_array_equal(obs, o.cpu().numpy())
        np.testing.assert_array_equal(rew, r.cpu().numpy())
        np.testing.assert_array_equal(gte, te.cpu().numpy())
        np.testing.assert_array_equal(gtr, tr.cpu().numpy())
        done = (gte | gtr).astype(bool)
        n_done += int(done.sum())
        np.testing.assert_array_equal(tobs[done], sim.terminal_obs.cpu().numpy()[done])
        assert not tobs[~done].any()
    sim.close()
    assert n_done > 0


@pytest.mark.parametrize("kw,mode", [
    (dict(task="hover"), "all_gather"),
    (dict(task="hover"), "gather"),
    (dict(task="multihover", drones_per_env=4, aero=("dw", "gnd", "drag")), "all_gather"),
], ids=["hover", "hover_gather", "multihover4_dw"])
def test_handoff_two_ranks_bit_identical_to_one_sim(kw, mode):
    E, T, world = 64, 260, 2          # 260 ctrl steps: past the 242-step time truncation
    outs = _run(kw, E, T, world, "gloo", mode)
    _check_against_one_sim(outs, kw, E, T)


@pytest.mark.parametrize("mode,graph_at", [("all_gather", None), ("gather", None), ("all_gather", 5), ("gather", 5)],
                         ids=["all_gather", "gather", "all_gather_graph", "gather_graph"])
def test_handoff_rccl_one_rank(mode, graph_at):
    """The RCCL code path of the hand-off (backend "nccl" = RCCL on ROCm) on the one-GPU box:
    a one-rank group with the collectives forced on, so that the action send / recv, the record
    gather (grouped ncclSend / ncclRecv) / ncclAllGather through rccl.RcclComm and the pack /
    unpack kernels really execute on RCCL.  Bit-identical to one sim stepping the
    same envs.  Steady-state steps run under torch.cuda.set_sync_debug_mode("error"): the
    hand-off never waits for the device.  ``graph_at``: from that step on, every step replays ONE
    captured hipGraph (scatter + step + pack + collective + unpack)."""
    kw = dict(task="hover")
    E, T = 64, 260
    outs = _run(kw, E, T, 1, "nccl", mode, sync_check=True, graph_at=graph_at)
    _check_against_one_sim(outs, kw, E, T)


@pytest.mark.parametrize("W,D", [(72, 1), (27, 2), (36, 3)])
def test_handoff_pack_unpack_kernels_match_host_restatement(W, D):
    """gpd_handoff_pack / gpd_handoff_unpack (csrc/gpd_handoff.h) against their torch
    restatement (shard._pack_host / _unpack_host) on random packs of 3 ranks: float4 rows
    (W % 4 == 0) and scalar rows, shards of 5 envs (unaligned field ends), random done flags."""
    import ctypes
    from gym_pybullet_drones_routing_amd import _lib
    from gym_pybullet_drones_routing_amd.shard import _pack_host, _unpack_host
    from gym_pybullet_drones_routing_amd.sim import pack_layout
    lib = _lib.load()
    G, E = 3, 5
    L = pack_layout(E, D, W)
    cl = _lib.PackLayout()
    _lib.check("gpd_pack_layout_of", lib.gpd_pack_layout_of(E, D, W, ctypes.byref(cl)))
    for k in ("prefix", "prefix_aligned", "record", "total"):
        assert getattr(cl, k) == L[k]
    for k in ("obs", "reward", "terminated", "truncated", "terminal_state", "terminal_obs"):
        assert getattr(cl, k) == L[k][0]
    g = torch.Generator().manual_seed(W)
    packs = []
    for r in range(G):
        p = torch.randint(0, 256, (L["total"],), dtype=torch.uint8, generator=g)
        for name in ("terminated", "truncated"):
            off, n = L[name]
            p[off:off + n] = (torch.rand(n, generator=g) < 0.4).to(torch.uint8)
        packs.append(p)
    # pack on the device vs the host restatement, rank by rank
    ref_packs = [p.clone() for p in packs]
    for p in ref_packs:
        _pack_host(p, L, E, D, W)
    dev_packs = [p.cuda() for p in packs]
    for p in dev_packs:
        _lib.check("gpd_handoff_pack", lib.gpd_handoff_pack(p.data_ptr(), ctypes.byref(cl), None))
    for p, q in zip(dev_packs, ref_packs):
        assert torch.equal(p.cpu(), q)
    rec = L["record"]
    gathered = torch.cat([q[:rec] for q in ref_packs])
    outs_ref = (torch.empty((G * E, D, W)), torch.empty(G * E), torch.empty(G * E, dtype=torch.uint8),
                torch.empty(G * E, dtype=torch.uint8), torch.empty((G * E, D, W)))
    _unpack_host(gathered, G, rec, L, E, D, W, *outs_ref)
    outs = [torch.full(tuple(o.shape), 7, dtype=o.dtype, device="cuda") for o in outs_ref]
    gd = gathered.cuda()
    _lib.check("gpd_handoff_unpack", lib.gpd_handoff_unpack(gd.data_ptr(), G, rec, ctypes.byref(cl),
                                                             *[o.data_ptr() for o in outs], None))
    torch.cuda.synchronize()
    for o, r in zip(outs, outs_ref):
        # bit patterns: random bytes hold NaNs, which compare unequal as floats
        assert torch.equal(o.cpu().view(torch.uint8), r.view(torch.uint8))
    # a stride that is neither record nor prefix_aligned, or terminal rows without records: rejected
    assert lib.gpd_handoff_unpack(gd.data_ptr(), G, rec + 256, ctypes.byref(cl), *[o.data_ptr() for o in outs],
                                  None) == _lib.GPD_EINVAL
    assert lib.gpd_handoff_unpack(gd.data_ptr(), G, L["prefix_aligned"], ctypes.byref(cl),
                                  *[o.data_ptr() for o in outs], None) == _lib.GPD_EINVAL


def _fused_rollout_worker(port, q, ack):
    """One-rank RCCL group: examples/learn.py's FusedRollout over ShardedAviaryVecEnv (graph=True,
    collectives forced: the hand-off's RCCL send / recv and gather inside the captured rollout)
    against FusedRollout over one AviaryVecEnv with the same policy and Philox key."""
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                            timeout=datetime.timedelta(seconds=60))
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
        import learn
        from gym_pybullet_drones_routing_amd.envs.vec_env import AviaryVecEnv, ShardedAviaryVecEnv
        from gym_pybullet_drones_routing_amd.enums import ActionType, Physics
        E, T = 256, 16
        kw = dict(task="hover", act=ActionType.ONE_D_RPM, physics=Physics.PYB, device=dev, output="torch")
        torch.manual_seed(3)
        pol = learn.ActorCritic(27, 1).to(dev)
        with torch.no_grad():
            pol.log_std.fill_(0.5)
            pol.pi[4].bias.fill_(1.5)               # climbing: z > 2 truncations (bootstraps) after ~60 steps
        outs = []
        for env in (AviaryVecEnv(E, **kw), ShardedAviaryVecEnv(E, graph=True, force_collectives=True, **kw)):
            env.reset()
            bufs = {n: torch.zeros((T, E) + sh, device=dev) for n, sh in
                    (("obs", (27,)), ("act", (1,)), ("logp", ()), ("val", ()), ("rew", ()), ("done", ()),
                     ("adv", ()), ("ret", ()))}
            fr = learn.FusedRollout(pol, env, T, 0.99, 0.95, 11, bufs)
            got = []
            for _ in range(5):                      # capture + replay, then four more replays
                fr.run()
                got.append({n: b.cpu().numpy().copy() for n, b in bufs.items()})
            outs.append(got)
            env.close()
        q.put(outs)
        ack.wait(120)          # stay alive until the parent has read the whole message
    finally:
        dist.destroy_process_group()


def test_fused_rollout_over_rccl_handoff():
    """The sharded fused rollout (policy kernel + RCCL hand-off step, n_steps of them in one
    hipGraph per rank) produces bit-identical rollout buffers to the single-sim fused rollout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ack = ctx.Event()
    p = ctx.Process(target=_fused_rollout_worker, args=(_free_port(), q, ack))
    p.start()
    try:
        outs = _collect(q, [p], ack=ack)
    finally:
        ack.set()
    single, sharded = outs
    n_done = 0
    for a, b in zip(single, sharded):
        for n in a:
            np.testing.assert_array_equal(a[n], b[n], err_msg=n)
        n_done += int(a["done"].sum())
    assert n_done > 0
