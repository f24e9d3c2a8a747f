"""Batched VecEnv view: ``num_envs`` HoverAviary / MultiHoverAviary envs in one HIP launch per step.

The reference reaches its env through stable-baselines3 ``make_vec_env(HoverAviary, n_envs=1)``
(DummyVecEnv, ``examples/learn.py:53-64``).  ``AviaryVecEnv`` is the MI355X replacement for that
whole vector: it implements the SB3 ``VecEnv`` protocol (``reset``, ``step_async``,
``step_wait``, ``num_envs``, spaces, ``get_attr`` ...) with DummyVecEnv's auto-reset semantics
(``infos[i]["terminal_observation"]``, ``infos[i]["TimeLimit.truncated"]``), so SB3 PPO can use it
where stable_baselines3 is installed.  ``output="torch"`` keeps everything in HBM for a
GPU-resident learner (infos become a dict of tensors).
"""
import numpy as np
import torch

from ..enums import ActionType, DroneModel, ObservationType, Physics
from ..sim import BatchedAviarySim
from .spaces import action_space, observation_space


try:  # a real SB3 VecEnv where stable-baselines3 is installed, so PPO(policy, env) takes it as is
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase
except Exception:  # SB3 absent (this image): same protocol, no base class
    _VecEnvBase = object


class AviaryVecEnv(_VecEnvBase):
    def __init__(self, num_envs, task="hover", num_drones=1, drone_model=DroneModel.CF2X, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.DYN, aero=(), pyb_freq=240, ctrl_freq=30,
                 obs=ObservationType.KIN, act=ActionType.RPM, precision="f64", device=None, output="numpy",
                 episode_len_sec=8, urdf_path=None, tuning=None):
        if ObservationType(obs) != ObservationType.KIN:
            raise NotImplementedError("ObservationType.RGB is out of scope")
        if output not in ("numpy", "torch"):
            raise ValueError("output must be 'numpy' or 'torch'")
        if task == "hover" and num_drones != 1:
            raise ValueError("HoverAviary is single-drone")
        self.sim = BatchedAviarySim(n_envs=num_envs, drones_per_env=num_drones, drone_model=drone_model,
                                    urdf_path=urdf_path, pyb_freq=pyb_freq, ctrl_freq=ctrl_freq, act=act,
                                    task=task, physics=physics, aero=aero, precision=precision, autoreset=True,
                                    episode_len_sec=episode_len_sec, initial_xyzs=initial_xyzs,
                                    initial_rpys=initial_rpys, device=device, tuning=tuning)
        self.num_envs = int(num_envs)
        self.num_drones = int(num_drones)
        self.output = output
        self.action_space = action_space(num_drones, self.sim.act_width)
        self.observation_space = observation_space(num_drones, self.sim.act_width, int(ctrl_freq // 2))
        self._actions = torch.zeros((num_envs, num_drones, self.sim.act_width), dtype=torch.float32,
                                    device=self.sim.device)
        self.render_mode = None
        if _VecEnvBase is not object:
            super().__init__(self.num_envs, self.observation_space, self.action_space)

    # ------------------------------------------------------------------ VecEnv protocol
    def reset(self):
        obs = self.sim.reset()
        return obs.clone() if self.output == "torch" else obs.cpu().numpy()

    def step_async(self, actions):
        if isinstance(actions, torch.Tensor):
            self._actions.copy_(actions.reshape(self._actions.shape))
        else:
            a = np.asarray(actions, dtype=np.float32).reshape(self._actions.shape)
            self._actions.copy_(torch.from_numpy(a))

    def step_wait(self):
        obs, rew, te, tr = self.sim.step(self._actions, terminal_obs=True)
        done = (te | tr).bool()
        if self.output == "torch":
            infos = {"terminal_observation": self.sim.terminal_obs.clone(),
                     "TimeLimit.truncated": (tr.bool() & ~te.bool()), "done_mask": done}
            return obs.clone(), rew.clone(), done, infos
        o, r, d = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        te_n, tr_n = te.cpu().numpy().astype(bool), tr.cpu().numpy().astype(bool)
        infos = [{"answer": 42} for _ in range(self.num_envs)]
        if d.any():
            tobs = self.sim.terminal_obs.cpu().numpy()
            for e in np.nonzero(d)[0]:
                infos[e]["TimeLimit.truncated"] = bool(tr_n[e] and not te_n[e])
                infos[e]["terminal_observation"] = tobs[e].copy()
        return o, r, d, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.sim.close()

    def seed(self, seed=None):
        return [None] * self.num_envs   # resets are deterministic, as in the reference (:243)

    def get_attr(self, attr_name, indices=None):
        n = len(self._indices(indices))
        return [getattr(self, attr_name)] * n

    def set_attr(self, attr_name, value, indices=None):
        setattr(self, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        return [getattr(self, method_name)(*args, **kwargs) for _ in self._indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        return [None] * self.num_envs

    def render(self, mode=None):
        return None

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)


def make_vec_env(env_cls, n_envs=1, seed=None, env_kwargs=None, distributed=False, **vec_kwargs):
    """``stable_baselines3.common.env_util.make_vec_env`` stand-in for the two RL aviaries:
    builds ONE batched ``AviaryVecEnv`` instead of ``n_envs`` Python env objects; with
    ``distributed=True`` (inside an initialised torch.distributed group) a
    ``ShardedAviaryVecEnv`` whose envs are split over the group's ranks."""
    from .HoverAviary import HoverAviary
    from .MultiHoverAviary import MultiHoverAviary
    kw = dict(env_kwargs or {})
    if env_cls is HoverAviary or env_cls == "hover-aviary-v0":
        task, nd = "hover", 1
    elif env_cls is MultiHoverAviary or env_cls == "multihover-aviary-v0":
        task, nd = "multihover", kw.pop("num_drones", 2)
    else:
        raise ValueError(f"no batched implementation for {env_cls}")
    for k in ("gui", "record", "neighbourhood_radius"):
        kw.pop(k, None)
    kw.setdefault("physics", Physics.PYB)   # the env classes' default (HoverAviary.py:20, MultiHoverAviary.py:22)
    if distributed:
        return ShardedAviaryVecEnv(n_envs, task=task, num_drones=nd, **kw, **vec_kwargs)
    return AviaryVecEnv(n_envs, task=task, num_drones=nd, **kw, **vec_kwargs)


class ShardedAviaryVecEnv:
    """``AviaryVecEnv`` (torch output) over env shards on every rank of a ``torch.distributed``
    group: BASELINE config 5 / SURVEY §8(e), the multi-GPU form of the reference's
    ``make_vec_env(HoverAviary, n_envs=...)`` + PPO loop (``examples/learn.py:52-94``).

    Rank r owns envs ``[r*E/G, (r+1)*E/G)`` (``shard.env_shard``) in its own ``BatchedAviarySim``.
    The learner (rank 0) uses this object exactly like ``AviaryVecEnv(output="torch")``:
    ``reset()``, ``step(actions [E, D, A])`` -> (obs [E, D, W], reward [E], done [E], infos) with
    SB3's ``terminal_observation`` / ``TimeLimit.truncated``.  Each call broadcasts a one-word
    command, then ``shard.LearnerHandoff`` scatters the actions and gathers the shards' output
    packs (and the finished envs' terminal rows) to rank 0.  Every other rank runs ``serve()``, which answers commands until ``close()``.

    Mode "gather" (one learner): on a fully connected xGMI node every rank's 1.4 MB record
    reaches rank 0 over its own link (~9 us at ~153 GB/s), where a ring all-gather would pass
    G-1 records through each link and land them on every rank.  ``graph=True``
    (RCCL only): from the second step on, every step replays the hand-off's captured hipGraph
    (``LearnerHandoff.capture``), on every rank at the same step.
    """
    STEP, RESET, STOP, ROLLOUT = 0, 1, 2, 3

    def __init__(self, num_envs, graph=False, force_collectives=False, **kw):
        import torch.distributed as dist

        from ..shard import LearnerHandoff, env_shard
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        _, count = env_shard(num_envs, self.rank, self.world)
        kw = dict(kw)
        kw["output"] = "torch"
        self.local = AviaryVecEnv(count, **kw)
        self.sim = self.local.sim
        self.handoff = LearnerHandoff(self.sim, num_envs, mode="gather",   # one learner: rank 0
                                      force_collectives=force_collectives)
        self.num_envs = int(num_envs)
        self.num_drones = self.local.num_drones
        self.action_space = self.local.action_space
        self.observation_space = self.local.observation_space
        self.output = "torch"
        gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        self._cmd = torch.zeros((2,), dtype=torch.int32, device="cpu" if gloo else self.sim.device)
        self._actions = self.handoff.global_actions if self.rank == 0 else None
        self._graph = bool(graph) and not gloo
        self.graphed = self._graph
        self._steps = 0
        self._rgraph = None                 # the captured rollout (ROLLOUT command)
        self._open = True

    def _handoff_step(self, actions):
        if self._graph and self._steps == 1:
            self.handoff.capture()          # every rank, at its second step
        self._steps += 1
        return self.handoff.step(actions)

    def _send(self, cmd, arg=0):
        if self.world > 1:
            import torch.distributed as dist
            self._cmd[0] = cmd
            self._cmd[1] = arg
            dist.broadcast(self._cmd, src=0)

    def rollout(self, n_steps, seq):
        """The learner's rollout of ``n_steps`` hand-off steps as one hipGraph, replayed on every rank:
        ``seq`` (the learner's body: its policy kernels and ``handoff.step_body`` calls) is captured on
        the first call, the other ranks capture ``n_steps`` x ``handoff.step_body(None)`` at the same
        time (``serve``), and later calls replay.  RCCL only (``graph=True``)."""
        if not self._graph:
            raise ValueError("rollout() needs graph=True (the RCCL hand-off)")
        self._send(self.ROLLOUT, n_steps)
        self._replay_rollout(n_steps, seq)

    def _replay_rollout(self, n_steps, seq):
        if self._rgraph is None:
            self._rgraph = torch.cuda.CUDAGraph()
            with torch.cuda.device(self.sim.device), torch.cuda.graph(self._rgraph):
                seq()
            self._rgraph_steps = n_steps
        elif n_steps != self._rgraph_steps:
            raise ValueError("a rollout graph replays a fixed number of steps")
        self._rgraph.replay()

    def reset(self):
        self._send(self.RESET)
        return self.handoff.reset().clone()

    def step(self, actions):
        self._actions.copy_(torch.as_tensor(actions, dtype=torch.float32).reshape(self._actions.shape))
        self._send(self.STEP)
        obs, rew, te, tr, tobs = self._handoff_step(self._actions)
        # the hand-off's buffers are rewritten by the next step: the VecEnv hands out copies (as
        # AviaryVecEnv(output="torch") does)
        done = (te | tr).bool()
        infos = {"terminal_observation": tobs.clone(), "TimeLimit.truncated": (tr.bool() & ~te.bool()),
                 "done_mask": done}
        return obs.clone(), rew.clone(), done, infos

    def serve(self):
        """Non-learner ranks: step / reset this rank's shard on the learner's command."""
        import torch.distributed as dist
        while True:
            dist.broadcast(self._cmd, src=0)
            cmd, arg = (int(x) for x in self._cmd.tolist())
            if cmd == self.STOP:
                self._rgraph = None
                self.handoff.close()
                break
            if cmd == self.RESET:
                self.handoff.reset()
            elif cmd == self.ROLLOUT:
                h = self.handoff
                self._replay_rollout(arg, lambda: [h.step_body(None) for _ in range(arg)])
            else:
                self._handoff_step(None)
        self.local.close()
        self._open = False

    def close(self):
        if self._open:
            if self.rank == 0:
                self._send(self.STOP)
            self._rgraph = None
            self.handoff.close()
            self.local.close()
            self._open = False
