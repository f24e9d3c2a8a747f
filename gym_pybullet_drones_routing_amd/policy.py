"""Fused rollout policy: the ctypes binding of ``include/gpd_policy.h`` (``libgpd_policy.so``).

The caller of the env step in the reference is stable-baselines3 PPO (``examples/learn.py:52-94``):
per env.step its rollout runs the MlpPolicy actor and critic ([64, 64] tanh), samples
Normal(mu, exp(log_std)), clips the action to the Box, writes the rollout buffer and, after the
step, bootstraps time-limit truncations with V(terminal_observation).  ``MlpPolicyKernel`` does
all of that in ONE HIP kernel per step (``gpd_policy_rollout_step``) reading the torch module's
parameters in place, and GAE in one more per rollout (``gpd_policy_gae``).  There is no torch
fallback: without the library every call raises ``GpdLibraryError``.
"""
import ctypes
import os
import pathlib

import torch

from ._lib import GpdError, GpdLibraryError

LIB_PATH = pathlib.Path(os.environ.get("GPD_POLICY_LIB") or (pathlib.Path(__file__).resolve().parent /
                                                               "libgpd_policy.so"))
GPD_POLICY_ABI_VERSION = 2
GROUP_ROWS = 16                 # rows per Philox call counter (the kernel's row group)
HIDDEN = 64
MAX_OBS = 192
MAX_ACT = 8
EXPORTED = ("gpd_policy_rollout_step", "gpd_policy_gae", "gpd_policy_abi_version", "gpd_policy_last_error")


class MlpPolicyStruct(ctypes.Structure):
    _fields_ = [("n_obs", ctypes.c_int), ("n_act", ctypes.c_int)] + [
        (n, ctypes.c_void_p) for n in ("pi_w1", "pi_b1", "pi_w2", "pi_b2", "pi_w3", "pi_b3",
                                       "vf_w1", "vf_b1", "vf_w2", "vf_b2", "vf_w3", "vf_b3", "log_std")]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise GpdLibraryError(f"{LIB_PATH} is missing: run `python -m gym_pybullet_drones_routing_amd._build` "
                              "(or __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(str(LIB_PATH))
    except OSError as exc:
        raise GpdLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.gpd_policy_abi_version.restype = ci
    lib.gpd_policy_abi_version.argtypes = []
    lib.gpd_policy_last_error.restype = ctypes.c_char_p
    lib.gpd_policy_last_error.argtypes = []
    lib.gpd_policy_rollout_step.restype = ci
    lib.gpd_policy_rollout_step.argtypes = [ctypes.POINTER(MlpPolicyStruct), ci, vp, vp, vp, vp, vp, vp, ci, vp, ci,
                                            vp, vp, vp, vp, ctypes.c_float, vp, vp, vp]
    lib.gpd_policy_gae.restype = ci
    lib.gpd_policy_gae.argtypes = [ci, ci, vp, vp, vp, vp, ctypes.c_double, ctypes.c_double, vp, vp, vp]
    if lib.gpd_policy_abi_version() != GPD_POLICY_ABI_VERSION:
        raise GpdLibraryError(f"{LIB_PATH} has ABI {lib.gpd_policy_abi_version()}, expected {GPD_POLICY_ABI_VERSION}")
    _lib = lib
    return lib


def _check(name, rc):
    if rc != 0:
        raise GpdError(name, rc, _lib.gpd_policy_last_error().decode(errors="replace"))


def _linears(seq):
    lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
    acts = [m for m in seq if not isinstance(m, torch.nn.Linear)]
    if len(lin) != 3 or not all(isinstance(a, torch.nn.Tanh) for a in acts) or len(acts) != 2 \
            or lin[0].out_features != HIDDEN or lin[1].in_features != HIDDEN or lin[1].out_features != HIDDEN \
            or lin[2].in_features != HIDDEN:
        raise ValueError("the fused policy runs SB3 MlpPolicy networks: Linear(n, 64) Tanh Linear(64, 64) Tanh "
                         "Linear(64, m)")
    return lin


class MlpPolicyKernel:
    """The actor-critic ``module`` (``.pi``, ``.vf`` as Linear-Tanh-Linear-Tanh-Linear, ``.log_std``;
    examples/learn.py's ``ActorCritic``) as one rollout kernel per step.  The parameters are read
    in place: an optimizer step that updates them in place is seen by the next call (and by a
    captured graph).  ``seed``: the Philox key; the call counters (one per group of 16 rows) live
    on the device (``rng``), sized for ``max_rows`` rows (grown by a call with more rows, which a
    captured graph must not do)."""

    def __init__(self, module, seed=0, max_rows=1 << 16):
        self._lib = load()
        pi, vf = _linears(module.pi), _linears(module.vf)
        if vf[2].out_features != 1:
            raise ValueError("the critic has one output")
        self.n_obs, self.n_act = pi[0].in_features, pi[2].out_features
        if vf[0].in_features != self.n_obs:
            raise ValueError("actor and critic read the same observation")
        if not 1 <= self.n_obs <= MAX_OBS or not 1 <= self.n_act <= MAX_ACT:
            raise ValueError(f"n_obs must be in [1, {MAX_OBS}] and n_act in [1, {MAX_ACT}]")
        params = [p for lin in pi + vf for p in (lin.weight, lin.bias)] + [module.log_std]
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev or dev.type != "cuda":
                raise ValueError("the fused policy reads contiguous float32 parameters on the GPU")
        self.device = dev
        self._params = params            # kept alive: the struct holds their addresses
        st = MlpPolicyStruct()
        st.n_obs, st.n_act = self.n_obs, self.n_act
        names = ("pi_w1", "pi_b1", "pi_w2", "pi_b2", "pi_w3", "pi_b3", "vf_w1", "vf_b1", "vf_w2", "vf_b2",
                 "vf_w3", "vf_b3", "log_std")
        for n, p in zip(names, params):
            setattr(st, n, p.data_ptr())
        self._st = st
        # {key, 0, call counter of row group 0, 1, ...} (include/gpd_policy.h)
        self.rng = torch.zeros(2 + -(-int(max_rows) // GROUP_ROWS), dtype=torch.int64, device=dev)
        self.rng[0] = int(seed)

    @property
    def rng_groups(self):
        return self.rng.numel() - 2

    def _fit(self, n_rows):
        need = -(-n_rows // GROUP_ROWS)
        if need > self.rng_groups:
            if torch.cuda.is_current_stream_capturing():
                raise ValueError(f"{n_rows} rows need {need} row-group counters, the rng holds {self.rng_groups}: "
                                 "pass max_rows >= the largest batch before capturing a graph")
            grown = torch.zeros(2 + need, dtype=torch.int64, device=self.device)
            grown[:self.rng.numel()] = self.rng
            grown[self.rng.numel():] = self.rng[2]      # new groups join at the batch's call count
            self.rng = grown

    @property
    def calls(self):
        """Sampling calls made so far (row group 0's device counter; reading it synchronises)."""
        return int(self.rng[2])

    def set_calls(self, n):
        """Rewind / advance the Philox call counters of every row group (the same key and counter draw
        the same numbers)."""
        self.rng[2:] = int(n)

    def _rows(self, t, width, name):
        if t is None:
            return None
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous float32 device tensor")
        if t.numel() != self._n * width:
            raise ValueError(f"{name} must hold {self._n} x {width} elements, has {t.numel()}")
        return ctypes.c_void_p(t.data_ptr())

    def step(self, obs=None, act_env=None, buf_obs=None, buf_act=None, buf_logp=None, buf_val=None,
             deterministic=False, prev=None, gamma=0.99, buf_rew=None, buf_done=None, n_rows=None):
        """One rollout step (gpd_policy_rollout_step); ``prev`` = (reward, terminated, truncated,
        terminal_obs) of the previous env.step, written to ``buf_rew`` / ``buf_done``."""
        src = obs if obs is not None else (prev[3] if prev is not None else None)
        if src is None:
            raise ValueError("nothing to do: neither obs nor prev")
        self._n = int(n_rows) if n_rows is not None else src.numel() // self.n_obs
        self._fit(self._n)
        args = [self._rows(obs, self.n_obs, "obs"), self._rows(act_env, self.n_act, "act_env"),
                self._rows(buf_obs, self.n_obs, "buf_obs"), self._rows(buf_act, self.n_act, "buf_act"),
                self._rows(buf_logp, 1, "buf_logp"), self._rows(buf_val, 1, "buf_val")]
        if prev is not None:
            rew, te, tr, tobs = prev
            for t, nm in ((te, "terminated"), (tr, "truncated")):
                if not (t.is_cuda and t.dtype == torch.uint8 and t.numel() == self._n):
                    raise ValueError(f"{nm} must be a uint8 device tensor of {self._n} flags")
            pv = [self._rows(rew, 1, "reward"), ctypes.c_void_p(te.data_ptr()), ctypes.c_void_p(tr.data_ptr()),
                  self._rows(tobs, self.n_obs, "terminal_obs")]
            outs = [self._rows(buf_rew, 1, "buf_rew"), self._rows(buf_done, 1, "buf_done")]
        else:
            pv, outs = [None] * 4, [None, None]
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _check("gpd_policy_rollout_step", self._lib.gpd_policy_rollout_step(
            ctypes.byref(self._st), self._n, *args, 1 if deterministic else 0, ctypes.c_void_p(self.rng.data_ptr()),
            self.rng_groups, *pv, float(gamma), *outs, ctypes.c_void_p(stream)))

    def gae(self, rew, val, done, last_val, gamma, lam, adv, ret):
        """GAE over a rollout, bit-identical to examples/learn.py's torch loop: [T, E] tensors."""
        T, E = rew.shape
        for t in (rew, val, done, adv, ret):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == (T, E)):
                raise ValueError("GAE buffers must be contiguous float32 [T, E] device tensors")
        if last_val.numel() != E:
            raise ValueError("last_val must hold E values")
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _check("gpd_policy_gae", self._lib.gpd_policy_gae(
            T, E, *(ctypes.c_void_p(t.data_ptr()) for t in (rew, val, done, last_val)), float(gamma), float(lam),
            ctypes.c_void_p(adv.data_ptr()), ctypes.c_void_p(ret.data_ptr()), ctypes.c_void_p(stream)))
