"""Batched aviary on one GPU: the Python owner of a ``gpd_sim`` (include/gpd.h).

``BatchedAviarySim`` holds the device state of ``n_envs`` identical aviaries (each with
``drones_per_env`` drones) and the caller-visible I/O buffers (torch tensors in HBM).  Every
call enqueues HIP work on the current torch stream of the sim's device; nothing here
computes physics on the CPU.
"""
import ctypes
import warnings

import numpy as np
import torch

from . import _lib
from .assets import default_params, model_id, parse_urdf
from .enums import ActionType, DroneModel, Physics

_ACTS = {ActionType.RPM: _lib.GPD_ACT_RPM, ActionType.ONE_D_RPM: _lib.GPD_ACT_ONE_D_RPM,
         ActionType.PID: _lib.GPD_ACT_PID, ActionType.VEL: _lib.GPD_ACT_VEL,
         ActionType.ONE_D_PID: _lib.GPD_ACT_ONE_D_PID}
PID_ACTS = (ActionType.PID, ActionType.VEL, ActionType.ONE_D_PID)
_TASKS = {"none": _lib.GPD_TASK_NONE, "hover": _lib.GPD_TASK_HOVER, "multihover": _lib.GPD_TASK_MULTIHOVER}
_AERO = {"gnd": _lib.GPD_F_GND, "drag": _lib.GPD_F_DRAG, "dw": _lib.GPD_F_DW, "geom": _lib.GPD_F_GEOM_WRENCH,
         "bullet": _lib.GPD_F_BULLET, "no_plane": _lib.GPD_F_NO_PLANE,
         "no_drone_contact": _lib.GPD_F_NO_DRONE_CONTACT}
_PHYSICS = {
    Physics.DYN: (),
    Physics.PYB: ("bullet",),
    Physics.PYB_GND: ("bullet", "gnd"),
    Physics.PYB_DRAG: ("bullet", "drag"),
    Physics.PYB_DW: ("bullet", "dw"),
    Physics.PYB_GND_DRAG_DW: ("bullet", "gnd", "drag", "dw"),
}
_warned = set()


def _warn_once(key, msg):
    if key not in _warned:
        _warned.add(key)
        warnings.warn(msg, stacklevel=3)


def physics_flags(physics=Physics.DYN, aero=()):
    """Map a reference ``Physics`` value (+ extra force terms) to GPD_F_* flags.

    DYN is the reference's explicit integrator (BaseAviary.py:352-353).  The PYB* values apply
    the reference's forces (``_physics`` / ``_groundEffect`` / ``_drag`` / ``_downwash``,
    :679-811) to a restated Bullet3 multibody base step (``p.stepSimulation``, :369-370; SURVEY
    §8 f3): default damping, world-frame angular velocity, exponential-map orientation, and the
    collision cylinder's contact with the ground plane (``plane.urdf``, BaseAviary.py:484) and,
    in envs of several drones, with the env's other drones (every drone is a colliding body,
    :486-491; envs of more than 64 drones raise NotImplementedError unless ``no_drone_contact``).
    Known deviations of the contact restatement from pybullet (parity unpinned):
    one point per pair (Bullet keeps a 4-point manifold), and the pair rows are solved before the
    plane rows instead of in one island solve, so a drone resting on another that rests on the
    plane sinks into it until the ERP push balances (~1 cm).  ``aero`` adds terms by name
    (``gnd``, ``drag``, ``dw``, ``geom``, ``bullet``, ``no_plane``, ``no_drone_contact``), e.g.
    the aero terms on the DYN integrator (BASELINE config 3), ``no_plane`` for the reference's
    commented-out plane collision filter (:500-503), or ``no_drone_contact``.
    """
    physics = Physics(physics)
    terms = set(_PHYSICS[physics]) | set(aero)
    unknown = terms - set(_AERO)
    if unknown:
        raise ValueError(f"unknown aero terms {sorted(unknown)}; expected a subset of {sorted(_AERO)}")
    for t in ("no_plane", "no_drone_contact"):
        if t in terms and "bullet" not in terms:
            raise ValueError(f"'{t}' applies to the Physics.PYB* modes only (Physics.DYN has no contacts)")
    flags = 0
    for t in terms:
        flags |= _AERO[t]
    return flags


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_raw_stream_fn = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(index):
    """The current stream of device `index` as an integer handle (torch's raw accessor when this
    build has it: the eager step() is host-bound, and the Stream object costs a microsecond)."""
    if _raw_stream_fn is not None:
        return _raw_stream_fn(index)
    return torch.cuda.current_stream(index).cuda_stream


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


STATE_COLS = 12   # KIN observation: pos, rpy, vel, ang_v (BaseRLAviary.py:313-316) before the history


def pack_layout(n_envs, drones_per_env, obs_width, align=256):
    """Byte layout of a sim's output pack, ``gpd_pack_layout_of`` (include/gpd.h) restated:
    {field: (offset, nbytes)} for obs | reward | terminated | truncated | terminal_state |
    terminal_obs (each 256-B aligned), "prefix" = the end of the truncated flags,
    "prefix_aligned" = that rounded up to 256, "record" = the end of terminal_state (one rank's
    hand-off record, ``shard.LearnerHandoff``) and "total"."""
    E, D, W = n_envs, drones_per_env, obs_width
    out, off = {}, 0
    for name, nbytes in (("obs", E * D * W * 4), ("reward", E * 4), ("terminated", E), ("truncated", E),
                         ("terminal_state", E * D * STATE_COLS * 4), ("terminal_obs", E * D * W * 4)):
        out[name] = (off, nbytes)
        if name == "truncated":
            out["prefix"] = off + nbytes
            out["prefix_aligned"] = -(-(off + nbytes) // align) * align
        off += -(-nbytes // align) * align
        if name == "terminal_state":
            out["record"] = off
    out["total"] = off
    return out


class BatchedAviarySim:
    """``n_envs`` x ``drones_per_env`` Crazyflie-class drones stepped in lockstep on one GPU."""

    def __init__(self, n_envs, drones_per_env=1, drone_model=DroneModel.CF2X, urdf_path=None,
                 pyb_freq=240, ctrl_freq=30, act=ActionType.RPM, task="hover",
                 physics=Physics.DYN, aero=(), precision="f64", autoreset=True, episode_len_sec=8,
                 initial_xyzs=None, initial_rpys=None, device=None, tuning=None):
        self._lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.GpdLibraryError("BatchedAviarySim needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        act = ActionType(act)
        if precision not in ("f32", "f64"):
            raise ValueError("precision must be 'f32' or 'f64'")
        if precision == "f32":
            _warn_once("f32", "precision='f32' does not meet the 1e-5 state-parity gate over 5 s (open-loop "
                       "attitude dynamics amplify float32 rounding to 1e-5..2e-4; DESIGN.md §5); f64 is the "
                       "reference's precision and costs about the same on MI355X")
        self.drone_model = DroneModel(drone_model)
        self.params = parse_urdf(urdf_path, self.drone_model) if urdf_path else default_params(self.drone_model)
        self.params.model = model_id(self.drone_model)
        self.n_envs, self.drones_per_env = int(n_envs), int(drones_per_env)
        self.act_type = act
        self.task = task
        self.precision = precision
        self.real_dtype = torch.float32 if precision == "f32" else torch.float64
        cfg = _lib.Config()
        cfg.n_envs = self.n_envs
        cfg.drones_per_env = self.drones_per_env
        cfg.pyb_freq = int(pyb_freq)
        cfg.ctrl_freq = int(ctrl_freq)
        cfg.act_type = _ACTS[act]
        cfg.task = _TASKS[task]
        cfg.physics_flags = physics_flags(physics, aero)
        if cfg.physics_flags & _lib.GPD_F_BULLET and self.drones_per_env > 64 \
                and not cfg.physics_flags & _lib.GPD_F_NO_DRONE_CONTACT:
            # a physics term is never dropped silently: the multi-wave kernels do not restate it
            raise NotImplementedError(
                f"{Physics(physics)} with {self.drones_per_env} drones per env: the drone <-> drone contact is "
                "implemented for envs of up to 64 drones; pass aero=('no_drone_contact',) to run larger "
                "PYB* envs without it")
        cfg.precision = _lib.GPD_F32 if precision == "f32" else _lib.GPD_F64
        cfg.autoreset = 1 if autoreset else 0
        cfg.episode_len_sec = float(episode_len_sec)
        # launch tuning (gpd_config: drones_per_block, step_waves, store_policy; 0 = automatic) and
        # the PYB* contact solver's numSolverIterations / solverResidualThreshold (0 = pybullet's)
        for name, val in (tuning or {}).items():
            if name == "solver_residual":
                cfg.solver_residual = float(val)
                continue
            if name not in ("drones_per_block", "step_waves", "store_policy", "solver_iterations"):
                raise ValueError(f"unknown tuning field {name!r}")
            setattr(cfg, name, int(val))
        keep = []
        for name, arr in (("init_xyzs_host", initial_xyzs), ("init_rpys_host", initial_rpys)):
            if arr is not None:
                a = np.ascontiguousarray(np.asarray(arr, dtype=np.float64).reshape(self.drones_per_env, 3))
                keep.append(a)
                setattr(cfg, name, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        self.physics_flags = cfg.physics_flags
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check("gpd_create", self._lib.gpd_create(ctypes.byref(self.params), ctypes.byref(cfg),
                                                          ctypes.byref(handle)))
        self._h = handle
        k = _lib.Constants()
        _lib.check("gpd_get_constants", self._lib.gpd_get_constants(self._h, ctypes.byref(k)))
        self.constants = k
        self.n_drones = k.n_drones
        self.obs_width = k.obs_width
        self.act_width = k.act_width
        self.pyb_steps_per_ctrl = k.pyb_steps_per_ctrl
        E, D, W = self.n_envs, self.drones_per_env, self.obs_width
        dev = self.device
        # every per-step output lives in ONE device buffer ("out pack"), so that a sharded run hands
        # a step to the learner with a single collective over the kernel's own output bytes
        # (shard.LearnerHandoff): [obs | reward | terminated | truncated | terminal_obs], each field
        # 256-B aligned; the terminal rows come last so that a hand-off without them is a prefix
        self.pack_layout = pack_layout(E, D, W)
        L = self.pack_layout
        self.out_pack = torch.zeros((L["total"],), dtype=torch.uint8, device=dev)
        self.obs = self._field("obs", torch.float32, (E, D, W))
        self.reward = self._field("reward", torch.float32, (E,))
        self.terminated = self._field("terminated", torch.uint8, (E,))
        self.truncated = self._field("truncated", torch.uint8, (E,))
        self.terminal_obs = self._field("terminal_obs", torch.float32, (E, D, W))
        # the sim-owned output buffers never move: their ctypes pointers are built once (the eager
        # step() is host-bound at 4096 envs, a few microseconds per call)
        self._step_fn = self._lib.gpd_step
        self._out_ptrs = (_ptr(self.obs), _ptr(self.reward), _ptr(self.terminated), _ptr(self.truncated))
        self._tobs_ptr = _ptr(self.terminal_obs)
        self.reset()

    def _field(self, name, dtype, shape):
        off, n = self.pack_layout[name]
        return self.out_pack[off:off + n].view(dtype).view(shape)

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self._lib.gpd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, name, *args):
        _lib.check(name, getattr(self._lib, name)(self._h, *args))

    # ------------------------------------------------------------------ RL surface
    def reset(self, env_mask=None):
        """BaseAviary.reset (:220-255) for all envs or the envs where ``env_mask`` is true."""
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
            assert m.numel() == self.n_envs
        with torch.cuda.device(self.device):
            self._call("gpd_reset", _ptr(m), _ptr(self.obs), _stream(self.device))
        return self.obs

    def step(self, actions, terminal_obs=True):
        """BaseAviary.step (:259-383) for every env; ``actions`` [E, D, A] float32 on the device.

        Returns the sim-owned (obs, reward, terminated, truncated) tensors; they are
        overwritten by the next call.  With autoreset, ``self.terminal_obs`` holds the final
        rows of the envs that finished in this step."""
        a = actions
        if not (isinstance(a, torch.Tensor) and a.device == self.device and a.dtype == torch.float32
                and a.is_contiguous()):
            a = torch.as_tensor(a, dtype=torch.float32, device=self.device).contiguous()
        if a.numel() != self.n_drones * self.act_width:
            raise ValueError(f"actions must have {self.n_envs}x{self.drones_per_env}x{self.act_width} elements")
        tptr = self._tobs_ptr if terminal_obs else None
        if torch.cuda.current_device() == self.device.index:
            rc = self._step_fn(self._h, a.data_ptr(), *self._out_ptrs, tptr, _raw_stream(self.device.index))
        else:
            with torch.cuda.device(self.device):
                rc = self._step_fn(self._h, a.data_ptr(), *self._out_ptrs, tptr, _stream(self.device))
        if rc != 0:
            _lib.check("gpd_step", rc)
        return self.obs, self.reward, self.terminated, self.truncated

    def step_seq(self, action_slots, n_steps, terminal_obs=True):
        """``n_steps`` consecutive :meth:`step` calls issued from native code (``gpd_step_seq``):
        step t reads ``action_slots[t % P]`` of ``action_slots`` [P, E, D, A] (float32, on the
        device); the output tensors hold the last step's results."""
        a = action_slots
        if not (isinstance(a, torch.Tensor) and a.device == self.device and a.dtype == torch.float32
                and a.is_contiguous() and a.numel() % (self.n_drones * self.act_width) == 0):
            raise ValueError("step_seq needs contiguous float32 action slots [P, E, D, A] on the sim's device")
        P = a.numel() // (self.n_drones * self.act_width)
        tptr = self._tobs_ptr if terminal_obs else None
        with torch.cuda.device(self.device):
            self._call("gpd_step_seq", ctypes.c_void_p(a.data_ptr()), int(P), int(n_steps), *self._out_ptrs, tptr,
                       _stream(self.device))
        return self.obs, self.reward, self.terminated, self.truncated

    def capture_graph(self, actions_seq, terminal_obs=True):
        """Record ``len(actions_seq)`` consecutive :meth:`step` launches into one HIP graph
        (``torch.cuda.CUDAGraph``).  Each ``replay()`` advances every env by that many steps,
        reading the given action tensors (refill them in place between replays).  gpd_step is
        a fixed-argument launch - the ring head and step counters live in device memory - so
        one recorded sequence stays valid for any number of replays.  Capture records only;
        the sim does not advance until the first replay."""
        seq = []
        for a in actions_seq:
            if not (isinstance(a, torch.Tensor) and a.device == self.device and a.dtype == torch.float32
                    and a.is_contiguous() and a.numel() == self.n_drones * self.act_width):
                raise ValueError("capture_graph needs contiguous float32 action tensors on the sim's device")
            seq.append(a)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.device(self.device), torch.cuda.graph(g):
            for a in seq:
                self.step(a, terminal_obs=terminal_obs)
        return g

    # ------------------------------------------------------------------ raw physics
    def integrate(self, rpm, record=False):
        """Raw DYN substeps: ``rpm`` [T, N, 4] (real dtype) -> optional trajectory [T, N, 20]."""
        r = torch.as_tensor(rpm, dtype=self.real_dtype, device=self.device).contiguous()
        T = r.shape[0]
        assert r.numel() == T * self.n_drones * 4
        traj = torch.empty((T, self.n_drones, 20), dtype=self.real_dtype, device=self.device) if record else None
        with torch.cuda.device(self.device):
            self._call("gpd_integrate", _ptr(r), int(T), _ptr(traj), _stream(self.device))
        return traj

    def state20(self):
        """BaseAviary._getDroneStateVector (:541-561) for every drone, [N, 20]."""
        out = torch.empty((self.n_drones, 20), dtype=self.real_dtype, device=self.device)
        with torch.cuda.device(self.device):
            self._call("gpd_get_state20", _ptr(out), _stream(self.device))
        return out

    def nonfinite(self):
        """Per-env non-finite guard (the reference has none): bool [E] on the device,
        True where any drone of the env holds a non-finite state component."""
        out = torch.empty((self.n_envs,), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            self._call("gpd_nonfinite", _ptr(out), _stream(self.device))
        return out.bool()

    def raw_state(self):
        out = torch.empty((self.n_drones, 20), dtype=self.real_dtype, device=self.device)
        with torch.cuda.device(self.device):
            self._call("gpd_get_raw_state", _ptr(out), _stream(self.device))
        return out

    def set_raw_state(self, raw):
        r = torch.as_tensor(raw, dtype=self.real_dtype, device=self.device).contiguous()
        assert r.numel() == self.n_drones * 20
        with torch.cuda.device(self.device):
            self._call("gpd_set_raw_state", _ptr(r), _stream(self.device))

    # ------------------------------------------------------------------ DSLPIDControl (PID types)
    def ctrl_state(self):
        """Per-drone controller state [N, 9]: integral_pos_e, integral_rpy_e, last_rpy
        (DSLPIDControl.py:65-78); only for the PID / VEL / ONE_D_PID action types."""
        out = torch.empty((self.n_drones, _lib.CTRL_COMPS), dtype=self.real_dtype, device=self.device)
        with torch.cuda.device(self.device):
            self._call("gpd_get_ctrl_state", _ptr(out), _stream(self.device))
        return out

    def set_ctrl_state(self, cs):
        t = torch.as_tensor(cs, dtype=self.real_dtype, device=self.device).contiguous()
        assert t.numel() == self.n_drones * _lib.CTRL_COMPS
        with torch.cuda.device(self.device):
            self._call("gpd_set_ctrl_state", _ptr(t), _stream(self.device))

    def set_pid_coefficients(self, p_coeff_pos=None, i_coeff_pos=None, d_coeff_pos=None,
                             p_coeff_att=None, i_coeff_att=None, d_coeff_att=None):
        """BaseControl.setPIDCoefficients (control/BaseControl.py:138-177) for every drone."""
        q = getattr(self, "_pid", None) or _lib.default_pid_params()
        for name, val in (("p_coeff_for", p_coeff_pos), ("i_coeff_for", i_coeff_pos), ("d_coeff_for", d_coeff_pos),
                          ("p_coeff_tor", p_coeff_att), ("i_coeff_tor", i_coeff_att), ("d_coeff_tor", d_coeff_att)):
            if val is not None:
                v = np.asarray(val, dtype=np.float64).reshape(3)
                getattr(q, name)[:] = v.tolist()
        with torch.cuda.device(self.device):
            _lib.check("gpd_set_pid_params", self._lib.gpd_set_pid_params(self._h, ctypes.byref(q)))
        self._pid = q

    def step_counters(self):
        out = torch.empty((self.n_envs,), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            self._call("gpd_get_step_counters", _ptr(out), _stream(self.device))
        return out

    def set_step_counters(self, sc):
        t = torch.as_tensor(sc, dtype=torch.int32, device=self.device).contiguous()
        with torch.cuda.device(self.device):
            self._call("gpd_set_step_counters", _ptr(t), _stream(self.device))

    def save_state(self):
        n = self._lib.gpd_state_bytes(self._h)
        buf = ctypes.create_string_buffer(n)
        with torch.cuda.device(self.device):
            self._call("gpd_save_state", ctypes.cast(buf, ctypes.c_void_p), _stream(self.device))
        return buf.raw

    def load_state(self, blob):
        n = self._lib.gpd_state_bytes(self._h)
        if len(blob) != n:
            raise ValueError(f"state blob has {len(blob)} bytes, expected {n}")
        buf = ctypes.create_string_buffer(blob, n)
        with torch.cuda.device(self.device):
            self._call("gpd_load_state", ctypes.cast(buf, ctypes.c_void_p), _stream(self.device))
