"""ctypes wrapper of the C oracle (oracle/gpd_oracle.c).  TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

from .params import derived

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liborc.so")
_MODELS = {"cf2x": 0, "cf2p": 1, "racer": 2}
_TASKS = {"none": 0, "hover": 1, "multihover": 2}
_FLAGS = {"gnd": 1, "drag": 2, "dw": 4, "geom": 8}


class OrcParams(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int)] + [(n, ctypes.c_double) for n in (
        "m", "arm", "thrust2weight", "ixx", "iyy", "izz", "kf", "km", "collision_h", "collision_r",
        "collision_z_offset", "gnd_eff_coeff", "prop_radius", "drag_coeff_xy", "drag_coeff_z",
        "dw1", "dw2", "dw3")] + [("prop_pos", (ctypes.c_double * 3) * 4)]


_lib = None


def load(build=True):
    global _lib
    if _lib is not None:
        return _lib
    if build and not os.path.exists(_LIB):
        subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
    lib = ctypes.CDLL(_LIB)
    vp, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.orc_create.restype = vp
    lib.orc_create.argtypes = [ctypes.POINTER(OrcParams), i, i, i, i, i, i, i, i, d, vp, vp]
    lib.orc_destroy.argtypes = [vp]
    lib.orc_obs_width.argtypes = [vp]
    lib.orc_obs_width.restype = i
    for fn in ("orc_reset", "orc_set_raw", "orc_get_raw", "orc_get_state20"):
        getattr(lib, fn).argtypes = [vp, vp]
    lib.orc_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, i]
    lib.orc_integrate.argtypes = [vp, vp, i, vp, i]
    _lib = lib
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class COracle:
    """Batched C oracle: E envs x D drones, same semantics as ref_aviary.RefAviary."""

    def __init__(self, n_envs, drones_per_env=1, model="cf2x", act="rpm", task="hover", aero=(),
                 wrench="dyn", pyb_freq=240, ctrl_freq=30, autoreset=True, episode_len_sec=8,
                 initial_xyzs=None, initial_rpys=None, threads=0):
        lib = load()
        p = derived(model)
        op = OrcParams()
        op.model = _MODELS[model]
        for name in ("m", "arm", "thrust2weight", "ixx", "iyy", "izz", "kf", "km", "collision_h",
                     "collision_r", "collision_z_offset", "gnd_eff_coeff", "prop_radius",
                     "drag_coeff_xy", "drag_coeff_z"):
            setattr(op, name, p[name])
        op.dw1, op.dw2, op.dw3 = p["dw_coeff_1"], p["dw_coeff_2"], p["dw_coeff_3"]
        for k in range(4):
            for j in range(3):
                op.prop_pos[k][j] = p["prop_pos"][k][j]
        flags = 0
        for t in aero:
            flags |= _FLAGS[t]
        if wrench == "geom":
            flags |= _FLAGS["geom"]
        self.A = 4 if act == "rpm" else 1
        self.E, self.D, self.N = n_envs, drones_per_env, n_envs * drones_per_env
        self._xyz = None if initial_xyzs is None else np.ascontiguousarray(initial_xyzs, dtype=np.float64)
        self._rpy = None if initial_rpys is None else np.ascontiguousarray(initial_rpys, dtype=np.float64)
        self._h = lib.orc_create(ctypes.byref(op), n_envs, drones_per_env, pyb_freq, ctrl_freq, self.A,
                                 _TASKS[task], flags, 1 if autoreset else 0, float(episode_len_sec),
                                 _ptr(self._xyz), _ptr(self._rpy))
        if not self._h:
            raise ValueError("orc_create rejected the configuration")
        self.W = lib.orc_obs_width(self._h)
        self.threads = threads
        self.obs = np.zeros((n_envs, drones_per_env, self.W), np.float32)
        self.terminal_obs = np.zeros_like(self.obs)
        self.reward = np.zeros(n_envs, np.float32)
        self.terminated = np.zeros(n_envs, np.uint8)
        self.truncated = np.zeros(n_envs, np.uint8)
        lib.orc_reset(self._h, _ptr(self.obs))

    def close(self):
        if self._h:
            _lib.orc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.orc_reset(self._h, _ptr(self.obs))
        return self.obs

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.N, self.A)
        _lib.orc_step(self._h, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                      _ptr(self.truncated), _ptr(self.terminal_obs), self.threads)
        return self.obs, self.reward, self.terminated.astype(bool), self.truncated.astype(bool)

    def integrate(self, rpm, record=True):
        r = np.ascontiguousarray(rpm, dtype=np.float64)
        T = r.shape[0]
        traj = np.zeros((T, self.N, 20)) if record else None
        _lib.orc_integrate(self._h, _ptr(r), T, _ptr(traj), self.threads)
        return traj

    def set_raw_state(self, raw):
        r = np.ascontiguousarray(raw, dtype=np.float64).reshape(self.N, 20)
        _lib.orc_set_raw(self._h, _ptr(r))

    def raw_state(self):
        out = np.zeros((self.N, 20))
        _lib.orc_get_raw(self._h, _ptr(out))
        return out

    def state20(self):
        out = np.zeros((self.N, 20))
        _lib.orc_get_state20(self._h, _ptr(out))
        return out
