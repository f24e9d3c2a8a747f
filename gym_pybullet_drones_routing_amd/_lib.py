"""ctypes binding of the C ABI declared in ``include/gpd.h``.

This is the same binding a maintainer of the reference would add.
There is deliberately NO CPU fallback: if ``libgpd.so`` is missing or fails to load,
every entry point raises ``GpdLibraryError``.
"""
import ctypes
import os
import pathlib

# The HIP runtime must be the one torch already loaded (same SONAME libamdhip64.so.7):
# import torch first so that libgpd.so binds to it instead of a second runtime copy.
import torch  # noqa: F401  (imported for its side effect on the dynamic linker)

LIB_PATH = pathlib.Path(os.environ.get("GPD_LIB") or (pathlib.Path(__file__).resolve().parent / "libgpd.so"))

GPD_OK = 0
GPD_EINVAL = -1
GPD_EHIP = -2
GPD_ENOMEM = -3
GPD_EUNSUPPORTED = -4

GPD_MODEL_CF2X, GPD_MODEL_CF2P, GPD_MODEL_RACE = 0, 1, 2
GPD_ACT_RPM, GPD_ACT_ONE_D_RPM, GPD_ACT_PID, GPD_ACT_VEL, GPD_ACT_ONE_D_PID = 0, 1, 2, 3, 4
GPD_ABI_VERSION = 7
CTRL_COMPS = 9  # integral_pos_e(3) integral_rpy_e(3) last_rpy(3)
GPD_TASK_NONE, GPD_TASK_HOVER, GPD_TASK_MULTIHOVER = 0, 1, 2
GPD_F_GND, GPD_F_DRAG, GPD_F_DW, GPD_F_GEOM_WRENCH, GPD_F_BULLET, GPD_F_NO_PLANE = 1, 2, 4, 8, 16, 32
GPD_F_NO_DRONE_CONTACT = 64
GPD_F32, GPD_F64 = 0, 1

# Every symbol include/gpd.h declares (checked by tests/test_lib_symbols.py).
EXPORTED = ("gpd_abi_version", "gpd_last_error", "gpd_default_params", "gpd_create", "gpd_destroy",
            "gpd_get_constants", "gpd_reset", "gpd_step", "gpd_step_seq", "gpd_integrate", "gpd_get_state20",
            "gpd_get_raw_state", "gpd_set_raw_state", "gpd_get_step_counters",
            "gpd_set_step_counters", "gpd_state_bytes", "gpd_save_state", "gpd_load_state",
            "gpd_default_pid_params", "gpd_set_pid_params", "gpd_get_ctrl_state", "gpd_set_ctrl_state",
            "gpd_nonfinite", "gpd_pack_layout_of", "gpd_handoff_pack", "gpd_handoff_unpack")


class GpdLibraryError(RuntimeError):
    pass


class GpdError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed with code {code}: {msg}")
        self.code = code


class DroneParams(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int)] + [(n, ctypes.c_double) for n in (
        "m", "arm", "thrust2weight", "ixx", "iyy", "izz", "kf", "km",
        "collision_h", "collision_r", "collision_z_offset", "max_speed_kmh",
        "gnd_eff_coeff", "prop_radius", "drag_coeff_xy", "drag_coeff_z",
        "dw_coeff_1", "dw_coeff_2", "dw_coeff_3")] + [("prop_pos", (ctypes.c_double * 3) * 4)]


class PidParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double * 3) for n in (
        "p_coeff_for", "i_coeff_for", "d_coeff_for", "p_coeff_tor", "i_coeff_tor", "d_coeff_tor")] + \
        [(n, ctypes.c_double) for n in ("pwm2rpm_scale", "pwm2rpm_const", "min_pwm", "max_pwm")] + \
        [("mixer", (ctypes.c_double * 3) * 4)] + [(n, ctypes.c_double) for n in ("gravity", "kf")]


class Config(ctypes.Structure):
    _fields_ = [("n_envs", ctypes.c_int), ("drones_per_env", ctypes.c_int), ("pyb_freq", ctypes.c_int),
                ("ctrl_freq", ctypes.c_int), ("act_type", ctypes.c_int), ("task", ctypes.c_int),
                ("physics_flags", ctypes.c_int), ("precision", ctypes.c_int), ("autoreset", ctypes.c_int),
                ("episode_len_sec", ctypes.c_double),
                ("init_xyzs_host", ctypes.POINTER(ctypes.c_double)),
                ("init_rpys_host", ctypes.POINTER(ctypes.c_double)),
                ("drones_per_block", ctypes.c_int), ("step_waves", ctypes.c_int), ("store_policy", ctypes.c_int),
                ("solver_iterations", ctypes.c_int), ("solver_residual", ctypes.c_double)]


class PackLayout(ctypes.Structure):
    """gpd_pack_layout: byte offsets of a shard's output pack (include/gpd.h)."""
    _fields_ = [(n, ctypes.c_int) for n in ("n_envs", "drones_per_env", "obs_width", "state_cols")] + \
        [(n, ctypes.c_longlong) for n in ("obs", "reward", "terminated", "truncated", "terminal_state",
                                          "terminal_obs", "prefix", "prefix_aligned", "record", "total")]


class Constants(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "gravity", "hover_rpm", "max_rpm", "max_thrust", "max_xy_torque", "max_z_torque",
        "gnd_eff_h_clip", "pyb_timestep", "ctrl_timestep")] + [(n, ctypes.c_int) for n in (
            "pyb_steps_per_ctrl", "action_buffer_size", "obs_width", "act_width", "n_drones",
            "trunc_step_counter", "drones_per_block", "lanes_per_block")]


_lib = None


def load():
    """Load libgpd.so (once) and declare the C signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise GpdLibraryError(f"{LIB_PATH} is missing: run `python -m gym_pybullet_drones_routing_amd._build` "
                              "(or __graft_entry__.build()) to compile the gfx950 HIP library")
    try:
        lib = ctypes.CDLL(str(LIB_PATH))
    except OSError as exc:
        raise GpdLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
    vp, i, ci = ctypes.c_void_p, ctypes.c_int, ctypes.c_int
    sig = {
        "gpd_abi_version": (ci, []),
        "gpd_last_error": (ctypes.c_char_p, []),
        "gpd_default_params": (ci, [i, ctypes.POINTER(DroneParams)]),
        "gpd_create": (ci, [ctypes.POINTER(DroneParams), ctypes.POINTER(Config), ctypes.POINTER(vp)]),
        "gpd_destroy": (ci, [vp]),
        "gpd_get_constants": (ci, [vp, ctypes.POINTER(Constants)]),
        "gpd_reset": (ci, [vp, vp, vp, vp]),
        "gpd_step": (ci, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "gpd_step_seq": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, vp, vp]),
        "gpd_integrate": (ci, [vp, vp, i, vp, vp]),
        "gpd_get_state20": (ci, [vp, vp, vp]),
        "gpd_get_raw_state": (ci, [vp, vp, vp]),
        "gpd_set_raw_state": (ci, [vp, vp, vp]),
        "gpd_get_step_counters": (ci, [vp, vp, vp]),
        "gpd_set_step_counters": (ci, [vp, vp, vp]),
        "gpd_state_bytes": (ctypes.c_size_t, [vp]),
        "gpd_save_state": (ci, [vp, vp, vp]),
        "gpd_load_state": (ci, [vp, vp, vp]),
        "gpd_default_pid_params": (ci, [ctypes.POINTER(PidParams)]),
        "gpd_set_pid_params": (ci, [vp, ctypes.POINTER(PidParams)]),
        "gpd_get_ctrl_state": (ci, [vp, vp, vp]),
        "gpd_set_ctrl_state": (ci, [vp, vp, vp]),
        "gpd_nonfinite": (ci, [vp, vp, vp]),
        "gpd_pack_layout_of": (ci, [i, i, i, ctypes.POINTER(PackLayout)]),
        "gpd_handoff_pack": (ci, [vp, ctypes.POINTER(PackLayout), vp]),
        "gpd_handoff_unpack": (ci, [vp, i, ctypes.c_longlong, ctypes.POINTER(PackLayout), vp, vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name) and os.environ.get("GPD_ALLOW_ABI_MISMATCH"):
            continue   # diagnostics against an older build (A/B timing only)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gpd_abi_version() != GPD_ABI_VERSION and not os.environ.get("GPD_ALLOW_ABI_MISMATCH"):
        raise GpdLibraryError(f"{LIB_PATH} has ABI {lib.gpd_abi_version()}, this binding expects {GPD_ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


def check(fn_name, rc):
    if rc != GPD_OK:
        raise GpdError(fn_name, rc, _lib.gpd_last_error().decode(errors="replace"))
    return rc


def default_pid_params():
    lib = load()
    q = PidParams()
    check("gpd_default_pid_params", lib.gpd_default_pid_params(ctypes.byref(q)))
    return q


def default_params(model):
    lib = load()
    p = DroneParams()
    check("gpd_default_params", lib.gpd_default_params(model, ctypes.byref(p)))
    return p
