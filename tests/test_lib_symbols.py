"""The C-ABI library builds, loads and exports every symbol include/gpd.h declares.

No compute call is made here (no GPU in the CPU suite); only host-side entry points that
never touch the device (ABI version, last error, built-in parameters) are called."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpd.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(gpd_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from gym_pybullet_drones_routing_amd import _build, _lib
    _build.build()
    return _lib.load()


def test_header_and_binding_agree():
    from gym_pybullet_drones_routing_amd import _lib
    assert set(_declared()) == set(_lib.EXPORTED)


def test_every_declared_symbol_is_exported(lib):
    for name in _declared():
        assert hasattr(lib, name), name
    out = os.popen(f"nm -D --defined-only {lib._name}").read()
    for name in _declared():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported as a text symbol"


def test_host_only_entry_points(lib):
    from gym_pybullet_drones_routing_amd import _lib
    assert lib.gpd_abi_version() == _lib.GPD_ABI_VERSION == 7
    assert lib.gpd_nonfinite(None, None, None) == _lib.GPD_EINVAL
    q = _lib.PidParams()
    assert lib.gpd_default_pid_params(ctypes.byref(q)) == _lib.GPD_OK
    assert list(q.p_coeff_tor) == [70000., 70000., 60000.] and q.pwm2rpm_const == 4070.3
    assert [list(r) for r in q.mixer] == [[-.5, -.5, -1], [-.5, .5, 1], [.5, .5, -1], [.5, -.5, 1]]
    assert lib.gpd_default_pid_params(None) == _lib.GPD_EINVAL
    assert lib.gpd_set_pid_params(None, ctypes.byref(q)) == _lib.GPD_EINVAL
    p = _lib.DroneParams()
    assert lib.gpd_default_params(7, ctypes.byref(p)) == _lib.GPD_EINVAL
    assert b"unknown drone model" in lib.gpd_last_error()
    assert lib.gpd_default_params(_lib.GPD_MODEL_CF2X, ctypes.byref(p)) == _lib.GPD_OK
    assert p.kf == 3.16e-10 and p.m == 0.027
    assert lib.gpd_destroy(None) == _lib.GPD_EINVAL
    assert lib.gpd_state_bytes(None) == 0
    # the contact solver's parameters (setPhysicsEngineParameter) are validated before any device call
    cfg = _lib.Config(n_envs=4, drones_per_env=1, pyb_freq=240, ctrl_freq=30, act_type=_lib.GPD_ACT_RPM,
                      task=1, physics_flags=0, precision=_lib.GPD_F64, autoreset=1, episode_len_sec=8.0)
    out = ctypes.c_void_p()
    for it, res, msg in ((1001, 0.0, b"solver_iterations"), (-1, 0.0, b"solver_iterations"),
                         (0, float("nan"), b"solver_residual")):
        cfg.solver_iterations, cfg.solver_residual = it, res
        assert lib.gpd_create(ctypes.byref(p), ctypes.byref(cfg), ctypes.byref(out)) == _lib.GPD_EINVAL
        assert msg in lib.gpd_last_error()


def test_policy_library_host_checks():
    """libgpd_policy.so: ABI 2 and the argument checks that run before any device call - in
    particular the per-row-group Philox counters must cover every sampled row."""
    from gym_pybullet_drones_routing_amd import _build, policy
    _build.build_policy()
    pl = policy.load()
    assert pl.gpd_policy_abi_version() == policy.GPD_POLICY_ABI_VERSION == 2
    st = policy.MlpPolicyStruct()
    st.n_obs, st.n_act = 72, 4
    fake = 256          # never dereferenced: every call below fails its host-side checks
    for n in ("pi_w1", "pi_b1", "pi_w2", "pi_b2", "pi_w3", "pi_b3", "vf_w1", "vf_b1", "vf_w2", "vf_b2", "vf_w3",
              "vf_b3", "log_std"):
        setattr(st, n, fake)
    vp = ctypes.c_void_p
    rc = pl.gpd_policy_rollout_step(ctypes.byref(st), 100, vp(fake), vp(fake), None, vp(fake), None, None, 0,
                                    vp(fake), 6, None, None, None, None, 0.99, None, None, None)
    assert rc == -1 and b"row-group counters" in pl.gpd_policy_last_error()
    assert pl.gpd_policy_rollout_step(None, 100, None, None, None, None, None, None, 0, None, 0, None, None, None,
                                      None, 0.99, None, None, None) == -1


@pytest.mark.parametrize("E,D,W", [(4096, 1, 72), (3, 1, 72), (5, 2, 27), (1, 8, 36), (4095, 3, 27)])
def test_pack_layout_matches_library(lib, E, D, W):
    """sim.pack_layout (the Python restatement the CPU tests use) equals gpd_pack_layout_of; every
    field 256-B aligned (float views at any shard size: ADVICE r5), the record ends where
    terminal_obs begins, invalid shapes rejected (host-only calls: no GPU needed)."""
    from gym_pybullet_drones_routing_amd import _lib
    from gym_pybullet_drones_routing_amd.sim import pack_layout
    L = pack_layout(E, D, W)
    c = _lib.PackLayout()
    assert lib.gpd_pack_layout_of(E, D, W, ctypes.byref(c)) == _lib.GPD_OK
    assert (c.n_envs, c.drones_per_env, c.obs_width, c.state_cols) == (E, D, W, 12)
    for k in ("obs", "reward", "terminated", "truncated", "terminal_state", "terminal_obs"):
        assert getattr(c, k) == L[k][0] and L[k][0] % 256 == 0
    for k in ("prefix", "prefix_aligned", "record", "total"):
        assert getattr(c, k) == L[k]
    assert L["prefix_aligned"] % 256 == 0 and L["record"] == L["terminal_obs"][0]
    assert L["terminal_state"][1] == E * D * 12 * 4
    assert lib.gpd_pack_layout_of(E, D, 11, ctypes.byref(c)) == _lib.GPD_EINVAL
    assert lib.gpd_pack_layout_of(0, D, W, ctypes.byref(c)) == _lib.GPD_EINVAL
    # the pack / unpack entry points validate before touching the device
    assert lib.gpd_handoff_pack(None, ctypes.byref(c), None) == _lib.GPD_EINVAL
    bad = _lib.PackLayout()
    ctypes.memmove(ctypes.byref(bad), ctypes.byref(c), ctypes.sizeof(c))
    bad.record += 256
    assert lib.gpd_handoff_pack(None, ctypes.byref(bad), None) == _lib.GPD_EINVAL
    assert b"layout" in lib.gpd_last_error()


def test_struct_sizes_match_header():
    """ctypes mirrors of gpd_drone_params / gpd_config / gpd_constants have the C layout."""
    from gym_pybullet_drones_routing_amd import _lib
    # the C compiler's view of include/gpd.h (sizes and a few field offsets)
    import subprocess
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = r"""
#include <stdio.h>
#include <stddef.h>
typedef void* hipStream_t;
#include "gpd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(gpd_drone_params), sizeof(gpd_config), sizeof(gpd_constants),
         sizeof(gpd_pid_params), offsetof(gpd_config, episode_len_sec), offsetof(gpd_config, drones_per_block),
         offsetof(gpd_config, store_policy), sizeof(gpd_pack_layout), offsetof(gpd_pack_layout, record));
  printf(" %zu %zu\n", offsetof(gpd_config, solver_iterations), offsetof(gpd_config, solver_residual));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "t.c"), "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(root, "include"), "-o", os.path.join(d, "t"), os.path.join(d, "t.c")],
                       check=True)
        got = [int(x) for x in subprocess.run([os.path.join(d, "t")], capture_output=True, text=True,
                                              check=True).stdout.split()]
    assert got[:4] == [ctypes.sizeof(_lib.DroneParams), ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.Constants),
                       ctypes.sizeof(_lib.PidParams)]
    assert got[4:7] == [_lib.Config.episode_len_sec.offset, _lib.Config.drones_per_block.offset,
                        _lib.Config.store_policy.offset]
    assert got[7:9] == [ctypes.sizeof(_lib.PackLayout), _lib.PackLayout.record.offset]
    assert got[9:] == [_lib.Config.solver_iterations.offset, _lib.Config.solver_residual.offset]


def test_abi_version_consistent():
    """include/gpd.h, the ctypes binding and the built library agree on GPD_ABI_VERSION (and
    __graft_entry__.build() checks against the binding, not a literal)."""
    from gym_pybullet_drones_routing_amd import _lib
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "gpd.h")).read()
    m = re.search(r"#define GPD_ABI_VERSION (\d+)", hdr)
    assert m and int(m.group(1)) == _lib.GPD_ABI_VERSION
    assert _lib.load().gpd_abi_version() == _lib.GPD_ABI_VERSION
    entry = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "__graft_entry__.py")).read()
    assert "gpd_abi_version() == _lib.GPD_ABI_VERSION" in entry
