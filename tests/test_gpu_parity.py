"""GPU-vs-oracle parity of the HIP DYN path (called through the C ABI via ctypes).

Tolerances (BASELINE.json north_star / SURVEY §8(d)): per-drone relative L2 error of the
state (pos, quat, rpy, vel, ang_v) vs the fp64 oracle over every substep of a 5 s
(1200-substep) run:
  * fp64 kernel (the default, parity path): max <= 1e-10   (measured ~5e-14)
  * fp32 kernel (opt-in fast path): median <= 1e-5 and max <= 1e-3.  Open-loop quadrotor
    attitude dynamics amplify float32 rounding (an omega error e grows into a position error
    ~ e*g*t^2/2), so the 1e-5 max gate is NOT met in fp32 for tumbling drones (measured max
    7e-5, median 2e-6 at 5 s); the parity claim is made for the fp64 path.
"""
import numpy as np
import pytest
import torch

from oracle.ref_aviary import RefAviary, rpm_from_action
from tests.oracle_runs import assert_obs_match, run_integrate, run_vec, state_rel_err

pytestmark = pytest.mark.gpu

TOL = {"f64": 1e-10, "f32": 1e-3}
TOL_MEDIAN = {"f64": 1e-10, "f32": 1e-5}
HOVER = 14468.429183500699


def _sim(**kw):
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    return BatchedAviarySim(device="cuda:0", **kw)


def _random_raw(rng, n, z=1.0, tilt=0.3, spin=2.0):
    """Random but well-defined raw states: position, orientation within `tilt` rad, body rates."""
    from oracle.bullet_math import quat_from_euler, quat_roundtrip
    raw = np.zeros((n, 20))
    raw[:, 0:2] = rng.uniform(-0.5, 0.5, (n, 2))
    raw[:, 2] = z + rng.uniform(-0.05, 0.05, n)
    for i in range(n):
        raw[i, 3:7] = quat_roundtrip(quat_from_euler(rng.uniform(-tilt, tilt, 3)))
    raw[:, 7:10] = rng.uniform(-0.5, 0.5, (n, 3))
    raw[:, 10:13] = rng.uniform(-spin, spin, (n, 3))
    raw[:, 16:20] = HOVER
    return raw


def _rpms(rng, T, n, scale=1.0):
    a = rng.uniform(-1, 1, (T, n, 4)).astype(np.float32) * np.float32(scale)
    return rpm_from_action(HOVER, a)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_integrate_parity_5s(prec):
    rng = np.random.default_rng(0)
    n, T = 64, 1200
    raw0 = _random_raw(rng, n)
    rpms = _rpms(rng, T, n)
    ref = run_integrate(rpms, raw0)
    sim = _sim(n_envs=n, task="none", precision=prec)
    sim.set_raw_state(raw0)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    err = state_rel_err(traj, ref)
    print(f"\n[parity] integrate {prec}: max rel err {err.max():.3e} median {np.median(err):.3e} (tol {TOL[prec]:.0e})")
    assert np.isfinite(traj).all()
    assert err.max() <= TOL[prec]
    assert np.median(err) <= TOL_MEDIAN[prec]
    sim.close()


def test_integrate_zero_rate_keeps_quaternion():
    """KAT-5 on the GPU: with |omega| <= 1e-8 _integrateQ returns its input, i.e. the
    read-back (re-normalised) orientation, and the body rates stay exactly zero."""
    from oracle.bullet_math import quat_roundtrip
    sim = _sim(n_envs=4, task="none", precision="f64")
    raw = np.zeros((4, 20))
    raw[:, 2] = 1.0
    raw[:, 3:7] = [[0, 0, 0, 1], [0.1, 0, 0, 0.99498743710662], [0, 0.2, 0, 0.9797958971132712],
                   [0, 0, 0.3, 0.9539392014169456]]
    sim.set_raw_state(raw)
    # equal rpm on all four props -> zero DYN torques -> omega stays exactly 0
    sim.integrate(np.full((5, 4, 4), HOVER))
    out = sim.raw_state().cpu().numpy()
    assert np.array_equal(out[:, 10:13], np.zeros((4, 3)))
    expect = np.array([quat_roundtrip(q) for q in raw[:, 3:7]])
    np.testing.assert_allclose(out[:, 3:7], expect, rtol=0, atol=4.5e-16)  # fused readback: <= 2 ulp
    sim.close()


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("aero", [("gnd",), ("drag",), ("gnd", "drag")])
def test_integrate_aero_parity(prec, aero):
    rng = np.random.default_rng(1)
    n, T = 32, 1200
    raw0 = _random_raw(rng, n, z=0.06, tilt=0.2, spin=0.5)   # in ground effect
    rpms = _rpms(rng, T, n, scale=0.5)
    ref = run_integrate(rpms, raw0, aero=aero)
    sim = _sim(n_envs=n, task="none", precision=prec, aero=aero)
    sim.set_raw_state(raw0)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    err = state_rel_err(traj, ref)
    print(f"\n[parity] integrate {prec} {aero}: max rel err {err.max():.3e} median {np.median(err):.3e}")
    assert err.max() <= TOL[prec]
    assert np.median(err) <= TOL_MEDIAN[prec]
    sim.close()


def test_integrate_geom_wrench_parity():
    rng = np.random.default_rng(2)
    n, T = 16, 600
    raw0 = _random_raw(rng, n)
    rpms = _rpms(rng, T, n)
    ref = run_integrate(rpms, raw0, wrench="geom")
    sim = _sim(n_envs=n, task="none", precision="f64", aero=("geom",))   # PYB force placement on DYN
    sim.set_raw_state(raw0)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    assert state_rel_err(traj, ref).max() <= TOL["f64"]
    sim.close()


def _staggered(D=8):
    """C4 init: drone i at (0.15cos, 0.15sin, 0.5+0.1i)."""
    i = np.arange(D)
    return np.stack([0.15 * np.cos(2 * np.pi * i / D), 0.15 * np.sin(2 * np.pi * i / D), 0.5 + 0.1 * i], 1)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_downwash_multi_parity(prec):
    rng = np.random.default_rng(3)
    E, D, T = 4, 8, 600
    xyz = _staggered(D)
    rpms = _rpms(rng, T, E * D, scale=0.3)
    refs = []
    for e in range(E):
        env = RefAviary(num_drones=D, task="none", aero=("dw",), initial_xyzs=xyz)
        refs.append(env.integrate(rpms[:, e * D:(e + 1) * D]))
    ref = np.concatenate(refs, axis=1)
    sim = _sim(n_envs=E, drones_per_env=D, task="none", precision=prec, aero=("dw",), initial_xyzs=xyz)
    traj = sim.integrate(rpms, record=True).cpu().numpy()
    err = state_rel_err(traj, ref)
    print(f"\n[parity] downwash {prec}: max rel err {err.max():.3e}")
    assert err.max() <= TOL[prec]
    # the downwash really acted: compare against a run without it
    nodw = RefAviary(num_drones=D, task="none", initial_xyzs=xyz).integrate(rpms[:, :D])
    assert np.abs(nodw[-1, :, 2] - ref[-1, :D, 2]).max() > 1e-4
    sim.close()


WAVES = {"io": 3, "duo": 2, "single": 1}


@pytest.mark.parametrize("kernel", ["io", "duo", "single"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("act", ["rpm", "one_d_rpm"])
def test_step_parity_hover(prec, act, kernel):
    """HoverAviary step(): obs / reward / terminated / truncated with SB3 auto-reset, through the
    three-wave step kernel (pose + rate + io waves, the default up to 64K drones), the two-wave
    one and the single-wave one (larger N)."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(4)
    E, T = 16, 80
    A = 4 if act == "rpm" else 1
    # hover-biased actions keep episodes alive; a few envs get full-range actions to force resets
    acts = np.clip(rng.normal(0, 0.1, (T, E, 1, A)), -1, 1).astype(np.float32)
    acts[:, :4] = rng.uniform(-1, 1, (T, 4, 1, A)).astype(np.float32)
    if A == 1:
        acts[:, 4:6] = 1.0   # full collective thrust: climbs through z > 2 -> truncation + reset
    obs_r, rew_r, te_r, tr_r, tobs_r = run_vec(acts, E, act=act)
    sim = _sim(n_envs=E, task="hover", precision=prec, act=ActionType(act), tuning={"step_waves": WAVES[kernel]})
    assert sim.constants.lanes_per_block == 64 * WAVES[kernel]
    obs0 = sim.obs.cpu().numpy()
    assert obs0.shape == (E, 1, 12 + 15 * A)
    n_done = 0
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        o, r, te, tr = o.cpu().numpy(), r.cpu().numpy(), te.cpu().numpy().astype(bool), tr.cpu().numpy().astype(bool)
        if prec == "f64":
            np.testing.assert_array_equal(te, te_r[t])
            np.testing.assert_array_equal(tr, tr_r[t])
            assert_obs_match(o, obs_r[t], 1e-5, 1e-6)
            np.testing.assert_allclose(r, rew_r[t], rtol=1e-6, atol=1e-6)
        else:
            same = (te == te_r[t]) & (tr == tr_r[t])
            assert same.all(), f"done flags differ at step {t}"
            assert_obs_match(o, obs_r[t], 1e-4, 1e-4)
            np.testing.assert_allclose(r, rew_r[t], rtol=1e-4, atol=1e-4)
        tobs = sim.terminal_obs.cpu().numpy()
        for e in np.nonzero(te | tr)[0]:
            n_done += 1
            assert_obs_match(tobs[e], tobs_r[(t, e)], 1e-4, 1e-4)
    assert n_done > 0, "test inputs should force at least one auto-reset"
    sim.close()


@pytest.mark.parametrize("dpb", [0, 4, 8, 64])
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("act", ["rpm", "one_d_rpm"])
def test_duo_kernel_matches_single_wave(prec, act, dpb):
    """The two-wave step kernel runs dyn_substep's operations split over two waves: the same
    obs, reward, done flags and state as the single-wave kernel up to rounding (hipcc contracts
    a few multiply-adds differently in the two code shapes: measured 1 ulp in f64); the
    three-wave kernel (io wave for the history columns) is bit-identical to the two-wave one.
    Ragged env count (the last block is partial), full-range actions (resets, tumbling drones
    past the small-angle series), 60 steps, automatic and pinned block sizes."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(21)
    E, T = 100, 60
    A = 4 if act == "rpm" else 1
    acts = rng.uniform(-1, 1, (T, E, 1, A)).astype(np.float32)
    acts[:, :50] *= np.float32(0.1)
    out = {}
    for kernel in ("io", "duo", "single"):
        sim = _sim(n_envs=E, task="hover", precision=prec, act=ActionType(act),
                   tuning={"step_waves": WAVES[kernel], "drones_per_block": dpb})
        assert sim.constants.lanes_per_block == 64 * WAVES[kernel]
        assert dpb == 0 or sim.constants.drones_per_block == dpb
        rec = []
        for t in range(T):
            o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
            rec.append((o.cpu().numpy().copy(), r.cpu().numpy().copy(), te.cpu().numpy().copy(),
                        tr.cpu().numpy().copy(), sim.terminal_obs.cpu().numpy().copy()))
        out[kernel] = (rec, sim.state20().cpu().numpy())
        sim.close()
    # the io and two-wave kernels run the same pose/rate code: bit-identical
    (ri, si), (ra, sa), (rb, sb) = out["io"], out["duo"], out["single"]
    for t in range(T):
        for x, y in zip(ri[t], ra[t]):
            np.testing.assert_array_equal(x, y, err_msg=f"io vs duo, step {t}")
    np.testing.assert_array_equal(si, sa)
    tol = 1e-12 if prec == "f64" else 1e-4
    for t in range(T):
        (oa, rwa, tea, tra, ta), (ob, rwb, teb, trb, tb) = ra[t], rb[t]
        np.testing.assert_array_equal(tea, teb, err_msg=f"terminated, step {t}")
        np.testing.assert_array_equal(tra, trb, err_msg=f"truncated, step {t}")
        for x, y in ((oa, ob), (ta, tb)):
            assert_obs_match(x, y, tol, tol if prec == "f64" else 1e-5, err_msg=f"step {t}")
        np.testing.assert_allclose(rwa, rwb, rtol=tol, atol=tol if prec == "f64" else 1e-5, err_msg=f"step {t}")
    assert state_rel_err(sa, sb).max() <= tol


@pytest.mark.parametrize("D", [2, 8])
def test_step_parity_multihover(D):
    rng = np.random.default_rng(5)
    E, T = 6, 40
    acts = np.clip(rng.normal(0, 0.2, (T, E, D, 4)), -1, 1).astype(np.float32)
    obs_r, rew_r, te_r, tr_r, _ = run_vec(acts, E, drones_per_env=D, task="multihover")
    sim = _sim(n_envs=E, drones_per_env=D, task="multihover", precision="f64")
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        np.testing.assert_array_equal(te.cpu().numpy().astype(bool), te_r[t])
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), tr_r[t])
        assert_obs_match(o.cpu().numpy(), obs_r[t], 1e-5, 1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), rew_r[t], rtol=1e-6, atol=1e-5)
    sim.close()


def test_truncation_at_step_242_and_history_survives_reset():
    """KAT-9 on the GPU: hover actions -> time truncation exactly at ctrl step 242; the action
    history in the reset observation still holds the previous episode's actions."""
    sim = _sim(n_envs=3, task="hover", precision="f32")
    a = np.zeros((3, 1, 4), np.float32)
    for k in range(1, 243):
        a[:] = (k % 7) * 0.01
        o, r, te, tr = sim.step(torch.from_numpy(a).cuda())
        trn = tr.cpu().numpy()
        if k < 242:
            assert not trn.any(), k
    assert trn.all()
    o = o.cpu().numpy()
    assert np.allclose(o[:, 0, 0:3], [0, 0, 0.1125])          # reset pose
    assert np.allclose(o[:, 0, -4:], (242 % 7) * 0.01)        # newest action kept
    sim.close()


def test_raw_state_and_checkpoint_roundtrip():
    rng = np.random.default_rng(6)
    sim = _sim(n_envs=32, task="hover", precision="f32")
    for _ in range(5):
        sim.step(torch.from_numpy(rng.uniform(-0.2, 0.2, (32, 1, 4)).astype(np.float32)).cuda())
    blob = sim.save_state()
    raw = sim.raw_state().cpu().numpy()
    sc = sim.step_counters().cpu().numpy()
    a = torch.from_numpy(rng.uniform(-0.2, 0.2, (32, 1, 4)).astype(np.float32)).cuda()
    o1 = sim.step(a)[0].clone()
    sim.load_state(blob)
    np.testing.assert_array_equal(sim.raw_state().cpu().numpy(), raw)
    np.testing.assert_array_equal(sim.step_counters().cpu().numpy(), sc)
    o2 = sim.step(a)[0]
    assert torch.equal(o1, o2)
    sim.close()


def test_state20_matches_oracle_layout():
    rng = np.random.default_rng(7)
    raw0 = _random_raw(rng, 8)
    sim = _sim(n_envs=8, task="none", precision="f64")
    sim.set_raw_state(raw0)
    s20 = sim.state20().cpu().numpy()
    env = RefAviary(num_drones=8, task="none")
    env.set_raw_state(raw0)
    np.testing.assert_allclose(s20, env.state20(), rtol=0, atol=1e-14)
    sim.close()


def test_graph_replay_matches_eager():
    """gpd_step is a fixed-argument launch (ring head + step counters in device memory), so a
    captured sequence replayed twice equals 2x the same steps launched eagerly, bit for bit."""
    rng = np.random.default_rng(8)
    E, G = 64, 5
    acts = [torch.from_numpy(rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)).cuda() for _ in range(G)]
    a = _sim(n_envs=E, task="hover", precision="f64")
    b = _sim(n_envs=E, task="hover", precision="f64")
    g = b.capture_graph(acts)
    for rep in range(2):
        for k in range(G):
            a.step(acts[k])
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b.obs)
    assert torch.equal(a.raw_state(), b.raw_state())
    assert torch.equal(a.step_counters(), b.step_counters())
    a.close()
    b.close()


@pytest.mark.parametrize("act", ["rpm", "one_d_rpm"])
def test_step_seq_matches_steps(act):
    """gpd_step_seq(P slots, T steps) == T gpd_step calls on slots t % P, bit for bit (outputs,
    terminal rows, state, counters, action ring via the next observation), past auto-resets."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(9)
    E, P, T = 96, 7, 40
    A = 4 if act == "rpm" else 1
    pool = torch.from_numpy(rng.uniform(-1, 1, (P, E, 1, A)).astype(np.float32)).cuda()
    a = _sim(n_envs=E, task="hover", precision="f64", act=ActionType(act))
    b = _sim(n_envs=E, task="hover", precision="f64", act=ActionType(act))
    for t in range(T):
        a.step(pool[t % P])
    b.step_seq(pool, T)
    torch.cuda.synchronize()
    for x, y in ((a.obs, b.obs), (a.reward, b.reward), (a.terminated, b.terminated), (a.truncated, b.truncated),
                 (a.terminal_obs, b.terminal_obs), (a.raw_state(), b.raw_state()), (a.step_counters(), b.step_counters())):
        assert torch.equal(x, y)
    a.step(pool[0])
    b.step(pool[0])
    assert torch.equal(a.obs, b.obs)
    a.close()
    b.close()


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_gpu_kat_hover_and_symmetric_thrust(prec):
    """KAT-1 on the GPU (hover from rest stays put) and the symmetry the reference has exactly:
    four equal RPMs (any ONE_D_RPM action) give zero roll/pitch torque, so x, y, roll, pitch
    and the body rates stay exactly 0 while z moves."""
    n, T = 8, 1200
    sim = _sim(n_envs=n, task="none", precision=prec)
    traj = sim.integrate(np.full((T, n, 4), HOVER), record=True).cpu().numpy()
    s0 = traj[0, 0]
    # float32 cannot represent the hover equilibrium exactly (4*kf*rpm^2 - M*G ~ 1e-9 N), so
    # the fp32 drone drifts by ~0.5*a*t^2 ~ 1e-5 m in 5 s; fp64 stays put to 1e-12.
    tol = 1e-12 if prec == "f64" else 1e-4
    assert np.abs(traj[..., :16] - s0[:16]).max() <= tol
    sim.close()
    rng = np.random.default_rng(9)
    rpm = np.repeat(rpm_from_action(HOVER, rng.uniform(-1, 1, (T, n, 1)).astype(np.float32)), 4, axis=2)
    sim = _sim(n_envs=n, task="none", precision=prec)
    traj = sim.integrate(rpm, record=True).cpu().numpy()
    for col in (0, 1, 7, 8, 13, 14):   # x, y, roll, pitch, ang_v x, ang_v y
        assert np.abs(traj[..., col]).max() == 0.0, col
    sim.close()


@pytest.mark.parametrize("case", ["c3_gnd_drag", "c4_downwash"])
def test_step_parity_aero_configs(case):
    """BASELINE configs 3 and 4 through step(): ground effect + drag on single-drone hover envs,
    and 8-drone MultiHover envs with downwash from a staggered start."""
    import math
    from gym_pybullet_drones_routing_amd.enums import ActionType
    rng = np.random.default_rng(21)
    if case == "c3_gnd_drag":
        E, D, T, task, aero, xyz = 16, 1, 60, "hover", ("gnd", "drag"), None
    else:
        E, D, T, task, aero = 4, 8, 40, "multihover", ("dw",)
        xyz = [[0.15 * math.cos(2 * math.pi * i / 8), 0.15 * math.sin(2 * math.pi * i / 8), 0.5 + 0.1 * i]
               for i in range(8)]
    acts = np.clip(rng.normal(0, 0.2, (T, E, D, 4)), -1, 1).astype(np.float32)
    envs = []
    obs_r, rew_r, te_r, tr_r, _ = run_vec(acts, E, drones_per_env=D, task=task, aero=aero, initial_xyzs=xyz,
                                          envs=envs)
    sim = _sim(n_envs=E, drones_per_env=D, task=task, precision="f64", act=ActionType.RPM, aero=aero,
               initial_xyzs=xyz)
    for t in range(T):
        o, r, te, tr = sim.step(torch.from_numpy(acts[t]).cuda())
        np.testing.assert_array_equal(te.cpu().numpy().astype(bool), te_r[t])
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), tr_r[t])
        assert_obs_match(o.cpu().numpy(), obs_r[t], 1e-5, 1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), rew_r[t], rtol=1e-6, atol=1e-5)
    ref = np.concatenate([e.state20() for e in envs])
    err = state_rel_err(sim.state20().cpu().numpy(), ref)
    assert err.max() <= TOL["f64"], err.max()
    sim.close()


def test_abi_error_paths():
    """Bad arguments come back as GPD_EINVAL with a message, never as a fault."""
    import ctypes
    from gym_pybullet_drones_routing_amd import _lib
    lib = _lib.load()
    sim = _sim(n_envs=4, task="hover", precision="f64")
    h = sim._h
    obs = torch.zeros((4, 1, 72), device="cuda:0")
    rew = torch.zeros(4, device="cuda:0")
    te = torch.zeros(4, dtype=torch.uint8, device="cuda:0")
    tr = torch.zeros(4, dtype=torch.uint8, device="cuda:0")
    acts = torch.zeros((4 * 4 + 1,), device="cuda:0")
    vp = ctypes.c_void_p
    rc = lib.gpd_step(h, None, vp(obs.data_ptr()), vp(rew.data_ptr()), vp(te.data_ptr()), vp(tr.data_ptr()), None, None)
    assert rc == _lib.GPD_EINVAL and b"NULL" in lib.gpd_last_error()
    rc = lib.gpd_step(h, vp(acts.data_ptr() + 4), vp(obs.data_ptr()), vp(rew.data_ptr()), vp(te.data_ptr()),
                      vp(tr.data_ptr()), None, None)
    assert rc == _lib.GPD_EINVAL and b"aligned" in lib.gpd_last_error()
    assert lib.gpd_integrate(h, vp(acts.data_ptr()), -1, None, None) == _lib.GPD_EINVAL
    assert lib.gpd_get_ctrl_state(h, vp(obs.data_ptr()), None) == _lib.GPD_EINVAL   # RPM sim has no controller
    other = _sim(n_envs=5, task="hover", precision="f64")
    ob = ctypes.create_string_buffer(lib.gpd_state_bytes(other._h))
    assert lib.gpd_save_state(other._h, ctypes.cast(ob, vp), None) == _lib.GPD_OK
    assert lib.gpd_load_state(h, ctypes.cast(ob, vp), None) == _lib.GPD_EINVAL      # blob of another sim
    with pytest.raises(ValueError):
        sim.step(torch.zeros((4, 1, 3), device="cuda:0"))                           # wrong action width
    sim.close()
    other.close()
