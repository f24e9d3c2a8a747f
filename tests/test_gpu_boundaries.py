"""Edge cases at the reference's decision thresholds, where a rounding difference flips a flag:

* HoverAviary ``np.linalg.norm(TARGET_POS - pos) < .0001`` (HoverAviary.py:92);
* MultiHoverAviary's summed distance ``dist < .0001`` accumulated in fp64
  (MultiHoverAviary.py:101-104) - one case flips if the sum is formed in float32;
* the downwash cull ``delta_z > 0 and delta_xy < 10`` (BaseAviary.py:801) at delta_xy = 10,
  including dx = 6, dy = 7.999999999999999 where dx^2 + dy^2 rounds to the double just below
  100 but its square root rounds to exactly 10 (culled by the reference, kept by a naive
  ``dxy^2 < 100``).

Drones start at rest at the hover action.  The RPM is float32-rounded (BaseRLAviary.py:191-192,
numpy 1.x scalar*float32 -> float32), so thrust and weight differ by ~1e-8 and one control step
moves a drone by ~6e-11 m in z: a first step measures that drift and the drones then start
that far below their targets, so the distances at the test are the seeded x offsets to ~1e-28.
Expected flags come from numpy fp64 on the GPU's own final positions (the reference's
arithmetic).
"""
import numpy as np
import pytest
import torch

from oracle.ref_aviary import RefAviary
from tests.oracle_runs import state_rel_err

pytestmark = pytest.mark.gpu

HOVER = 14468.429183500699


def _rest_raw(pos):
    pos = np.asarray(pos, dtype=np.float64)
    raw = np.zeros((len(pos), 20))
    raw[:, 0:3] = pos
    raw[:, 6] = 1.0
    raw[:, 16:20] = HOVER
    return raw


def _drift_corrected(make_sim, pos, actions):
    """Start positions that land on `pos` (up to an ulp of z) after one step from rest."""
    sim = make_sim()
    sim.set_raw_state(_rest_raw(pos))
    sim.step(actions)
    moved = sim.state20().cpu().numpy()[:, 0:3] - pos
    sim.close()
    assert np.abs(moved).max() < 1e-9
    return pos - moved


def test_hover_terminated_at_1e4_boundary():
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    b = 1e-4
    dxs = np.array([np.nextafter(b, 0), b, np.nextafter(b, 1), 0.0, 0.5e-4, -np.nextafter(b, 0), -b, 3e-4])
    E = len(dxs)
    target = np.array([0.0, 0.0, 1.0])
    def make():
        return BatchedAviarySim(n_envs=E, task="hover", precision="f64", autoreset=False, device="cuda:0")
    zero = torch.zeros((E, 1, 4), device="cuda:0")
    start = _drift_corrected(make, target + np.stack([dxs, 0 * dxs, 0 * dxs], 1), zero)
    sim = make()
    sim.set_raw_state(_rest_raw(start))
    _, _, te, tr = sim.step(zero)
    pos = sim.state20().cpu().numpy()[:, 0:3]
    np.testing.assert_array_equal(pos[:, 0], dxs)                    # x did not move
    expect = np.array([np.linalg.norm(target - p) < .0001 for p in pos])
    np.testing.assert_array_equal(expect, [True, False, False, True, True, True, False, False])
    np.testing.assert_array_equal(te.cpu().numpy().astype(bool), expect)
    assert not tr.cpu().numpy().any()
    sim.close()


def test_multihover_summed_distance_is_fp64():
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    init = np.array([[0.0, 0.0, 0.1], [1.0, 1.0, 0.1]])
    target = init + np.array([[0, 0, 1 / (i + 1)] for i in range(2)])   # MultiHoverAviary.py:71
    # offsets at the exact boundary go to drone 0 (target x = 0: the distance is the offset
    # itself); drone 1 (target x = 1) only carries offsets with margins far above 1e-16
    cases = [(4.99999999e-5, 5e-5), (1e-4, 0.0), (4.9e-5, 5e-5), (6e-5, 5e-5), (np.nextafter(1e-4, 0), 0.0),
             (7.4999999e-5, 2.5e-5)]
    E = len(cases)
    pos = np.concatenate([target + np.array([[d0, 0, 0], [d1, 0, 0]]) for d0, d1 in cases])
    def make():
        return BatchedAviarySim(n_envs=E, drones_per_env=2, task="multihover", precision="f64", autoreset=False,
                                initial_xyzs=init, device="cuda:0")
    zero = torch.zeros((E, 2, 4), device="cuda:0")
    start = _drift_corrected(make, pos, zero)
    sim = make()
    sim.set_raw_state(_rest_raw(start))
    _, rew, te, _ = sim.step(zero)
    p = sim.state20().cpu().numpy()[:, 0:3].reshape(E, 2, 3)
    expect = np.array([sum(np.linalg.norm(target[i] - p[e, i]) for i in range(2)) < .0001 for e in range(E)])
    np.testing.assert_array_equal(expect, [True, False, True, False, True, True])
    # the test has power: the same sums formed in float32 flip at least one flag
    f32 = np.array([(np.float32(np.linalg.norm(target[0] - p[e, 0])) + np.float32(np.linalg.norm(target[1] - p[e, 1])))
                    < np.float32(1e-4) for e in range(E)])
    assert (f32 != expect).any()
    np.testing.assert_array_equal(te.cpu().numpy().astype(bool), expect)
    exp_rew = np.array([sum(max(0, 2 - np.linalg.norm(target[i] - p[e, i]) ** 4) for i in range(2)) for e in range(E)],
                       dtype=np.float32)
    np.testing.assert_array_equal(rew.cpu().numpy(), exp_rew)
    sim.close()


@pytest.mark.parametrize("dxy,active", [
    ((np.nextafter(10.0, 0), 0.0), True),
    ((10.0, 0.0), False),
    ((6.0, np.nextafter(8.0, 0)), False),          # dx^2 + dy^2 = pred(100), sqrt rounds to 10
    ((6.0, np.nextafter(np.nextafter(8.0, 0), 0)), True),
    ((0.0, 9.99), True),
], ids=["just_inside", "at_10", "sqrt_rounds_to_10", "below_pred100", "inside"])
def test_downwash_cull_at_10(dxy, active):
    """Lower drone at (0,0,1), upper drone at (dx, dy, 51): beta = 0.16*50 - 0.11 = 7.89, so the
    force at delta_xy ~ 10 is exp(-0.8)-sized and visible in the lower drone's z velocity."""
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    dx, dy = dxy
    xyz = np.array([[0.0, 0.0, 1.0], [dx, dy, 51.0]])
    raw = _rest_raw(xyz)
    rpm = np.full((1, 2, 4), HOVER)
    sim = BatchedAviarySim(n_envs=1, drones_per_env=2, task="none", aero=("dw",), precision="f64",
                           initial_xyzs=xyz, device="cuda:0")
    sim.set_raw_state(raw)
    traj = sim.integrate(rpm, record=True).cpu().numpy()[0]
    ref = RefAviary(num_drones=2, task="none", aero=("dw",), initial_xyzs=xyz)
    ref.set_raw_state(raw)
    rtraj = ref.integrate(rpm)[0]
    dxy_ref = np.linalg.norm(np.array([dx, dy]))
    assert (dxy_ref < 10) == active
    vz = traj[0, 12]                   # state20: vel at columns 10..12
    if active:
        assert vz < -1e-7, vz          # pushed down by the drone above
    else:
        assert abs(vz) < 1e-12, vz
    assert state_rel_err(traj, rtraj).max() <= 1e-10
    sim.close()


def test_nonfinite_guard_flags_only_the_poisoned_env():
    """gpd_nonfinite: a NaN seeded into one drone of env 2 (as the downwash quotient
    at beta = 0 would produce, BaseAviary.py:802-804) flags env 2 only, before and after a step;
    the other envs step on unaffected."""
    from gym_pybullet_drones_routing_amd.enums import ActionType
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    E, D = 6, 2
    sim = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM, device="cuda:0")
    assert not sim.nonfinite().any()
    raw = sim.raw_state().cpu().numpy()
    raw[2 * D + 1, 8] = np.nan
    sim.set_raw_state(raw)
    assert sim.nonfinite().cpu().numpy().tolist() == [False, False, True, False, False, False]
    ref = BatchedAviarySim(n_envs=E, drones_per_env=D, task="multihover", act=ActionType.RPM, device="cuda:0")
    acts = torch.zeros((E, D, 4), device="cuda:0")
    sim.step(acts)
    ref.step(acts)
    assert sim.nonfinite().cpu().numpy().tolist() == [False, False, True, False, False, False]
    a, b = sim.state20().cpu().numpy(), ref.state20().cpu().numpy()
    keep = np.ones(E * D, bool)
    keep[2 * D:3 * D] = False
    np.testing.assert_array_equal(a[keep], b[keep])
    sim.close()
    ref.close()


# ---------------------------------------------------------------- attitude thresholds
# The reference's attitude decisions are made on libm atan2 / asin outputs of the readback
# quaternion (HoverAviary.py:111, MultiHoverAviary.py:124, BaseAviary.py:742).  The kernels
# decide the lanes within ~1e-12 of a threshold exactly (gpd_device.h attitude_decide; the rules
# are pinned against glibc in tests/test_attitude_rules.py).  Expected flags come from the
# oracle's literal readback + glibc on the GPU's own stored quaternions after the step; the only
# tolerated difference is a case where glibc's atan2 is not correctly rounded (within 1e-2 ulp
# of a rounding midpoint), and there the GPU must give the correctly rounded decision.

def _level_raw(n, xyz):
    raw = np.zeros((n, 20))
    raw[:, 0:3] = xyz
    raw[:, 6] = 1.0
    raw[:, 16:20] = HOVER
    return raw


def _expect_tilt(quats):
    from tests.attitude_cases import literal_args, tilted
    from tests.test_attitude_rules import kernel_tilt
    exp, kern = [], []
    for q in quats:
        exp.append(tilted(q))
        kern.append(kernel_tilt(*literal_args(q)))
    return np.array(exp), np.array(kern)


def _check_tilt(got, quats):
    exp, kern = _expect_tilt(quats)
    np.testing.assert_array_equal(got, kern)          # the exact rule, always
    mis = np.nonzero(exp != kern)[0]                   # glibc misroundings only
    assert len(mis) <= 2, mis
    return exp


@pytest.mark.parametrize("kind", ["hover", "multihover2", "wide65"])
def test_truncation_at_roll_pitch_limit(kind):
    """|roll| or |pitch| = 0.4 +- a few ulp, both signs, with yaw and a second tilt axis, plus
    roll near +-pi (b <= 0) and exactly +-pi/2 (b = +-0): `truncated` bit for bit."""
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    from tests.attitude_cases import oracle_rpy, roll_beyond_half_pi_cases, tilt_cases
    q, _ = tilt_cases()
    q = np.concatenate([q, roll_beyond_half_pi_cases()])
    K = len(q)
    D = {"hover": 1, "multihover2": 2, "wide65": 65}[kind]
    init = np.array([[(i % 8) * 0.2 - 0.7, (i // 8) * 0.2 - 0.8, 0.5] for i in range(D)])   # inside the bounds
    sim = BatchedAviarySim(n_envs=K, drones_per_env=D, task="hover" if D == 1 else "multihover",
                           precision="f64", autoreset=False, initial_xyzs=init, device="cuda:0")
    raw = np.concatenate([_level_raw(D, init) for _ in range(K)])
    raw[0::D, 3:7] = q                                 # drone 0 of every env sits at the boundary
    sim.set_raw_state(raw)
    _, _, _, tr = sim.step(torch.zeros((K, D, 4), device="cuda:0"))
    after = sim.raw_state().cpu().numpy()
    assert np.abs(after[:, 0:2]).max() < 1.5 and after[:, 2].max() < 2.0     # inside the position bounds
    exp = _check_tilt(tr.cpu().numpy().astype(bool), after[0::D, 3:7])
    # power: decisions at |angle| within 4 ulp of 0.4 fall both ways
    near = []
    for x, e in zip(after[0::D, 3:7], exp):
        r = oracle_rpy(x)
        d = min(abs(abs(r[0]) - 0.4), abs(abs(r[1]) - 0.4)) / np.spacing(0.4)
        if d <= 4:
            near.append(e)
    assert 0 < sum(near) < len(near), near
    sim.close()


def _zero_rpy(t, keep):
    out = np.zeros_like(t)
    out[..., keep] = t[..., keep]
    return out


@pytest.mark.parametrize("physics", ["dyn", "pyb"])
def test_ground_effect_gate_at_half_pi_and_gimbal_edge(physics):
    """The ground-effect gate |roll|, |pitch| < pi/2 (BaseAviary.py:742) at roll = pi/2 - ~1e-16
    (atan2 rounds to RN(pi/2) or just below) and at the getEulerZYX gimbal edge |sarg| = 0.99999 +-
    ulp: one substep (gpd_integrate) from each stored quaternion against the oracle.  A wrong gate
    moves the velocity by ~1e-3 (the ground effect is ~3 % of the thrust at this height)."""
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    from oracle.ref_aviary import RefAviary
    from tests.attitude_cases import upright, upright_edge_cases
    q = upright_edge_cases()
    K = len(q)
    aero = ("gnd",) if physics == "dyn" else ("bullet", "gnd", "no_plane")
    raw = _level_raw(K, np.array([0.0, 0.0, 0.1125]))
    raw[:, 3:7] = q
    rpm = np.full((1, K, 4), HOVER)
    sim = BatchedAviarySim(n_envs=K, task="none", aero=aero, precision="f64", device="cuda:0")
    sim.set_raw_state(raw)
    traj = sim.integrate(rpm, record=True).cpu().numpy()[0]
    ref = RefAviary(num_drones=K, task="none", aero=tuple(a for a in aero if a != "bullet"),
                    integrator="bullet" if physics == "pyb" else "dyn", initial_xyzs=raw[:, 0:3])
    ref.set_raw_state(raw)
    rtraj = ref.integrate(rpm)[0]
    up = np.array([upright(x) for x in q])
    assert 0 < up.sum() < K
    # pos, quat, vel, ang_v: what the gate changes.  The rpy columns are left out: a stored
    # quaternion that ends the substep within an ulp of the gimbal edge may take the other
    # getEulerZYX branch on the two sides (pitch 1.5663 vs pi/2), which is not the gate
    cols = np.r_[0:7, 10:16]
    err = state_rel_err(_zero_rpy(traj, cols)[None], _zero_rpy(rtraj, cols)[None])[0]
    assert err.max() <= 1e-10, (err.max(), np.nonzero(err > 1e-10)[0][:10], up[err > 1e-10][:10])
    sim.close()
