#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the numpy oracle (oracle/ref_aviary.py).

The reference ships no golden vectors for the DYN path and cannot be executed here (SURVEY
§8(c)); these fixtures are outputs of the oracle, which is itself pinned by the analytic KATs
(tests/test_oracle_kat.py).  They freeze the oracle's behaviour (regression) and give the GPU
tests a fixed input/expected-output set that needs no oracle run.

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.bullet_math import quat_from_euler, quat_roundtrip  # noqa: E402
from oracle.params import derived  # noqa: E402
from oracle.ref_aviary import ACT_WIDTH, RefAviary, rpm_from_action  # noqa: E402
from tests.oracle_runs import run_vec  # noqa: E402

HOVER = derived("cf2x")["hover_rpm"]


def raw_states(rng, n, z=1.0, tilt=0.3, spin=2.0):
    raw = np.zeros((n, 20))
    raw[:, 0:2] = rng.uniform(-0.5, 0.5, (n, 2))
    raw[:, 2] = z
    for i in range(n):
        raw[i, 3:7] = quat_roundtrip(quat_from_euler(rng.uniform(-tilt, tilt, 3)))
    raw[:, 7:10] = rng.uniform(-0.5, 0.5, (n, 3))
    raw[:, 10:13] = rng.uniform(-spin, spin, (n, 3))
    raw[:, 16:20] = HOVER
    return raw


def integrate_fixture(name, n, T, every, aero=(), z=1.0, scale=1.0, seed=0, drones_per_env=1, xyz=None,
                      integrator="dyn"):
    rng = np.random.default_rng(seed)
    actions = (rng.uniform(-1, 1, (T, n, 4)) * scale).astype(np.float32)
    rpm = rpm_from_action(HOVER, actions)
    if drones_per_env == 1:
        raw0 = raw_states(rng, n, z=z)
        env = RefAviary(num_drones=n, task="none", aero=aero, integrator=integrator)
        env.set_raw_state(raw0)
        traj = env.integrate(rpm)
    else:
        raw0 = np.zeros((0, 20))
        traj = np.concatenate([RefAviary(num_drones=drones_per_env, task="none", aero=aero, initial_xyzs=xyz,
                                         integrator=integrator)
                               .integrate(rpm[:, e * drones_per_env:(e + 1) * drones_per_env])
                               for e in range(n // drones_per_env)], axis=1)
    np.savez_compressed(os.path.join(HERE, name), actions=actions, raw0=raw0, every=every,
                        aero=np.array(list(aero), dtype="U8"), drones_per_env=drones_per_env,
                        init_xyzs=np.zeros((0, 3)) if xyz is None else xyz, integrator=integrator,
                        traj=traj[every - 1::every])


def step_fixture(name, n_envs, T, act, task, D=1, seed=0, integrator="dyn", scale=1.0):
    rng = np.random.default_rng(seed)
    A = ACT_WIDTH[act]
    actions = (rng.uniform(-1, 1, (T, n_envs, D, A)) * scale).astype(np.float32)
    envs = []
    obs, rew, te, tr, tobs = run_vec(actions, n_envs, drones_per_env=D, act=act, task=task, integrator=integrator,
                                     envs=envs)
    extra = {}
    if hasattr(envs[0], "ctrl"):
        extra["ctrl_state"] = np.concatenate([e.ctrl_state() for e in envs])
        extra["state20"] = np.concatenate([e.state20() for e in envs])
    keys = sorted(tobs)
    W = obs.shape[-1]
    np.savez_compressed(os.path.join(HERE, name), actions=actions, obs=obs, reward=rew, terminated=te,
                        truncated=tr, terminal_keys=np.array(keys, dtype=np.int64).reshape(-1, 2),
                        terminal_obs=np.array([tobs[k] for k in keys], dtype=np.float32).reshape(len(keys), D, W),
                        integrator=integrator, **extra)


def main():
    # C1 (BASELINE configs[0]): 1 HoverAviary, DYN, 240/30 Hz, U[-1,1] actions from default_rng(0), 150 steps
    step_fixture("c1_hover_rpm.npz", 1, 150, "rpm", "hover")
    step_fixture("c1_hover_one_d_rpm.npz", 1, 150, "one_d_rpm", "hover")
    step_fixture("hover_rpm_8env.npz", 8, 60, "rpm", "hover", seed=3)
    step_fixture("multihover_2x2.npz", 2, 60, "rpm", "multihover", D=2, seed=4)
    # DSLPIDControl action types; the VEL loop is chaotic, so its horizon is short
    step_fixture("pid_waypoint_pyb.npz", 4, 60, "pid", "hover", seed=8, integrator="bullet", scale=0.5)
    step_fixture("one_d_pid_dyn.npz", 4, 60, "one_d_pid", "hover", seed=9)
    step_fixture("vel_pyb.npz", 4, 16, "vel", "hover", seed=10, integrator="bullet")
    # Physics.PYB (HoverAviary's default): restated Bullet multibody step, RPM actions
    step_fixture("c1_hover_rpm_pyb.npz", 1, 150, "rpm", "hover", seed=12, integrator="bullet")
    # raw DYN integrator, 5 s (1200 substeps), every 10th substep kept
    integrate_fixture("integrate_dyn_5s.npz", n=8, T=1200, every=10, seed=5)
    integrate_fixture("integrate_gnd_drag.npz", n=8, T=600, every=10, aero=("gnd", "drag"), z=0.06, scale=0.5, seed=6)
    i = np.arange(8)
    xyz = np.stack([0.15 * np.cos(2 * np.pi * i / 8), 0.15 * np.sin(2 * np.pi * i / 8), 0.5 + 0.1 * i], 1)
    integrate_fixture("integrate_pyb_gnd_drag.npz", n=8, T=600, every=10, aero=("gnd", "drag"), z=0.06, scale=0.5,
                      seed=13, integrator="bullet")
    integrate_fixture("integrate_downwash_8.npz", n=8, T=600, every=10, aero=("dw",), scale=0.3, seed=7,
                      drones_per_env=8, xyz=xyz)


if __name__ == "__main__":
    main()
