"""Debug probe: Bullet step kernel vs oracle for 8-drone stacks under several physics / aero sets
(resynced control steps), per-drone error of the first step."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_pybullet_drones_routing_amd.enums import ActionType, Physics  # noqa: E402
from oracle.ref_aviary import RefAviary  # noqa: E402
from tests.oracle_runs import oracle_raw, state_rel_err  # noqa: E402
from tests.test_gpu_drone_contact import _cube  # noqa: E402
from tests.test_gpu_parity import _sim  # noqa: E402

D = 8
cases = [("PYB", Physics.PYB, (), ()), ("PYB_GND_DRAG_DW", Physics.PYB_GND_DRAG_DW, ("gnd", "drag", "dw"), ()),
         ("PYB_GND_DRAG_DW nodc", Physics.PYB_GND_DRAG_DW, ("gnd", "drag", "dw", "no_drone_contact"), ("no_drone_contact",)),
         ("PYB_DW", Physics.PYB_DW, ("dw",), ()), ("PYB_GND", Physics.PYB_GND, ("gnd",), ()),
         ("PYB_DRAG", Physics.PYB_DRAG, ("drag",), ())]
for spread in (0.0, 1.0):
    for name, phys, oaero, saero in cases:
        raw0 = np.concatenate([_cube(np.random.default_rng(3)) for _ in range(2)])
        raw0[8:, 0] += 1.0
        if spread:
            raw0[:, 0:3] += np.repeat(np.arange(16)[:, None] * [0.3, 0, 0], 1, 0)   # far apart: no contact
        n = raw0.shape[0]
        env = RefAviary(num_drones=n, task="none", integrator="bullet", act="rpm", drones_per_env=D, aero=oaero)
        env.set_raw_state(raw0)
        sim = _sim(n_envs=n // D, drones_per_env=D, task="none", precision="f64", physics=phys, act=ActionType.RPM,
                   aero=saero)
        sim.reset()
        rng = np.random.default_rng(5)
        errs = []
        for t in range(4):
            a = rng.uniform(-0.2, 0.2, (n, 4)).astype(np.float32)
            sim.set_raw_state(oracle_raw(env))
            sim.step(torch.from_numpy(a.reshape(n // D, D, 4)).cuda())
            env.step(a)
            g = sim.raw_state().cpu().numpy()[:, :16]
            o = oracle_raw(env)[:, :16]
            errs.append(state_rel_err(g[None], o[None])[0])
            if t == 0:
                per = np.abs(g - o).max(axis=1)
                print(f"{name:22s} spread={spread}: step0 per-drone max abs err {np.array2string(per, precision=1)}", flush=True)
        print(f"{name:22s} spread={spread}: errs {np.array2string(np.array(errs), precision=2)}", flush=True)
        sim.close()
