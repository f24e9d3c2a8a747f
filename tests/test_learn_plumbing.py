"""examples/learn.py plumbing: the GPU-resident PPO drives the batched
VecEnv surface end to end.  The full run (reward threshold 474.15 / 949.5) is recorded in
profiles/learn_r1.json; here two short iterations check that rollout, TimeLimit bootstrapping,
GAE, the update and the deterministic evaluation episode all run on the device."""
import math
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("multi", [False, True])
def test_ppo_two_iterations(multi):
    import learn
    logs = []
    policy, hist, best, target = learn.train(multiagent=multi, n_envs=256, n_steps=16, total_timesteps=2 * 256 * 16,
                                             minibatch=1024, epochs=2, eval_every=1, log=logs.append)
    assert len(hist) == 2
    assert target == (949.5 if multi else 474.15)
    for h in hist:
        assert math.isfinite(h["mean_step_reward"]) and h["eval_len"] >= 1
    assert any("Observation space" in l for l in logs if isinstance(l, str))
