"""Logger-compatible recorder against the restated reference bookkeeping
(oracle/ref_logger.py, Logger.py:19-135)."""
import os

import numpy as np
import pytest
import torch

from oracle.ref_logger import RefLogger


def _states(rng, T, D):
    s = rng.normal(0, 1, (T, D, 20))
    s[..., 16:20] = rng.uniform(10000, 20000, (T, D, 4))
    return s


@pytest.mark.parametrize("duration_sec", [0, 2])
def test_log_matches_reference_bookkeeping(tmp_path, duration_sec):
    from gym_pybullet_drones_routing_amd.logger import Logger
    rng = np.random.default_rng(0)
    T, D, F = 75, 3, 30          # 75 > 2 s * 30 Hz: the preallocated arrays must grow too
    S = _states(rng, T, D)
    C = rng.normal(0, 1, (T, D, 12))
    ref = RefLogger(F, num_drones=D, duration_sec=duration_sec)
    lg = Logger(F, output_folder=str(tmp_path / "res"), num_drones=D, duration_sec=duration_sec)
    for t in range(T):
        for d in range(D):
            ref.log(d, t / F, S[t, d], C[t, d])
        if t % 2:
            lg.log_batch(t / F, S[t], C[t])
        else:
            for d in range(D):
                lg.log(d, t / F, S[t, d], C[t, d])
    for k, v in ref.arrays().items():
        np.testing.assert_array_equal(getattr(lg, k), v, err_msg=k)
    path = lg.save()
    with np.load(path, allow_pickle=False) as z:
        for k, v in ref.arrays().items():
            np.testing.assert_array_equal(z[k], v)
    csv_dir = lg.save_as_csv("t")
    x0 = np.loadtxt(os.path.join(csv_dir, "x0.csv"), delimiter=",")
    np.testing.assert_allclose(x0[:, 1], ref.states[0, 0, :])
    assert len(os.listdir(csv_dir)) == D * 23


def test_unequal_counters_fall_back_to_reference_rule(tmp_path):
    from gym_pybullet_drones_routing_amd.logger import Logger
    rng = np.random.default_rng(1)
    S = _states(rng, 6, 2)
    ref = RefLogger(10, num_drones=2)
    lg = Logger(10, output_folder=str(tmp_path), num_drones=2)
    ref.log(0, 0.0, S[0, 0]); lg.log(0, 0.0, S[0, 0])
    for t in range(1, 6):
        for d in range(2):
            ref.log(d, t / 10, S[t, d])
        lg.log_batch(t / 10, S[t])
    for k, v in ref.arrays().items():
        np.testing.assert_array_equal(getattr(lg, k), v, err_msg=k)


@pytest.mark.gpu
def test_logger_records_gpu_flight(tmp_path):
    """A 2-drone GPU flight logged from device memory equals the oracle's flight logged by the
    reference bookkeeping (states to the f64 parity tolerance)."""
    from gym_pybullet_drones_routing_amd.logger import Logger
    from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
    from oracle.ref_aviary import RefAviary
    rng = np.random.default_rng(2)
    T, D = 40, 2
    acts = np.clip(rng.normal(0, 0.2, (T, 1, D, 4)), -1, 1).astype(np.float32)
    sim = BatchedAviarySim(n_envs=1, drones_per_env=D, task="none", precision="f64", device="cuda:0")
    env = RefAviary(num_drones=D, task="none")
    lg = Logger(30, output_folder=str(tmp_path), num_drones=D, duration_sec=1, device="cuda:0")
    ref = RefLogger(30, num_drones=D, duration_sec=1)
    for t in range(T):
        sim.step(torch.from_numpy(acts[t]).cuda())
        env.step(acts[t, 0])
        lg.log_batch(t / 30, sim.state20())
        s = env.state20()
        for d in range(D):
            ref.log(d, t / 30, s[d])
    np.testing.assert_array_equal(lg.timestamps, ref.timestamps)
    np.testing.assert_allclose(lg.states, ref.states, rtol=1e-10, atol=1e-10)
    sim.close()
