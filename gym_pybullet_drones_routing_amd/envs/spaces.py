"""Observation/action spaces with the reference's bounds (BaseRLAviary.py:132-156, :243-280).

Uses ``gymnasium.spaces.Box`` when gymnasium is importable; otherwise a minimal Box with the
same attributes (low, high, shape, dtype, sample, contains) so the envs still work.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium import spaces as _gym_spaces
    Box = _gym_spaces.Box
except Exception:  # gymnasium is not installed in this image
    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            low = np.asarray(low, dtype=np.float64)
            high = np.asarray(high, dtype=np.float64)
            if shape is not None:
                low = np.broadcast_to(low, shape)
                high = np.broadcast_to(high, shape)
            self.low = low.astype(self.dtype)
            self.high = high.astype(self.dtype)
            self.shape = self.low.shape
            self._rng = np.random.default_rng()

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def action_space(num_drones, act_width):
    """BaseRLAviary._actionSpace: Box(-1, 1, (NUM_DRONES, size), float32)."""
    return Box(low=-np.ones((num_drones, act_width)), high=np.ones((num_drones, act_width)), dtype=np.float32)


def observation_space(num_drones, act_width, buffer_size):
    """BaseRLAviary._observationSpace (KIN): 12 kinematic entries (z >= 0) + the action buffer."""
    lo = np.full((num_drones, 12), -np.inf)
    lo[:, 2] = 0.0
    hi = np.full((num_drones, 12), np.inf)
    lo = np.hstack([lo, -np.ones((num_drones, buffer_size * act_width))])
    hi = np.hstack([hi, np.ones((num_drones, buffer_size * act_width))])
    return Box(low=lo, high=hi, dtype=np.float32)
