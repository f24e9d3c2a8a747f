"""HoverAviary on the HIP path (reference: ``envs/HoverAviary.py``).

Single drone, target (0, 0, 1), reward max(0, 2 - |e|^4), truncation outside |x|,|y| <= 1.5,
z <= 2, |roll|,|pitch| <= 0.4 or after 8 s (HoverAviary.py:51-117) - all evaluated inside the
step kernel.
"""
import numpy as np

from ..enums import ActionType, DroneModel, ObservationType, Physics
from .BaseRLAviary import BaseRLAviary


class HoverAviary(BaseRLAviary):
    """Single agent RL problem: hover at position."""

    TASK = "hover"

    def __init__(self, drone_model=DroneModel.CF2X, initial_xyzs=None, initial_rpys=None, physics=Physics.PYB,
                 pyb_freq=240, ctrl_freq=30, gui=False, record=False, obs=ObservationType.KIN,
                 act=ActionType.RPM, **kwargs):
        self.TARGET_POS = np.array([0, 0, 1])
        self.EPISODE_LEN_SEC = 8
        super().__init__(drone_model=drone_model, num_drones=1, initial_xyzs=initial_xyzs,
                         initial_rpys=initial_rpys, physics=physics, pyb_freq=pyb_freq, ctrl_freq=ctrl_freq,
                         gui=gui, record=record, obs=obs, act=act, episode_len_sec=self.EPISODE_LEN_SEC, **kwargs)

    def _computeReward(self):
        """HoverAviary._computeReward (:68-79): fp64 from the position after the step."""
        return max(0, 2 - np.linalg.norm(self.TARGET_POS - self._pos[0]) ** 4)
