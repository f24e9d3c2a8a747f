"""MultiHoverAviary on the HIP path (reference: ``envs/MultiHoverAviary.py``).

N drones, per-drone targets INIT_XYZS + (0, 0, 1/(i+1)), summed reward, termination when the
summed distance < 1e-4, truncation when any drone leaves |x|,|y| <= 2, z <= 2,
|roll|,|pitch| <= 0.4 or after 8 s (MultiHoverAviary.py:57-130) - reduced across the env's
drones inside the step kernel.
"""
import numpy as np

from ..enums import ActionType, DroneModel, ObservationType, Physics
from .BaseRLAviary import BaseRLAviary


class MultiHoverAviary(BaseRLAviary):
    """Multi-agent RL problem: leader-follower."""

    TASK = "multihover"

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=2, neighbourhood_radius=np.inf, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=30, gui=False, record=False,
                 obs=ObservationType.KIN, act=ActionType.RPM, **kwargs):
        self.EPISODE_LEN_SEC = 8
        super().__init__(drone_model=drone_model, num_drones=num_drones, neighbourhood_radius=neighbourhood_radius,
                         initial_xyzs=initial_xyzs, initial_rpys=initial_rpys, physics=physics, pyb_freq=pyb_freq,
                         ctrl_freq=ctrl_freq, gui=gui, record=record, obs=obs, act=act,
                         episode_len_sec=self.EPISODE_LEN_SEC, **kwargs)
        self.TARGET_POS = self.INIT_XYZS + np.array([[0, 0, 1 / (i + 1)] for i in range(num_drones)])

    def _computeReward(self):
        """MultiHoverAviary._computeReward (:75-89): the per-drone rewards summed in fp64."""
        ret = 0
        for i in range(self.NUM_DRONES):
            ret += max(0, 2 - np.linalg.norm(self.TARGET_POS[i, :] - self._pos[i]) ** 4)
        return ret
