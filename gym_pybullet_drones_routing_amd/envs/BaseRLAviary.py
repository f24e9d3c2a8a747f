"""Single-env Gymnasium view over the batched HIP simulator.

Mirrors the outward surface of the reference's ``BaseRLAviary`` / ``BaseAviary``
(``envs/BaseRLAviary.py``, ``envs/BaseAviary.py:220-383``): same constructor keywords,
``reset(seed, options) -> (obs, info)``, ``step(action) -> (obs, reward, terminated,
truncated, info)``, ``action_space`` / ``observation_space``, the 20-float
``_getDroneStateVector`` and the derived constants (``HOVER_RPM``, ``MAX_RPM``, ...).  One env is
one ``BatchedAviarySim`` with ``n_envs=1`` and no auto-reset; every step is one HIP launch
followed by a device->host copy of the observation.

Not on this path (raise): GUI, video recording, RGB observations.
"""
import numpy as np
import torch

from ..enums import ActionType, DroneModel, ObservationType, Physics
from ..sim import BatchedAviarySim
from .spaces import action_space, observation_space


class BaseRLAviary:
    """Common part of HoverAviary / MultiHoverAviary (task = 'hover' | 'multihover')."""

    TASK = "none"

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=1, neighbourhood_radius=np.inf,
                 initial_xyzs=None, initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=240,
                 gui=False, record=False, obs=ObservationType.KIN, act=ActionType.RPM,
                 precision="f64", device=None, episode_len_sec=8, urdf_path=None):
        if gui or record:
            raise NotImplementedError("GUI / recording need the PyBullet renderer (out of scope: headless batched sim)")
        if ObservationType(obs) != ObservationType.KIN:
            raise NotImplementedError("ObservationType.RGB needs onboard cameras (out of scope)")
        if pyb_freq % ctrl_freq != 0:
            raise ValueError('[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.')
        self.DRONE_MODEL = DroneModel(drone_model)
        self.NUM_DRONES = int(num_drones)
        self.NEIGHBOURHOOD_RADIUS = neighbourhood_radius
        self.PHYSICS = Physics(physics)
        self.OBS_TYPE = ObservationType(obs)
        self.ACT_TYPE = ActionType(act)
        self.PYB_FREQ, self.CTRL_FREQ = int(pyb_freq), int(ctrl_freq)
        self.PYB_STEPS_PER_CTRL = self.PYB_FREQ // self.CTRL_FREQ
        self.CTRL_TIMESTEP = 1.0 / self.CTRL_FREQ
        self.PYB_TIMESTEP = 1.0 / self.PYB_FREQ
        self.EPISODE_LEN_SEC = episode_len_sec
        self.ACTION_BUFFER_SIZE = int(self.CTRL_FREQ // 2)
        self.sim = BatchedAviarySim(n_envs=1, drones_per_env=self.NUM_DRONES, drone_model=self.DRONE_MODEL,
                                    urdf_path=urdf_path, pyb_freq=self.PYB_FREQ, ctrl_freq=self.CTRL_FREQ,
                                    act=self.ACT_TYPE, task=self.TASK, physics=self.PHYSICS,
                                    precision=precision, autoreset=False, episode_len_sec=episode_len_sec,
                                    initial_xyzs=initial_xyzs, initial_rpys=initial_rpys, device=device)
        k = self.sim.constants
        p = self.sim.params
        self.G = 9.8
        self.M, self.L, self.KF, self.KM = p.m, p.arm, p.kf, p.km
        self.J = np.diag([p.ixx, p.iyy, p.izz])
        self.J_INV = np.linalg.inv(self.J)
        self.THRUST2WEIGHT_RATIO = p.thrust2weight
        self.GRAVITY, self.HOVER_RPM, self.MAX_RPM = k.gravity, k.hover_rpm, k.max_rpm
        self.MAX_THRUST, self.MAX_XY_TORQUE, self.MAX_Z_TORQUE = k.max_thrust, k.max_xy_torque, k.max_z_torque
        self.GND_EFF_H_CLIP = k.gnd_eff_h_clip
        self.PROP_RADIUS, self.GND_EFF_COEFF = p.prop_radius, p.gnd_eff_coeff
        self.DRAG_COEFF = np.array([p.drag_coeff_xy, p.drag_coeff_xy, p.drag_coeff_z])
        self.DW_COEFF_1, self.DW_COEFF_2, self.DW_COEFF_3 = p.dw_coeff_1, p.dw_coeff_2, p.dw_coeff_3
        self.COLLISION_H, self.COLLISION_R, self.COLLISION_Z_OFFSET = p.collision_h, p.collision_r, p.collision_z_offset
        self.MAX_SPEED_KMH = p.max_speed_kmh
        if self.ACT_TYPE == ActionType.VEL:                                   # BaseRLAviary.py:94-95
            self.SPEED_LIMIT = 0.03 * self.MAX_SPEED_KMH * (1000 / 3600)
        if initial_xyzs is None:
            self.INIT_XYZS = np.array([[i * 4 * self.L, i * 4 * self.L, self.COLLISION_H / 2 - self.COLLISION_Z_OFFSET + .1]
                                       for i in range(self.NUM_DRONES)])
        else:
            self.INIT_XYZS = np.asarray(initial_xyzs, dtype=np.float64).reshape(self.NUM_DRONES, 3)
        self.INIT_RPYS = (np.zeros((self.NUM_DRONES, 3)) if initial_rpys is None
                          else np.asarray(initial_rpys, dtype=np.float64).reshape(self.NUM_DRONES, 3))
        self.action_space = action_space(self.NUM_DRONES, self.sim.act_width)
        self.observation_space = observation_space(self.NUM_DRONES, self.sim.act_width, self.ACTION_BUFFER_SIZE)
        self._act_dev = torch.zeros((1, self.NUM_DRONES, self.sim.act_width), dtype=torch.float32,
                                    device=self.sim.device)
        self.step_counter = 0

    # ------------------------------------------------------------------ Gymnasium surface
    def reset(self, seed=None, options=None):
        """BaseAviary.reset (:220-255).  The seed is ignored, as in the reference (:243)."""
        obs = self.sim.reset()
        self.step_counter = 0
        return obs[0].cpu().numpy(), self._computeInfo()

    def step(self, action):
        """BaseAviary.step (:259-383): one HIP launch for the PYB_STEPS_PER_CTRL substeps."""
        a = np.asarray(action, dtype=np.float32).reshape(self._act_dev.shape)
        self._act_dev.copy_(torch.from_numpy(a))
        obs, _, te, tr = self.sim.step(self._act_dev, terminal_obs=False)
        out = torch.cat([obs.reshape(-1), te.float(), tr.float()]).cpu().numpy()
        # the reward as the reference returns it: a Python float computed in fp64 from the state
        # vector (HoverAviary.py:78, MultiHoverAviary.py:84-89), not the batched path's float32 copy
        self._pos = self.sim.raw_state()[:, 0:3].cpu().numpy().astype(np.float64)
        W = self.NUM_DRONES * self.sim.obs_width
        self.step_counter += self.PYB_STEPS_PER_CTRL
        return (out[:W].reshape(self.NUM_DRONES, self.sim.obs_width), self._computeReward(), bool(out[W]),
                bool(out[W + 1]), self._computeInfo())

    def close(self):
        self.sim.close()

    def render(self, mode="human", close=False):
        s = self.sim.state20().cpu().numpy()
        for i in range(self.NUM_DRONES):
            print(f"[INFO] drone {i} pos {s[i, 0:3]} rpy {s[i, 7:10]} vel {s[i, 10:13]} ang_v {s[i, 13:16]}")

    # ------------------------------------------------------------------ reference helpers
    def _getDroneStateVector(self, nth_drone):
        """BaseAviary._getDroneStateVector (:541-561)."""
        return self.sim.state20()[nth_drone].cpu().numpy().astype(np.float64)

    def _computeInfo(self):
        return {"answer": 42}

    def _computeReward(self):
        raise NotImplementedError   # HoverAviary / MultiHoverAviary

    def _normalizedActionToRPM(self, action):
        """BaseAviary._normalizedActionToRPM (:893-911)."""
        action = np.asarray(action)
        return np.where(action <= 0, (action + 1) * self.HOVER_RPM,
                        self.HOVER_RPM + (self.MAX_RPM - self.HOVER_RPM) * action)

    def setPIDCoefficients(self, **coeffs):
        """BaseControl.setPIDCoefficients on every drone's DSLPIDControl (PID action types)."""
        self.sim.set_pid_coefficients(**coeffs)

    def getDroneIds(self):
        return np.arange(self.NUM_DRONES)

    def _getAdjacencyMatrix(self):
        """BaseAviary._getAdjacencyMatrix (:658-675) from the current positions."""
        pos = self.sim.state20()[:, 0:3].cpu().numpy()
        d = np.linalg.norm(pos[:, None, :] - pos[None, :, :], axis=-1)
        adj = (d < self.NEIGHBOURHOOD_RADIUS).astype(float)
        np.fill_diagonal(adj, 1.0)
        return adj
