"""Reference-shaped CPU restatement of the DYN hot path (TEST INFRASTRUCTURE ONLY).

ORACLE - only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product path (``gym_pybullet_drones_routing_amd``)
never does.

What it restates (paths relative to the reference root, ``gym_pybullet_drones/``):
  * ``envs/BaseAviary.py:341-383``  step(): preprocess, substep loop with readback cadence,
    ``last_clipped_action`` update, final readback, obs/reward/done before step_counter += 8
  * ``envs/BaseAviary.py:451-505``  _housekeeping()/reset() state initialisation
  * ``envs/BaseAviary.py:509-519``  _updateAndStoreKinematicInformation() (readback)
  * ``envs/BaseAviary.py:541-561``  _getDroneStateVector() 20-float state
  * ``envs/BaseAviary.py:715-811``  ground effect / drag / downwash force terms
  * ``envs/BaseAviary.py:815-889``  _dynamics() + _integrateQ()
  * ``envs/BaseRLAviary.py:66-67,132-156,160-239,284-319`` action buffer, action->RPM, KIN obs
  * ``envs/HoverAviary.py:51-132``, ``envs/MultiHoverAviary.py:57-145`` reward / done
It keeps the reference's structure on purpose (one object per env, a Python loop over
drones, small numpy ops per drone) so that ``bench.py`` can time it as the stand-in for the
reference's own ``env.step()`` (which cannot run here: pybullet/gymnasium are absent and
importing the reference was denied).

PyBullet itself is replaced by ``_b_*`` arrays that play the role of the physics client's
stored base state, plus the helpers in ``bullet_math.py``.

Parity status: **parity unpinned** against the reference's own outputs - the reference holds
no golden vectors, fixtures or numeric tests for this path and could
not be executed here.  The oracle is pinned only by analytic known-answer tests
(``tests/test_oracle_kat.py``: hover equilibrium, free fall, pure yaw, roll sign, ground
effect and downwash magnitudes, truncation timing, obs layout) and by scipy cross-checks of
the rotation helpers.

Numeric conventions restated from the reference's pinned toolchain:
  * numpy ``^1.24`` (``pyproject.toml:18``) uses legacy value-based casting, so
    ``self.HOVER_RPM * (1 + 0.05*target)`` with a float32 action (SB3 clips to the float32
    Box) is evaluated entirely in float32: ``f32(HOVER) * (1f + 0.05f*a)``, then stored into
    the float64 ``rpm`` array (``BaseRLAviary.py:191-192, 224-225``).
  * Bullet3 is built in double precision; the DYN integrator runs in float64 numpy.

"New combination" (SURVEY.md §8(d) C3): the reference only applies ground effect / drag /
downwash under Bullet integration (PYB_* modes).  With ``aero`` set, this oracle adds the
same force terms to the explicit DYN integrator as a body wrench:
  total body-z force  T = sum(f_k) [+ sum(g_k)] [+ sum_j dw_j]
  body torque        += sum_k r_k x (0, 0, g_k)       (ground effect at the prop links)
  world force         F = R (0,0,T) [+ drag_factors * v] - (0,0,M*G)
and ``wrench='geom'`` swaps the DYN torque formula (with its roll-sign quirk, :847) for the
torque Bullet would produce from forces at the URDF prop positions (``_physics``, :679-711).

``integrator='bullet'`` (the ``Physics.PYB*`` modes): the same forces are
handed to the restated ``btMultiBody`` base step of ``bullet_mb.py`` instead of the explicit
integrator - forces at the prop links, default multibody damping, world-frame angular velocity,
Bullet's exponential-map orientation update; no contacts.
"""
import collections
import math

import numpy as np

from .bullet_math import euler_from_quat, quat_from_euler, quat_roundtrip, quat_to_mat
from .bullet_mb import drone_contact, multibody_finish, multibody_velocity
from .params import derived
from .ref_pid import RefDSLPID, pid_action_rpm

ACT_WIDTH = {"rpm": 4, "one_d_rpm": 1, "pid": 3, "vel": 4, "one_d_pid": 1}   # BaseRLAviary.py:141-147
PID_ACTS = ("pid", "vel", "one_d_pid")


def rpm_from_action(hover_rpm, a):
    """BaseRLAviary._preprocessAction (:191-192 RPM, :224-225 ONE_D_RPM) under numpy 1.x casting."""
    a32 = np.asarray(a, dtype=np.float32)
    h32 = np.float32(hover_rpm)
    with np.errstate(all="ignore"):
        r = h32 * (np.float32(1.0) + np.float32(0.05) * a32)
    return r.astype(np.float64)


class RefAviary:
    """One env (HoverAviary / MultiHoverAviary / raw) on the DYN path, reference-shaped."""

    def __init__(self, model="cf2x", num_drones=1, initial_xyzs=None, initial_rpys=None,
                 pyb_freq=240, ctrl_freq=30, act="rpm", task="hover", aero=(), wrench="dyn",
                 episode_len_sec=8, integrator="dyn", drones_per_env=None):
        if pyb_freq % ctrl_freq != 0:
            raise ValueError("[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.")
        p = derived(model)
        self.P = p
        self.MODEL = model
        self.NUM_DRONES = num_drones
        # drones that collide with each other under PYB* (consecutive groups): the whole
        # MultiHoverAviary; raw (task "none") instances default to a batch of one-drone envs
        self.DRONES_PER_ENV = drones_per_env or (num_drones if task == "multihover" else 1)
        self.PYB_FREQ, self.CTRL_FREQ = pyb_freq, ctrl_freq
        self.PYB_STEPS_PER_CTRL = int(pyb_freq / ctrl_freq)
        self.PYB_TIMESTEP = 1. / pyb_freq
        self.M, self.L, self.KF, self.KM = p["m"], p["arm"], p["kf"], p["km"]
        self.GRAVITY = p["gravity"]
        self.J = np.diag([p["ixx"], p["iyy"], p["izz"]])
        self.J_INV = np.linalg.inv(self.J)
        self.HOVER_RPM = np.float64(p["hover_rpm"])
        self.GND_EFF_COEFF, self.PROP_RADIUS = p["gnd_eff_coeff"], p["prop_radius"]
        self.GND_EFF_H_CLIP = p["gnd_eff_h_clip"]
        self.DRAG_COEFF = np.array([p["drag_coeff_xy"], p["drag_coeff_xy"], p["drag_coeff_z"]])
        self.DW_COEFF_1, self.DW_COEFF_2, self.DW_COEFF_3 = p["dw_coeff_1"], p["dw_coeff_2"], p["dw_coeff_3"]
        self.PROP_POS = np.array(p["prop_pos"])
        self.AERO = set(aero)
        if integrator not in ("dyn", "bullet"):
            raise ValueError("integrator must be 'dyn' or 'bullet'")
        self.INTEGRATOR = integrator
        self.WRENCH = "geom" if integrator == "bullet" else wrench   # Bullet: forces at the prop links
        self.ACT = act
        self.A = ACT_WIDTH[act]
        if act in PID_ACTS:                     # BaseRLAviary.py:73-78, 93-95
            if model not in ("cf2x", "cf2p"):
                raise NotImplementedError("no controller is available for the specified drone_model")
            self.ctrl = [RefDSLPID() for _ in range(num_drones)]
            self.CTRL_TIMESTEP = 1. / ctrl_freq
            self.SPEED_LIMIT = 0.03 * p["max_speed_kmh"] * (1000 / 3600)
        self.TASK = task
        self.EPISODE_LEN_SEC = episode_len_sec
        # BaseAviary.py:194-207
        if initial_xyzs is None:
            z0 = p["collision_h"] / 2 - p["collision_z_offset"] + .1
            self.INIT_XYZS = np.array([[i * 4 * self.L, i * 4 * self.L, z0] for i in range(num_drones)])
        else:
            self.INIT_XYZS = np.array(initial_xyzs, dtype=np.float64).reshape(num_drones, 3)
        self.INIT_RPYS = (np.zeros((num_drones, 3)) if initial_rpys is None
                          else np.array(initial_rpys, dtype=np.float64).reshape(num_drones, 3))
        # BaseRLAviary.py:66-67, 153-154: 15 zero actions, NOT cleared on reset
        self.ACTION_BUFFER_SIZE = int(ctrl_freq // 2)
        self.action_buffer = collections.deque(maxlen=self.ACTION_BUFFER_SIZE)
        for _ in range(self.ACTION_BUFFER_SIZE):
            self.action_buffer.append(np.zeros((num_drones, self.A)))
        if task == "hover":
            self.TARGET_POS = np.array([0, 0, 1])                                  # HoverAviary.py:51
        elif task == "multihover":
            self.TARGET_POS = self.INIT_XYZS + np.array([[0, 0, 1 / (i + 1)] for i in range(num_drones)])  # :71
        self._housekeeping()
        self._updateAndStoreKinematicInformation()

    # ------------------------------------------------------------------ state plumbing
    def _housekeeping(self):
        """BaseAviary._housekeeping (:451-505) minus GUI/URDF loading."""
        n = self.NUM_DRONES
        self.step_counter = 0
        self.last_clipped_action = np.zeros((n, 4))
        self.pos = np.zeros((n, 3))
        self.quat = np.zeros((n, 4))
        self.rpy = np.zeros((n, 3))
        self.vel = np.zeros((n, 3))
        self.ang_v = np.zeros((n, 3))
        self.rpy_rates = np.zeros((n, 3))
        # the physics client's stored base state after loadURDF(INIT_XYZS, quat(INIT_RPYS))
        self._b_pos = self.INIT_XYZS.astype(np.float64).copy()
        self._b_quat = np.array([quat_roundtrip(quat_from_euler(self.INIT_RPYS[i])) for i in range(n)])
        self._b_vel = np.zeros((n, 3))
        self._b_angv = np.zeros((n, 3))

    def _updateAndStoreKinematicInformation(self):
        """BaseAviary.py:509-519; orientation comes back through a btTransform."""
        for i in range(self.NUM_DRONES):
            self.pos[i], self.quat[i] = self._b_pos[i], quat_roundtrip(self._b_quat[i])
            self.rpy[i] = euler_from_quat(self.quat[i])
            self.vel[i], self.ang_v[i] = self._b_vel[i], self._b_angv[i]

    def _getDroneStateVector(self, i):
        """BaseAviary.py:541-561."""
        return np.hstack([self.pos[i, :], self.quat[i, :], self.rpy[i, :],
                          self.vel[i, :], self.ang_v[i, :], self.last_clipped_action[i, :]])

    def state20(self):
        return np.array([self._getDroneStateVector(i) for i in range(self.NUM_DRONES)])

    # ------------------------------------------------------------------ physics
    def _integrateQ(self, quat, omega, dt):
        """BaseAviary.py:876-889."""
        omega_norm = np.linalg.norm(omega)
        p, q, r = omega
        if np.isclose(omega_norm, 0):
            return quat
        lambda_ = np.array([[0, r, -q, p],
                            [-r, 0, p, q],
                            [q, -p, 0, r],
                            [-p, -q, -r, 0]]) * .5
        theta = omega_norm * dt / 2
        return np.dot(np.eye(4) * np.cos(theta) + 2 / omega_norm * lambda_ * np.sin(theta), quat)

    def _ground_effect_wrench(self, rpm, i, rotation):
        """BaseAviary._groundEffect (:715-750) as a body wrench (forces at the prop links)."""
        if not (np.abs(self.rpy[i, 0]) < np.pi / 2 and np.abs(self.rpy[i, 1]) < np.pi / 2):
            return 0.0, 0.0, 0.0
        prop_heights = np.array([self.pos[i, 2] + np.dot(rotation[2, :], self.PROP_POS[k]) for k in range(4)])
        prop_heights = np.clip(prop_heights, self.GND_EFF_H_CLIP, np.inf)
        g = np.array(rpm ** 2) * self.KF * self.GND_EFF_COEFF * (self.PROP_RADIUS / (4 * prop_heights)) ** 2
        fz = g[0] + g[1] + g[2] + g[3]
        tx = 0.0
        ty = 0.0
        for k in range(4):                      # r_k x (0, 0, g_k)
            tx = tx + self.PROP_POS[k, 1] * g[k]
            ty = ty - self.PROP_POS[k, 0] * g[k]
        return fz, tx, ty

    def _drag_force(self, rpm, i):
        """BaseAviary._drag (:754-781): world force = drag_factors * v (R R^T = I)."""
        drag_factors = -1 * self.DRAG_COEFF * np.sum(np.array(2 * np.pi * rpm / 60))
        return drag_factors * np.array(self.vel[i, :])

    def _downwash_force(self, i):
        """BaseAviary._downwash (:785-811): summed body -z force from drones above."""
        total = 0.0
        for j in range(self.NUM_DRONES):
            delta_z = self.pos[j, 2] - self.pos[i, 2]
            delta_xy = np.linalg.norm(np.array(self.pos[j, 0:2]) - np.array(self.pos[i, 0:2]))
            if delta_z > 0 and delta_xy < 10:
                alpha = self.DW_COEFF_1 * (self.PROP_RADIUS / (4 * delta_z)) ** 2
                beta = self.DW_COEFF_2 * delta_z + self.DW_COEFF_3
                with np.errstate(all="ignore"):
                    total = total + (-alpha * np.exp(-.5 * (delta_xy / beta) ** 2))
        return total

    def _bullet_physics(self, rpm, i):
        """PYB* modes: _physics (:679-711) [+ _groundEffect / _drag / _downwash, :715-811] as
        forces on the links, then one p.stepSimulation() (:369-370) restated by
        bullet_mb (the unconstrained half here; _bullet_step_all finishes it).  Body frame: prop forces (0,0,f_k) at r_k, ground effect
        (0,0,g_k) at r_k, downwash (0,0,dw) and drag R^T (drag_factors * vel) at the COM link."""
        forces = np.array(rpm ** 2) * self.KF
        torques = np.array(rpm ** 2) * self.KM
        if self.MODEL == "racer":
            torques = -torques
        z_torque = (-torques[0] + torques[1] - torques[2] + torques[3])
        fz = forces[0] + forces[1] + forces[2] + forces[3]
        tx = 0.0
        ty = 0.0
        for k in range(4):
            tx = tx + self.PROP_POS[k, 1] * forces[k]
            ty = ty - self.PROP_POS[k, 0] * forces[k]
        if "gnd" in self.AERO:
            gz, gx, gy = self._ground_effect_wrench(rpm, i, quat_to_mat(self.quat[i, :]))
            fz = fz + gz
            tx = tx + gx
            ty = ty + gy
        if "dw" in self.AERO:
            fz = fz + self._downwash_force(i)
        f_base = np.array([0.0, 0.0, fz])
        if "drag" in self.AERO:
            f_base = f_base + quat_to_mat(self.quat[i, :]).T @ self._drag_force(self.last_clipped_action[i, :], i)
        p = self.P
        return multibody_velocity(self._b_pos[i], self._b_quat[i], self._b_vel[i], self._b_angv[i],
                                  f_base, np.array([tx, ty, z_torque]),
                                  np.array([0.0, 0.0, -p["G"]]) * self.M, self.M,
                                  np.array([p["ixx"], p["iyy"], p["izz"]]), self.PYB_TIMESTEP)

    def _bullet_step_all(self, rpms):
        """One p.stepSimulation() of every drone (PYB* modes): the unconstrained velocity update
        of each drone (_bullet_physics), the drone <-> drone contact over the env (envs of D > 1
        drones, bullet_mb.drone_contact: the island solve, which also takes the plane rows of the
        drones in a pair contact that touch the plane), then each other drone's ground-plane contact
        and every drone's position update (bullet_mb.multibody_finish)."""
        p = self.P
        cyl = (p["collision_r"], p["collision_h"] / 2, p["collision_z_offset"])
        inertia = np.array([p["ixx"], p["iyy"], p["izz"]])
        mids = [self._bullet_physics(rpms[i, :], i) for i in range(self.NUM_DRONES)]
        G = self.DRONES_PER_ENV
        plane = "no_plane" not in self.AERO
        island = set()                   # drones whose plane rows the island solve took
        if G > 1 and "no_drone_contact" not in self.AERO:
            for e0 in range(0, self.NUM_DRONES, G):
                env = mids[e0:e0 + G]
                out = drone_contact(self._b_pos[e0:e0 + G], np.array([m[1].T for m in env]),
                                    np.array([m[2] for m in env]), np.array([m[3] for m in env]),
                                    self.M, inertia, self.PYB_TIMESTEP, *cyl, plane=plane)
                vel, omg = out[0], out[1]
                if plane:
                    island |= {e0 + i for i in out[2]}
                mids[e0:e0 + G] = [(m[0], m[1], vel[i], omg[i]) for i, m in enumerate(env)]
        for i, (q_wb, rot, vel, omega) in enumerate(mids):
            pos, q_s, vel, omega = multibody_finish(self._b_pos[i], q_wb, rot, vel, omega, self.M, inertia,
                                                    self.PYB_TIMESTEP, cyl if plane and i not in island else None)
            self._b_pos[i], self._b_quat[i], self._b_vel[i], self._b_angv[i] = pos, q_s, vel, omega
            self.rpy_rates[i, :] = omega

    def _substep_all(self, rpms):
        """One physics substep of every drone (BaseAviary.py:368-370)."""
        if self.INTEGRATOR == "bullet":
            return self._bullet_step_all(rpms)
        for i in range(self.NUM_DRONES):
            self._dynamics(rpms[i, :], i)

    def _dynamics(self, rpm, i):
        """BaseAviary._dynamics (:815-874) (+ optional aero wrench, see module doc)."""
        assert self.INTEGRATOR != "bullet", "PYB* substeps go through _bullet_step_all"
        pos = self.pos[i, :]
        quat = self.quat[i, :]
        vel = self.vel[i, :]
        rpy_rates = self.rpy_rates[i, :]
        rotation = quat_to_mat(quat)
        forces = np.array(rpm ** 2) * self.KF
        fz = np.sum(forces)
        z_torques = np.array(rpm ** 2) * self.KM
        if self.MODEL == "racer":
            z_torques = -z_torques
        z_torque = (-z_torques[0] + z_torques[1] - z_torques[2] + z_torques[3])
        if self.WRENCH == "geom":               # _physics (:693-711): forces at the prop links
            x_torque = 0.0
            y_torque = 0.0
            for k in range(4):
                x_torque = x_torque + self.PROP_POS[k, 1] * forces[k]
                y_torque = y_torque - self.PROP_POS[k, 0] * forces[k]
        elif self.MODEL in ("cf2x", "racer"):
            x_torque = (forces[0] + forces[1] - forces[2] - forces[3]) * (self.L / np.sqrt(2))
            y_torque = (- forces[0] + forces[1] + forces[2] - forces[3]) * (self.L / np.sqrt(2))
        else:
            x_torque = (forces[1] - forces[3]) * self.L
            y_torque = (-forces[0] + forces[2]) * self.L
        if "gnd" in self.AERO:
            gz, gx, gy = self._ground_effect_wrench(rpm, i, rotation)
            fz = fz + gz
            x_torque = x_torque + gx
            y_torque = y_torque + gy
        if "dw" in self.AERO:
            fz = fz + self._downwash_force(i)
        thrust = np.array([0, 0, fz])
        force_world_frame = np.dot(rotation, thrust)
        if "drag" in self.AERO:
            force_world_frame = force_world_frame + self._drag_force(self.last_clipped_action[i, :], i)
        force_world_frame = force_world_frame - np.array([0, 0, self.GRAVITY])
        torques = np.array([x_torque, y_torque, z_torque])
        torques = torques - np.cross(rpy_rates, np.dot(self.J, rpy_rates))
        rpy_rates_deriv = np.dot(self.J_INV, torques)
        no_pybullet_dyn_accs = force_world_frame / self.M
        vel = vel + self.PYB_TIMESTEP * no_pybullet_dyn_accs
        rpy_rates = rpy_rates + self.PYB_TIMESTEP * rpy_rates_deriv
        pos = pos + self.PYB_TIMESTEP * vel
        quat = self._integrateQ(quat, rpy_rates, self.PYB_TIMESTEP)
        # resetBasePositionAndOrientation / resetBaseVelocity (:862-872)
        self._b_pos[i] = pos
        self._b_quat[i] = quat
        self._b_vel[i] = vel
        self._b_angv[i] = np.dot(rotation, rpy_rates)
        self.rpy_rates[i, :] = rpy_rates

    # ------------------------------------------------------------------ RL surface
    def _preprocessAction(self, action):
        self.action_buffer.append(action)
        rpm = np.zeros((self.NUM_DRONES, 4))
        for k in range(action.shape[0]):
            target = action[k, :]
            if self.ACT == "rpm":
                rpm[k, :] = rpm_from_action(self.HOVER_RPM, target)
            elif self.ACT == "one_d_rpm":
                rpm[k, :] = np.repeat(rpm_from_action(self.HOVER_RPM, target), 4)
            else:
                rpm[k, :] = pid_action_rpm(self.ACT, self.ctrl[k], self._getDroneStateVector(k), target,
                                           self.CTRL_TIMESTEP, self.SPEED_LIMIT)
        return rpm

    def _computeObs(self):
        obs_12 = np.zeros((self.NUM_DRONES, 12))
        for i in range(self.NUM_DRONES):
            obs = self._getDroneStateVector(i)
            obs_12[i, :] = np.hstack([obs[0:3], obs[7:10], obs[10:13], obs[13:16]]).reshape(12,)
        ret = np.array([obs_12[i, :] for i in range(self.NUM_DRONES)]).astype('float32')
        for i in range(self.ACTION_BUFFER_SIZE):
            ret = np.hstack([ret, np.array([self.action_buffer[i][j, :] for j in range(self.NUM_DRONES)])])
        return ret.astype(np.float32)

    def _computeReward(self):
        if self.TASK == "hover":
            state = self._getDroneStateVector(0)
            return max(0, 2 - np.linalg.norm(self.TARGET_POS - state[0:3]) ** 4)
        if self.TASK == "multihover":
            ret = 0
            for i in range(self.NUM_DRONES):
                ret += max(0, 2 - np.linalg.norm(self.TARGET_POS[i, :] - self._getDroneStateVector(i)[0:3]) ** 4)
            return ret
        return -1

    def _computeTerminated(self):
        if self.TASK == "hover":
            return bool(np.linalg.norm(self.TARGET_POS - self._getDroneStateVector(0)[0:3]) < .0001)
        if self.TASK == "multihover":
            dist = 0
            for i in range(self.NUM_DRONES):
                dist += np.linalg.norm(self.TARGET_POS[i, :] - self._getDroneStateVector(i)[0:3])
            return bool(dist < .0001)
        return False

    def _computeTruncated(self):
        if self.TASK not in ("hover", "multihover"):
            return False
        lim = 1.5 if self.TASK == "hover" else 2.0
        for i in range(self.NUM_DRONES):
            s = self._getDroneStateVector(i)
            if (abs(s[0]) > lim or abs(s[1]) > lim or s[2] > 2.0
                    or abs(s[7]) > .4 or abs(s[8]) > .4):
                return True
        return bool(self.step_counter / self.PYB_FREQ > self.EPISODE_LEN_SEC)

    def reset(self):
        self._housekeeping()
        self._updateAndStoreKinematicInformation()
        return self._computeObs(), {"answer": 42}

    def step(self, action):
        action = np.asarray(action, dtype=np.float32).reshape(self.NUM_DRONES, self.A)
        clipped_action = np.reshape(self._preprocessAction(action), (self.NUM_DRONES, 4))
        # :346 - plain PYB skips the readback between substeps (its forces do not read it)
        plain_pyb = self.INTEGRATOR == "bullet" and not self.AERO
        for _ in range(self.PYB_STEPS_PER_CTRL):
            if self.PYB_STEPS_PER_CTRL > 1 and not plain_pyb:
                self._updateAndStoreKinematicInformation()
            self._substep_all(clipped_action)
            self.last_clipped_action = clipped_action
        self._updateAndStoreKinematicInformation()
        obs = self._computeObs()
        reward = self._computeReward()
        terminated = self._computeTerminated()
        truncated = self._computeTruncated()
        self.step_counter = self.step_counter + (1 * self.PYB_STEPS_PER_CTRL)
        return obs, reward, terminated, truncated, {"answer": 42}

    # ------------------------------------------------------------------ raw integrator
    def integrate(self, rpms, record=True):
        """Raw DYN path (gpd_integrate): one substep per row of ``rpms`` [T, N, 4] float64,
        each followed by a readback (= PYB_STEPS_PER_CTRL 1 cadence).  Returns the
        state20 after every substep, [T, N, 20]."""
        rpms = np.asarray(rpms, dtype=np.float64)
        out = []
        for t in range(rpms.shape[0]):
            self._substep_all(rpms[t])
            self.last_clipped_action = rpms[t].copy()
            self._updateAndStoreKinematicInformation()
            if record:
                out.append(self.state20())
        return np.array(out) if record else None

    # ------------------------------------------------------------------ test seeding
    def ctrl_state(self):
        """[N, 9] controller state (integral_pos_e, integral_rpy_e, last_rpy) per drone."""
        return np.array([c.get_state() for c in self.ctrl])

    def set_ctrl_state(self, v):
        v = np.asarray(v, dtype=np.float64).reshape(self.NUM_DRONES, 9)
        for c, row in zip(self.ctrl, v):
            c.set_state(row)

    def set_raw_state(self, raw):
        """Seed the physics-client state from a raw [N, 20] array laid out as gpd_get_raw_state:
        pos(3) quat_as_stored(4) vel(3) rpy_rates(3) ang_v(3) last_clipped_action(4).  With the
        Bullet integrator rpy_rates(3) is the world angular velocity the step integrates."""
        raw = np.asarray(raw, dtype=np.float64).reshape(self.NUM_DRONES, 20)
        self._b_pos = raw[:, 0:3].copy()
        self._b_quat = raw[:, 3:7].copy()
        self._b_vel = raw[:, 7:10].copy()
        self.rpy_rates = raw[:, 10:13].copy()
        # Bullet: slots 10..12 hold the integrated world angular velocity (m_realBuf[0:3])
        self._b_angv = raw[:, 10:13].copy() if self.INTEGRATOR == "bullet" else raw[:, 13:16].copy()
        self.last_clipped_action = raw[:, 16:20].copy()
        self._updateAndStoreKinematicInformation()
