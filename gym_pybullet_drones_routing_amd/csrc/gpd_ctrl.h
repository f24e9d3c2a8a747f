// gpd_ctrl.h — batched DSLPIDControl for the PID / VEL / ONE_D_PID action types (gfx950).
//
// One lane runs its drone's controller once per control step, before the substeps, on the
// state of the last readback (BaseRLAviary._preprocessAction, envs/BaseRLAviary.py:193-235).
// The per-drone controller state (integral_pos_e, integral_rpy_e, last_rpy; 9 reals) lives in
// an SoA buffer beside the physics state and, like the reference's DSLPIDControl objects
// (created once in BaseRLAviary.__init__, :73-76, never reset by env.reset()), survives resets.
//
// Restated from control/DSLPIDControl.py (paths relative to gym_pybullet_drones/):
//   _dslPIDPositionControl  :187-208      _dslPIDAttitudeControl  :240-259
// One deliberate, rounding-level simplification: the reference turns the target rotation
// matrix into intrinsic 'XYZ' Euler angles with scipy (:205) and back into a matrix (:242-244)
// before using it.  That round trip is the identity on rotation matrices (also at gimbal lock,
// where scipy zeroes the third angle and folds it into the first), and the angles themselves
// are only returned to the caller as a yaw error that BaseRLAviary discards, so the matrix is
// used directly; tests/test_oracle_pid.py bounds the difference against scipy's round trip.
#pragma once
#include "gpd_device.h"

namespace gpd {

enum : int { ACT_RPM = 0, ACT_ONE_D_RPM = 1, ACT_PID = 2, ACT_VEL = 3, ACT_ONE_D_PID = 4 };

// action width (BaseRLAviary._actionSpace, envs/BaseRLAviary.py:141-147)
__host__ __device__ constexpr int act_width(int act) {
  return (act == ACT_RPM || act == ACT_VEL) ? 4 : (act == ACT_PID ? 3 : 1);
}
__host__ __device__ constexpr bool act_is_pid(int act) { return act >= ACT_PID; }

// np.clip(x, lo, hi) = minimum(maximum(x, lo), hi); NaN passes through as in numpy.
template <typename R>
__device__ __forceinline__ R np_clip(R x, R lo, R hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

// DSLPIDControl.computeControl for one drone.  cs = {integral_pos_e[3], integral_rpy_e[3],
// last_rpy[3]} (updated in place), Rm = getMatrixFromQuaternion(cur_quat) row-major,
// rpy = getEulerFromQuaternion(cur_quat).  Evaluated with FP contraction off, like numpy.
// YAW0: the target yaw is the default 0 (PID, ONE_D_PID), so target_x_c = (1, 0, 0) exactly.
template <typename R, bool YAW0 = false>
__device__ __forceinline__ void dsl_pid(const PidConsts<R>& k, const R pos[3], const R Rm[9], const R rpy[3],
                                        const R vel[3], const R tpos[3], R tyaw, const R tvel[3], R cs[9],
                                        R rpm[4]) {
#pragma clang fp contract(off)
  const R dt = k.ctrl_dt;
  // ---- position control (:187-208)
  R tt[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const R pe = tpos[i] - pos[i];
    const R ve = tvel[i] - vel[i];
    R ip = np_clip(cs[i] + pe * dt, R(-2), R(2));
    if (i == 2) ip = np_clip(ip, R(-0.15), R(0.15));
    cs[i] = ip;
    tt[i] = ((k.p_for[i] * pe + k.i_for[i] * ip) + k.d_for[i] * ve) + (i == 2 ? k.gravity : R(0));
  }
  const R dot = (tt[0] * Rm[2] + tt[1] * Rm[5]) + tt[2] * Rm[8];   // target_thrust . R[:,2]
  const R scalar_thrust = dot > R(0) ? dot : R(0);                  // max(0., ...)
  const R thrust = (g_sqrt(scalar_thrust / (R(4) * k.kf)) - k.pwm2rpm_const) / k.pwm2rpm_scale;
  const R ntt = g_sqrt((tt[0] * tt[0] + tt[1] * tt[1]) + tt[2] * tt[2]);
  const R z0 = tt[0] / ntt, z1 = tt[1] / ntt, z2 = tt[2] / ntt;   // target_z_ax
  const R xc0 = YAW0 ? R(1) : g_cos(tyaw), xc1 = YAW0 ? R(0) : g_sin(tyaw);   // target_x_c (z = 0)
  const R c0 = z1 * R(0) - z2 * xc1, c1 = z2 * xc0 - z0 * R(0), c2 = z0 * xc1 - z1 * xc0;
  const R nc = g_sqrt((c0 * c0 + c1 * c1) + c2 * c2);
  const R y0 = c0 / nc, y1 = c1 / nc, y2 = c2 / nc;               // target_y_ax
  const R x0 = y1 * z2 - y2 * z1, x1 = y2 * z0 - y0 * z2, x2 = y0 * z1 - y1 * z0;  // target_x_ax
  // ---- attitude control (:240-259); target_rotation has columns (x, y, z)
  // rot_matrix_e = Rt^T R - R^T Rt; rot_e = (e[2,1], e[0,2], e[1,0])
  const R e0 = ((z0 * Rm[1] + z1 * Rm[4]) + z2 * Rm[7]) - ((Rm[2] * y0 + Rm[5] * y1) + Rm[8] * y2);
  const R e1 = ((x0 * Rm[2] + x1 * Rm[5]) + x2 * Rm[8]) - ((Rm[0] * z0 + Rm[3] * z1) + Rm[6] * z2);
  const R e2 = ((y0 * Rm[0] + y1 * Rm[3]) + y2 * Rm[6]) - ((Rm[1] * x0 + Rm[4] * x1) + Rm[7] * x2);
  const R rot_e[3] = {e0, e1, e2};
  R tq[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const R rre = R(0) - (rpy[i] - cs[6 + i]) / dt;               // target_rpy_rates = 0
    R ir = np_clip(cs[3 + i] - rot_e[i] * dt, R(-1500), R(1500));
    if (i < 2) ir = np_clip(ir, R(-1), R(1));
    cs[3 + i] = ir;
    const R t = ((-(k.p_tor[i] * rot_e[i])) + k.d_tor[i] * rre) + k.i_tor[i] * ir;
    tq[i] = np_clip(t, R(-3200), R(3200));
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) cs[6 + i] = rpy[i];                  // self.last_rpy = cur_rpy
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const R mix = (k.mixer[j * 3 + 0] * tq[0] + k.mixer[j * 3 + 1] * tq[1]) + k.mixer[j * 3 + 2] * tq[2];
    const R pwm = np_clip(thrust + mix, k.min_pwm, k.max_pwm);
    rpm[j] = k.pwm2rpm_scale * pwm + k.pwm2rpm_const;
  }
}

// float32 Euclidean norm of a 3-vector, fixed order, no FMA (ref: oracle/ref_pid.py norm3_f32)
__device__ __forceinline__ float norm3_f32(float a, float b, float c) {
#pragma clang fp contract(off)
  const float s = (a * a + b * b) + c * c;
  return sqrtf(s);
}

// The controller targets of the three action types for one drone (BaseRLAviary.py:193-235)
// from its float32 action row `act` and its last-readback state.
template <typename R, int ACT>
__device__ __forceinline__ void pid_targets(const PidConsts<R>& k, const float* act, const R pos[3], const R rpy[3],
                                            R tpos[3], R& tyaw, R tvel[3]) {
#pragma clang fp contract(off)
  tyaw = R(0);
  tvel[0] = tvel[1] = tvel[2] = R(0);
  if (ACT == ACT_PID) {
    // _calculateNextStep(current_position, destination=action, step_size=1) (BaseAviary.py:1129-1147)
    const R d0 = (R)act[0] - pos[0], d1 = (R)act[1] - pos[1], d2 = (R)act[2] - pos[2];
    const R dist = g_sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    if (dist <= R(1)) {
      tpos[0] = (R)act[0]; tpos[1] = (R)act[1]; tpos[2] = (R)act[2];
    } else {
      tpos[0] = pos[0] + (d0 / dist) * R(1);
      tpos[1] = pos[1] + (d1 / dist) * R(1);
      tpos[2] = pos[2] + (d2 / dist) * R(1);
    }
  } else if (ACT == ACT_VEL) {
    // target_pos = current position, target_rpy = (0, 0, yaw), target_vel =
    // SPEED_LIMIT*|a3| * a[0:3]/|a[0:3]| with numpy 1.x float32 casting (BaseRLAviary.py:210-221)
    tpos[0] = pos[0]; tpos[1] = pos[1]; tpos[2] = pos[2];
    tyaw = rpy[2];
    const float n = norm3_f32(act[0], act[1], act[2]);
    if (n != 0.0f) {
      const float s = (float)((double)k.speed_limit * (double)fabsf(act[3]));
      tvel[0] = (R)(s * (act[0] / n));
      tvel[1] = (R)(s * (act[1] / n));
      tvel[2] = (R)(s * (act[2] / n));
    }
  } else {  // ACT_ONE_D_PID: state[0:3] + 0.1*np.array([0, 0, target[0]])  (float64)
    tpos[0] = pos[0] + R(0);
    tpos[1] = pos[1] + R(0);
    tpos[2] = pos[2] + (R)(0.1 * (double)act[0]);
  }
}

}  // namespace gpd
