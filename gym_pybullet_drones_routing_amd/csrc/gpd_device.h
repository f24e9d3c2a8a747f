// gpd_device.h — per-drone DYN physics for gfx950, templated on the real type.
//
// One lane owns one drone for the whole launch: the raw state lives in VGPRs across all
// PYB_STEPS_PER_CTRL substeps, the model constants are read through a uniform device pointer
// (scalar loads into SGPRs, re-loaded rather than spilled), and only the per-env neighbour
// positions (downwash), the reward reduction and the observation tile go through LDS.
//
// Every function cites the reference code it restates (paths relative to
// gym_pybullet_drones/ in the reference) or the Bullet3 routine pybullet runs for it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace gpd {

// ---------------------------------------------------------------- precision-overloaded math
// A wave-uniform branch that practically never runs: laid out after the hot path, so its code
// is not fetched into the instruction cache on the launches that skip it.
#if defined(GPD_NOCOLD)
#define GPD_RARE(x) ((x) && false)   // diagnostic build: every rare branch compiled out (bounds the
                                     // instruction-cache gain of moving them out of line)
#elif defined(GPD_NOEXPECT)
#define GPD_RARE(x) (x)
#else
#define GPD_RARE(x) __builtin_expect((x), 0)
#endif
__device__ __forceinline__ float g_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ double g_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float g_sin(float x) { return sinf(x); }
__device__ __forceinline__ double g_sin(double x) { return sin(x); }
__device__ __forceinline__ float g_cos(float x) { return cosf(x); }
__device__ __forceinline__ double g_cos(double x) { return cos(x); }
__device__ __forceinline__ float g_atan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double g_atan2(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float g_asin(float x) { return asinf(x); }
__device__ __forceinline__ double g_asin(double x) { return asin(x); }
__device__ __forceinline__ float g_exp(float x) { return expf(x); }
__device__ __forceinline__ double g_exp(double x) { return exp(x); }
__device__ __forceinline__ float g_abs(float x) { return fabsf(x); }
__device__ __forceinline__ double g_abs(double x) { return fabs(x); }
__device__ __forceinline__ float g_fmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double g_fmax(double a, double b) { return fmax(a, b); }

// 1/sqrt(x) for x > 0: the hardware estimate (v_rsq_*) refined by Newton steps
// y <- y + y*(1/2 - x*y*y/2); two steps for double (error <= ~2 ulp), one for float.  Replaces
// a divide + square-root pair (~20 dependent f64 instructions) on the substep's critical chain.
__device__ __forceinline__ double g_rsqrt(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}
// One Newton step only: v_rsq_f64 is good to ~2^29 ulp (2^-23 relative), one step squares that
// to ~2^-46 - for the drone <-> drone narrowphase's radial scaling (0.06 m x 2^-46 ~ 1e-15 m).
__device__ __forceinline__ double g_rsqrt1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return fma(y, fma(-(0.5 * x) * y, y, 0.5), y);
}
__device__ __forceinline__ float g_rsqrt1(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  return fmaf(y, fmaf(-(0.5f * x) * y, y, 0.5f), y);
}
// k / sqrt(x) with g_rsqrt1's one Newton step, the scale folded into the step (one dependent
// operation fewer than k * g_rsqrt1(x)).  x = 0 gives NaN (0 * inf in the step), not inf.
__device__ __forceinline__ double g_krsqrt1(double x, double k) {
  const double y = __builtin_amdgcn_rsq(x), ky = k * y;
  return fma(ky, fma(-(0.5 * x) * y, y, 0.5), ky);
}
__device__ __forceinline__ float g_krsqrt1(float x, float k) {
  const float y = __builtin_amdgcn_rsqf(x), ky = k * y;
  return fmaf(ky, fmaf(-(0.5f * x) * y, y, 0.5f), ky);
}
// IEEE minNum / maxNum as ONE instruction each (a NaN operand yields the other operand): for
// operands that are arithmetic results, where fmin / fmax would add canonicalising maxes
__device__ __forceinline__ double g_min1(double a, double b) {
  double o;
  asm("v_min_f64 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}
__device__ __forceinline__ double g_max1(double a, double b) {
  double o;
  asm("v_max_f64 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}
__device__ __forceinline__ float g_min1(float a, float b) {
  float o;
  asm("v_min_f32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}
__device__ __forceinline__ float g_max1(float a, float b) {
  float o;
  asm("v_max_f32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}
__device__ __forceinline__ float g_rsqrt(float x) {
  float y = __builtin_amdgcn_rsqf(x);
  const float h = 0.5f * x;
  const float e = fmaf(-h * y, y, 0.5f);
  return fmaf(y, e, y);
}

// 1/x for finite x != 0: the hardware estimate (v_rcp_*) refined by Newton steps
// y <- y + y*(1 - x*y); two steps for double (within ~1 ulp of the IEEE quotient), one for float.
// An IEEE f64 divide is a ~10-instruction dependent sequence (div_scale / rcp / 4 fma /
// div_fmas / div_fixup).  Only for operands bounded away from 0 and inf (the ground-effect prop
// heights are clipped at GND_EFF_H_CLIP > 0).
__device__ __forceinline__ double g_rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ float g_rcp(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  return fmaf(y, fmaf(-x, y, 1.0f), y);
}

template <typename R> struct PiC;
template <> struct PiC<float> { static constexpr float pi = 3.14159265358979323846f; };
template <> struct PiC<double> { static constexpr double pi = 3.14159265358979323846; };

// ---------------------------------------------------------------- model constants (device memory)
enum : int { MODEL_CF2X = 0, MODEL_CF2P = 1, MODEL_RACE = 2 };
enum : int { F_GND = 1, F_DRAG = 2, F_DW = 4, F_GEOM = 8, F_BULLET = 16, F_NO_PLANE = 32, F_NO_DC = 64 };
// PF, the physics flags a kernel is compiled for: 0 = plain DYN (the FAST path), a flag set =
// those terms compiled in (no flag tests, one basic block per substep), kPfRuntime = the terms
// selected at run time from Consts::flags (every other combination).
constexpr int kPfRuntime = -1;
template <int PF>
__device__ __forceinline__ bool pf_on(int flags, int f) {
  return PF == kPfRuntime ? (flags & f) != 0 : (PF & f) != 0;
}

// DSLPIDControl coefficients (control/DSLPIDControl.py:37-60, settable like
// BaseControl.setPIDCoefficients :138-177) and the controller's own constants.
template <typename R>
struct PidConsts {
  R p_for[3], i_for[3], d_for[3];          // P/I/D_COEFF_FOR
  R p_tor[3], i_tor[3], d_tor[3];          // P/I/D_COEFF_TOR
  R pwm2rpm_scale, pwm2rpm_const, min_pwm, max_pwm;
  R mixer[12];                             // MIXER_MATRIX [4][3]
  R gravity, kf;                           // g*m and KF of the cf2x URDF (BaseControl.py:35-39)
  R ctrl_dt;                               // CTRL_TIMESTEP = 1./CTRL_FREQ
  double speed_limit;                      // VEL: 0.03*MAX_SPEED_KMH*(1000/3600)  BaseRLAviary.py:95
};

template <typename R>
struct Consts {
  R dt;                    // PYB_TIMESTEP = 1./PYB_FREQ              BaseAviary.py:83
  R hdt, hdt2;             // dt/2 and (dt/2)^2 (_integrateQ half angle, :887)
  R m, gravity;            // M, GRAVITY = G*M                        :97, :117
  R kf, km, L, Ls2;        // KF, KM, L, L/np.sqrt(2)                 :847
  R jx, jy, jz;            // J diagonal                              :996
  R ijx, ijy, ijz;         // J_INV diagonal                          :997
  R ge_coeff, prop_r, ge_clip;             // :108-109, :128
  R drag_xy, drag_z, two_pi;               // :1009, 2*np.pi (:773)
  R dw1, dw2, dw3;                         // :1010-1012
  R dwk1;                                  // DW1 * (PROP_RADIUS/4)^2 (downwash alpha numerator)
  R rx[4], ry[4], rz[4];                   // prop link origins (cf2x.urdf:42,54,66,78)
  R inv_m;                 // 1/M      (F/M as a multiply; differs from the division by <= 1 ulp)
  R rpm2rad;               // 2*pi/60  (drag: sum(2*pi*rpm/60))
  R lin_damp, ang_damp;    // btMultiBody m_linearDamping / m_angularDamping defaults (F_BULLET)
  R max_vel;               // btMultiBody m_maxCoordinateVelocity (F_BULLET)
  R ang_thr2;              // (ANGULAR_MOTION_THRESHOLD/2)^2: the clamped half angle, squared
  // ground-plane contact of the PYB* modes (plane_contact; oracle/bullet_mb.py plane_contact)
  R cyl_r, cyl_hh, cyl_zoff;   // collision cylinder (cf2x.urdf:31-35): radius, half length, z offset
  R brk;                       // contact breaking threshold (0.02 x the cylinder's motion disc)
  R slop, erp, mu, plane_half, resid;   // m_linearSlop, m_erp2, combined friction, plane box, residual
  R dd_reach2, dd_mu;          // drone <-> drone contact: broadphase (2 x bounding sphere + brk)^2, friction
  int iters;                   // m_numIterations
  R init0[10];             // reset template of drone 0 (pos, stored quat, rpy): single-drone envs
  R target0[3];            // task target of drone 0 (single-drone envs: no dependent global load)
                           // read it with scalar loads instead of a dependent per-lane load
  float hover_f32;         // float32(HOVER_RPM) (numpy 1.x casting, BaseRLAviary.py:192)
  int model, flags, nsub;
  PidConsts<R> pid;        // PID / VEL / ONE_D_PID action types only
};

// The constants the substep loop reads every iteration, held in VGPRs: with the 64-bit
// constants in SGPRs the loop runs out of scalar registers and hipcc re-loads them with
// s_load + s_waitcnt inside the loop (a scalar-cache round trip per use).
template <typename R>
struct DynK {
  R dt, inv_m, gravity, jx, jy, jz, ijx, ijy, ijz, hdt, hdt2;
  R kf, km, L, Ls2;        // propeller wrench (rpm_wrench)
  float hover_f32;         // action -> RPM
  int model, flags, nsub;
};
template <typename R>
__device__ __forceinline__ R vpin(R x) {
  asm volatile("" : "+v"(x));
  return x;
}
// warm0 / warm1: optional kernel-argument values to have in SGPRs by the same wait (their
// scalar loads then go out in the same batch as the constant block's).
template <typename R>
__device__ __forceinline__ DynK<R> dyn_consts(const Consts<R>& c, int warm0 = 0, const void* warm1 = nullptr) {
  DynK<R> k;
  k.dt = c.dt; k.inv_m = c.inv_m; k.gravity = c.gravity;
  k.jx = c.jx; k.jy = c.jy; k.jz = c.jz;
  k.ijx = c.ijx; k.ijy = c.ijy; k.ijz = c.ijz;
  k.hdt = c.hdt; k.hdt2 = c.hdt2;
  k.kf = c.kf; k.km = c.km; k.L = c.L; k.Ls2 = c.Ls2; k.hover_f32 = c.hover_f32; k.model = c.model;
  k.flags = c.flags; k.nsub = c.nsub;
  // one statement for all of them: hipcc issues the scalar loads of every constant-block line
  // back to back and waits once (K$ misses in parallel), instead of a load + wait pair per use
  // behind each model / flag branch
#ifndef GPD_NO_DYNK_PIN
  asm volatile("" : "+v"(k.dt), "+v"(k.inv_m), "+v"(k.gravity), "+v"(k.jx), "+v"(k.jy), "+v"(k.jz),
               "+v"(k.ijx), "+v"(k.ijy), "+v"(k.ijz), "+v"(k.hdt), "+v"(k.hdt2), "+v"(k.kf), "+v"(k.km),
               "+v"(k.L), "+v"(k.Ls2), "+v"(k.hover_f32), "+s"(k.model), "+s"(k.flags),
               "+s"(k.nsub)
               : "s"(warm0), "s"(warm1));
#endif
  return k;
}

template <typename R>
struct Drone {
  R px, py, pz;            // base position (physics-client copy == self.pos)
  R qx, qy, qz, qw;        // base orientation AS STORED by resetBasePositionAndOrientation
  R vx, vy, vz;            // base linear velocity
  R wx, wy, wz;            // self.rpy_rates (body rates, DYN only)      :477, :874
  R ax, ay, az;            // base angular velocity as written, R(q)·ω   :870
};

// ---------------------------------------------------------------- Bullet3 rotation helpers
// btMatrix3x3::setRotation (pybullet getMatrixFromQuaternion, BaseAviary.py:836): row-major.
// The literal Bullet helpers (quat_to_mat, mat_to_quat, quat_to_euler) are compiled without FP
// contraction: Bullet's double-precision build (and numpy) rounds every product and sum.
template <typename R>
__device__ __forceinline__ void quat_to_mat(R x, R y, R z, R w, R m[9]) {
#pragma clang fp contract(off)
  const R d = x * x + y * y + z * z + w * w;
  const R s = R(2) / d;
  const R xs = x * s, ys = y * s, zs = z * s;
  const R wx = w * xs, wy = w * ys, wz = w * zs;
  const R xx = x * xs, xy = x * ys, xz = x * zs;
  const R yy = y * ys, yz = y * zs, zz = z * zs;
  m[0] = R(1) - (yy + zz); m[1] = xy - wz;           m[2] = xz + wy;
  m[3] = xy + wz;          m[4] = R(1) - (xx + zz);  m[5] = yz - wx;
  m[6] = xz - wy;          m[7] = yz + wx;           m[8] = R(1) - (xx + yy);
}

// btMatrix3x3::getRotation: basis -> quaternion [x,y,z,w] (w > 0 when trace > 0).
template <typename R>
__device__ __forceinline__ void mat_to_quat(const R m[9], R q[4]) {
#pragma clang fp contract(off)
  const R trace = m[0] + m[4] + m[8];
  if (trace > R(0)) {
    R s = g_sqrt(trace + R(1));
    q[3] = s * R(0.5);
    s = R(0.5) / s;
    q[0] = (m[7] - m[5]) * s;
    q[1] = (m[2] - m[6]) * s;
    q[2] = (m[3] - m[1]) * s;
  } else {
    // i = index of the largest diagonal entry, j = i+1, k = i+2 (mod 3); the three cases are
    // spelled out so that every matrix access is a compile-time register index.
    const int i = m[0] < m[4] ? (m[4] < m[8] ? 2 : 1) : (m[0] < m[8] ? 2 : 0);
    if (i == 0) {         // j = 1, k = 2
      R s = g_sqrt(((m[0] - m[4]) - m[8]) + R(1));
      q[0] = s * R(0.5);
      s = R(0.5) / s;
      q[3] = (m[7] - m[5]) * s;
      q[1] = (m[3] + m[1]) * s;
      q[2] = (m[6] + m[2]) * s;
    } else if (i == 1) {  // j = 2, k = 0
      R s = g_sqrt(((m[4] - m[8]) - m[0]) + R(1));
      q[1] = s * R(0.5);
      s = R(0.5) / s;
      q[3] = (m[2] - m[6]) * s;
      q[2] = (m[7] + m[5]) * s;
      q[0] = (m[1] + m[3]) * s;
    } else {              // j = 0, k = 1
      R s = g_sqrt(((m[8] - m[0]) - m[4]) + R(1));
      q[2] = s * R(0.5);
      s = R(0.5) / s;
      q[3] = (m[3] - m[1]) * s;
      q[0] = (m[2] + m[6]) * s;
      q[1] = (m[5] + m[7]) * s;
    }
  }
}

// Readback of the orientation (BaseAviary.py:517): the stored quaternion comes back through
// a btTransform basis, which re-normalises it.
template <typename R>
__device__ __forceinline__ void quat_readback(R x, R y, R z, R w, R qn[4]) {
  R m[9];
  quat_to_mat(x, y, z, w, m);
  mat_to_quat(m, qn);
}

// Fused readback + rotation matrix, the form the hot loop uses.  Mathematically identical to
// quat_readback() followed by quat_to_mat(qn): Bullet's basis->quaternion conversion returns
// q/|q| with the sign chosen so that w > 0 when trace(R) > 0, else so that the component of the
// largest diagonal entry is positive, and mat(q/|q|) == mat(q) because setRotation divides by
// |q|^2.  Computing it this way saves a second matrix build and a square-root branch per
// substep; the results differ from the literal Bullet sequence only by rounding (~1 ulp).
template <typename R> struct UnitTol;
template <> struct UnitTol<double> { static constexpr double v = 1e-9; };
template <> struct UnitTol<float> { static constexpr float v = 1e-4f; };

// 1/|q| with Bullet's sign (inv) and the rotation matrix.  Bullet's basis->quaternion
// conversion returns q/|q| with the sign chosen so that w > 0 when trace(R) > 0 (rotation angle
// < 120 deg), else so that the component of the largest diagonal entry is positive.  The angle
// includes yaw, which HoverAviary leaves free: a tenth of the drones of a random-action batch
// sit past 120 deg, so the key is selected branch-free (a branch would cost every wave that
// holds one of them).
template <typename R>
__device__ __forceinline__ void readback_core(R x, R y, R z, R w, R& inv, R m[9]) {
  const R d = x * x + y * y + z * z + w * w;
  // |q| = 1 +- eps (every quaternion _integrateQ produces from a unit one: its update matrix
  // is orthogonal): one Newton step from 1 gives 1/sqrt(d) and 2/d with errors 3eps^2/8 and
  // 2eps^2, below the last bit for |eps| < 1e-9 (double) / 1e-4 (float).  Both forms are
  // evaluated and selected, which keeps the substep one basic block (no exec-mask branch).
  const bool unit = g_abs(d - R(1)) < UnitTol<R>::v;
  const R invr = g_rsqrt(d);                            // 1/|q|
  const R inv0 = unit ? R(1.5) - R(0.5) * d : invr;
  const R s = unit ? R(2) * (R(2) - d) : R(2) * (invr * invr);   // 2/|q|^2 (setRotation's s)
  const R xs = x * s, ys = y * s, zs = z * s;
  const R wx = w * xs, wy = w * ys, wz = w * zs;
  const R xx = x * xs, xy = x * ys, xz = x * zs;
  const R yy = y * ys, yz = y * zs, zz = z * zs;
  m[0] = R(1) - (yy + zz); m[1] = xy - wz;           m[2] = xz + wy;
  m[3] = xy + wz;          m[4] = R(1) - (xx + zz);  m[5] = yz - wx;
  m[6] = xz - wy;          m[7] = yz + wx;           m[8] = R(1) - (xx + yy);
  const R trace = m[0] + m[4] + m[8];
  const R kd = m[0] < m[4] ? (m[4] < m[8] ? z : y) : (m[0] < m[8] ? z : x);
  const R key = trace > R(0) ? w : kd;
  inv = key < R(0) ? -inv0 : inv0;
}

// Sign transfer through the high 32-bit word (the sign bit): mag carries sign(key).
__device__ __forceinline__ int hi_word(double x) { return __double2hiint(x); }
__device__ __forceinline__ int hi_word(float x) { return __float_as_int(x); }
__device__ __forceinline__ double with_sign_word(double mag, int kw) {
  return __hiloint2double((__double2hiint(mag) & 0x7fffffff) | (kw & int(0x80000000)), __double2loint(mag));
}
__device__ __forceinline__ float with_sign_word(float mag, int kw) {
  return __int_as_float((__float_as_int(mag) & 0x7fffffff) | (kw & int(0x80000000)));
}

// The substep's readback for a quaternion with |q|^2 = d within UnitTol of 1 (dyn_substep
// re-normalises any other lane first): inv = 1/|q| and the rotation matrix entries the substep
// uses - the third column (thrust direction) and, with FULL, all nine (world-frame ang_v).
// SIGN: apply Bullet's sign rule to inv (w > 0 when trace > 0, else the component of the largest
// diagonal entry positive).  The substeps do not need it: the rotation matrix, the attitude
// predicates and the force terms are quadratic in q, and _integrateQ is linear in q, so a
// quaternion carried with the opposite sign gives bit-identical physics and a stored quaternion
// of the opposite sign; the step's final readback (readback_fused) applies the rule for the
// observation and the state vector.  The sign key is chosen on the high words only (one select
// per candidate); it is never +-0 for a unit quaternion (trace > 0 gives w^2 > 1/4, else the
// component of the largest diagonal entry has square >= 1/12), so its sign bit is the "< 0" test.
template <typename R, bool FULL, bool SIGN = true>
__device__ __forceinline__ void readback_unit(R x, R y, R z, R w, R d, R& inv, R m[9]) {
  const R inv0 = R(1.5) - R(0.5) * d;                   // 1/|q| (one Newton step from 1)
  const R s = R(2) * (R(2) - d);                         // 2/|q|^2
  const R xs = x * s, ys = y * s, zs = z * s;
  const R wx = w * xs, wy = w * ys, wz = w * zs;
  const R xx = x * xs, xy = x * ys, xz = x * zs;
  const R yy = y * ys, yz = y * zs, zz = z * zs;
  m[2] = xz + wy;
  m[5] = yz - wx;
  m[8] = R(1) - (xx + yy);
  if (FULL || SIGN) {
    m[0] = R(1) - (yy + zz);
    m[4] = R(1) - (xx + zz);
  }
  if (FULL) {
    m[1] = xy - wz; m[3] = xy + wz; m[6] = xz - wy; m[7] = yz + wx;
  }
  if (SIGN) {
    const R trace = m[0] + m[4] + m[8];
    int kw = m[0] < m[4] ? (m[4] < m[8] ? hi_word(z) : hi_word(y)) : (m[0] < m[8] ? hi_word(z) : hi_word(x));
    kw = trace > R(0) ? hi_word(w) : kw;
    inv = with_sign_word(inv0, kw);
  } else {
    inv = inv0;
  }
}

template <typename R>
__device__ __forceinline__ void readback_fused(R x, R y, R z, R w, R qn[4], R m[9]) {
  R inv;
  readback_core(x, y, z, w, inv, m);
  qn[0] = x * inv; qn[1] = y * inv; qn[2] = z * inv; qn[3] = w * inv;
}

// cos(theta) and sin(theta)/theta of the half rotation angle of _integrateQ (:887-888) from
// t2 = theta^2, |theta| < 0.5.  Both are even series in theta, so the step needs neither the
// square root of |omega|^2 nor a division by |omega| (error < 1e-17 relative in double,
// < 1e-9 in float).
__device__ __forceinline__ void cos_sinc(double t2, double& c, double& sc) {
  // Estrin's scheme (dependency depth 4 instead of Horner's 8; same truncation, ~1 ulp rounding)
  const double t4 = t2 * t2, t8 = t4 * t4;
  const double s01 = 1.0 + t2 * (-1.0 / 6), s23 = 1.0 / 120 + t2 * (-1.0 / 5040);
  const double s45 = 1.0 / 362880 + t2 * (-1.0 / 39916800);
  const double s67 = 1.0 / 6227020800.0 + t2 * (-1.0 / 1307674368000.0);
  sc = (s01 + t4 * s23) + t8 * (s45 + t4 * s67);
  const double c01 = 1.0 + t2 * (-0.5), c23 = 1.0 / 24 + t2 * (-1.0 / 720);
  const double c45 = 1.0 / 40320 + t2 * (-1.0 / 3628800);
  const double c67 = 1.0 / 479001600.0 + t2 * (-1.0 / 87178291200.0);
  c = (c01 + t4 * c23) + t8 * (c45 + t4 * c67);
}
__device__ __forceinline__ void cos_sinc(float t2, float& c, float& sc) {
  sc = 1.0f + t2 * (-1.0f / 6 + t2 * (1.0f / 120 + t2 * (-1.0f / 5040 + t2 * (1.0f / 362880))));
  c = 1.0f + t2 * (-0.5f + t2 * (1.0f / 24 + t2 * (-1.0f / 720 + t2 * (1.0f / 40320 + t2 * (-1.0f / 3628800)))));
}

// btQuaternion::getEulerZYX (pybullet getEulerFromQuaternion, BaseAviary.py:518).
template <typename R>
__device__ __forceinline__ void quat_to_euler(const R q[4], R& roll, R& pitch, R& yaw) {
#pragma clang fp contract(off)
  const R x = q[0], y = q[1], z = q[2], w = q[3];
  const R sqx = x * x, sqy = y * y, sqz = z * z, squ = w * w;
  const R sarg = R(-2) * (x * z - w * y);
  if (sarg <= R(-0.99999)) {
    pitch = R(-0.5) * PiC<R>::pi;
    roll = R(0);
    yaw = R(2) * g_atan2(x, -y);
  } else if (sarg >= R(0.99999)) {
    pitch = R(0.5) * PiC<R>::pi;
    roll = R(0);
    yaw = R(2) * g_atan2(-x, y);
  } else {
    R sa = sarg < R(-1) ? R(-1) : (sarg > R(1) ? R(1) : sarg);  // btAsin clamp
    pitch = g_asin(sa);
    roll = g_atan2(R(2) * (y * z + w * x), squ - sqx - sqy + sqz);
    yaw = g_atan2(R(2) * (x * y + w * z), squ + sqx - sqy - sqz);
  }
}

// Attitude predicates of the reference evaluated WITHOUT atan2/asin.  getEulerZYX gives
// pitch = asin(sarg) (or +-pi/2 in the gimbal branches) and roll = atan2(a, b) (0 in the
// branches), with sarg = -2(xz - wy), a = 2(yz + wx), b = w^2 - x^2 - y^2 + z^2.  Because asin
// and atan2 are monotonic in the relevant argument, the comparisons below are the reference's
// comparisons up to rounding exactly at the threshold.
template <typename R>
struct AttitudeArgs {
  R sarg, a, b;
  bool gimbal;  // |sarg| >= 0.99999: pitch = +-pi/2, roll = 0
};
template <typename R>
__device__ __forceinline__ AttitudeArgs<R> attitude_args(const R q[4]) {
  const R x = q[0], y = q[1], z = q[2], w = q[3];
  AttitudeArgs<R> t;
  t.sarg = R(-2) * (x * z - w * y);
  t.a = R(2) * (y * z + w * x);
  t.b = w * w - x * x - y * y + z * z;
  t.gimbal = t.sarg <= R(-0.99999) || t.sarg >= R(0.99999);
  return t;
}
// |roll| > lim or |pitch| > lim, 0 < lim < pi/2 (HoverAviary.py:112, MultiHoverAviary.py:121)
template <typename R>
__device__ __forceinline__ bool tilted_beyond(const AttitudeArgs<R>& t, R sin_lim, R tan_lim) {
  // gimbal: |pitch| = pi/2; |asin(sarg)| > lim; |atan2(a, b)| > lim (b > 0), >= pi/2 (b <= 0)
  // except atan2(+-0, +0) = 0.  Written as one predicate (no branches).
  const bool zero_roll = t.b == R(0) && t.a == R(0) && !signbit(t.b);
  const bool roll_out = t.b > R(0) ? g_abs(t.a) > tan_lim * t.b : !zero_roll;
  return t.gimbal || g_abs(t.sarg) > sin_lim || roll_out;
}
// |roll| < pi/2 and |pitch| < pi/2 (the _groundEffect condition, BaseAviary.py:742)
template <typename R>
__device__ __forceinline__ bool upright(const AttitudeArgs<R>& t) {
  return !t.gimbal && (t.b > R(0) || (t.b == R(0) && t.a == R(0) && !signbit(t.b)));
}

// ---------------------------------------------------------------- cold paths out of line
// GPD_COLD_CALLS=1: the rare branches' bodies (the library cos / sin of the _integrateQ weights for
// |theta| >= 0.5, the exact attitude re-decision) become calls, so their code sits outside the
// kernel's instruction stream instead of after its end (instruction fetch).
// Measured: headline kernel 4.97 us vs 5.03-5.34 us inline (profiles/r4/cold/); 0 = inline.
#ifndef GPD_COLD_CALLS
#define GPD_COLD_CALLS 1
#endif
#if GPD_COLD_CALLS
#define GPD_COLD __attribute__((noinline, cold))
#else
#define GPD_COLD __forceinline__
#endif
template <typename R>
struct CoSh {
  R co, sh;
};
// cos(|w| hdt) and sin(|w| hdt) / |w| from |w|^2 (the library functions: |theta| >= 0.5)
template <typename R>
__device__ GPD_COLD CoSh<R> cold_cos_sinc(R n2, R hdt) {
  const R nrm = g_sqrt(n2), th = nrm * hdt;
  return CoSh<R>{g_cos(th), g_sin(th) / nrm};
}

// ---------------------------------------------------------------- exact attitude decisions (f64)
// tilted_beyond / upright see the fused readback's quaternion (~1 ulp from Bullet's) and compare
// against rounded limits, so within a few ulp of a threshold they can disagree with the
// reference, whose decisions are made on libm atan2 / asin outputs (HoverAviary.py:111,
// MultiHoverAviary.py:124, BaseAviary.py:742).  attitude_decide re-decides the lanes of that band
// exactly: the literal Bullet readback of the stored quaternion (quat_to_mat -> mat_to_quat ->
// getEulerZYX's arguments, no FP contraction), then comparisons that equal "RN(atan2(a, b)) > 0.4",
// "RN(asin(s)) > 0.4" and "RN(atan2(a, b)) < RN(pi/2)" for correctly rounded atan2 / asin
// (glibc's, to which pybullet's btAtan2 / btAsin resolve):
//   RN(x) > 0.4   <=>  x > M  = 0.4 + ulp(0.4)/2           (the rounding midpoint)
//   asin(s) > M   <=>  s >= kSinLim, the smallest double above sin(M)
//   atan2(a,b) > M, b > 0  <=>  |a| > tan(M) b             (tan(M) as a double-double)
//   RN(x) < RN(pi/2) <=> x < Mg = RN(pi/2) - ulp/2;  atan2 < Mg, b > 0  <=>  b > cot(Mg) |a|
// The constants come from mpmath at 400 bits (tests/test_oracle_kat.py re-derives them and checks
// the rules against glibc on near-threshold samples).  Each double-double product is compared
// exactly to ~2^-106 relative (an FMA gives the product's rounding error).
struct AttK {
  static constexpr double sin_lim = 0x1.8ec3ae92b676cp-2;                                  // asin > M
  static constexpr double tan_hi = 0x1.b0f0b49dcdcd9p-2, tan_lo = -0x1.10521c23b5ec7p-56;  // tan(M)
  static constexpr double cot_hi = 0x1.8d313198a2e03p-53, cot_lo = 0x1.c1cd129024e0ap-107; // cot(Mg)
  static constexpr double gimbal = 0.99999;
  static constexpr double band = 1e-12;   // fused vs literal arguments differ by a few 1e-16
};
// u > (hi + lo) * v for u, v >= 0
__device__ __forceinline__ bool dd_above(double u, double hi, double lo, double v) {
#pragma clang fp contract(off)
  const double p = hi * v;
  const double e = fma(hi, v, -p);      // hi*v = p + e exactly
  return ((u - p) - e) - lo * v > 0.0;  // u - p is exact whenever the sign is in doubt (Sterbenz)
}

// getEulerZYX's arguments from the literal readback of the stored quaternion (x, y, z, w)
// (BaseAviary.py:517-518: getBasePositionAndOrientation -> getEulerFromQuaternion)
template <typename R>
__device__ __forceinline__ void attitude_literal(R x, R y, R z, R w, AttitudeArgs<R>& t) {
#pragma clang fp contract(off)
  R m[9], q[4];
  quat_to_mat(x, y, z, w, m);
  mat_to_quat(m, q);
  const R qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  t.sarg = R(-2) * (qx * qz - qw * qy);
  t.a = R(2) * (qy * qz + qw * qx);
  t.b = ((qw * qw - qx * qx) - qy * qy) + qz * qz;   // squ - sqx - sqy + sqz
  t.gimbal = t.sarg <= R(-0.99999) || t.sarg >= R(0.99999);
}

// the exact decisions from the literal Bullet readback (attitude_decide's rare lanes)
struct AttExact {
  double sarg, a, b;
  bool gimbal, tilt, up;
};
__device__ GPD_COLD AttExact attitude_exact(double qx, double qy, double qz, double qw) {
  AttitudeArgs<double> t;
  attitude_literal(qx, qy, qz, qw, t);
  const bool zero_roll = t.a == 0.0 && t.b == 0.0 && !signbit(t.b);   // atan2(+-0, +0) = +-0
  const bool roll_out = t.b > 0.0 ? dd_above(fabs(t.a), AttK::tan_hi, AttK::tan_lo, t.b) : !zero_roll;
  const bool roll_in = t.b > 0.0 ? dd_above(t.b, AttK::cot_hi, AttK::cot_lo, fabs(t.a)) : zero_roll;
  return AttExact{t.sarg, t.a, t.b, t.gimbal, t.gimbal || fabs(t.sarg) >= AttK::sin_lim || roll_out,
                  !t.gimbal && roll_in};
}
// TILT: tilt = |roll| > 0.4 or |pitch| > 0.4; UP: up = |roll| < pi/2 and |pitch| < pi/2.
// qs = the stored quaternion the readback starts from; t = attitude_args of the fused readback,
// replaced by the literal arguments on the lanes that were re-decided (so that the observation's
// gimbal branch follows the reference too).  Lanes outside the band keep the fused decision,
// which equals the exact one there.  f32 builds keep the fused predicates.
template <typename R, bool TILT, bool UP>
__device__ __forceinline__ void attitude_decide(R qx, R qy, R qz, R qw, AttitudeArgs<R>& t, bool& tilt, bool& up) {
  if (TILT) tilt = tilted_beyond(t, R(0.38941834230865049), R(0.42279321873816178));   // ~sin/tan(0.4)
  if (UP) up = upright(t);
  if constexpr (sizeof(R) == 8) {
    const double as = fabs(t.sarg);
    bool near = fabs(as - AttK::gimbal) < AttK::band;
    if (TILT) near = near || fabs(as - AttK::sin_lim) < AttK::band || fabs(fabs(t.a) - AttK::tan_hi * t.b) < AttK::band;
    if (UP) near = near || fabs(t.b) < AttK::band;
    if (GPD_RARE(__ballot(near) != 0ull)) {
      if (near) {
        const AttExact e = attitude_exact(qx, qy, qz, qw);
        t.sarg = e.sarg; t.a = e.a; t.b = e.b; t.gimbal = e.gimbal;
        if (TILT) tilt = e.tilt;
        if (UP) up = e.up;
      }
    }
  }
}
// float32 Euler angles for the float32 observation.  The reference computes them in float64
// (pybullet's getEulerFromQuaternion, BaseAviary.py:518) and casts them (BaseRLAviary.py:313-315).
// Here they are float32 asinf / atan2f of the double arguments (within ~2 float32 ulp of the cast
// double result).  GPD_OBS_ANGLES_F64=1 builds the reference's order - double asin / atan2, then
// the cast - and was measured on the 4096-env headline kernel (budget 0.1 us):
// 5.01-5.04 -> 5.41-5.73 us per launch (three alternations, profiles/r4/angles/), ~2 KB more code
// in the epilogue; not the default.
#ifndef GPD_OBS_ANGLES_F64
#define GPD_OBS_ANGLES_F64 0
#endif
template <typename R>
__device__ __forceinline__ void obs_euler_f32(const R q[4], const AttitudeArgs<R>& t, float& roll, float& pitch,
                                              float& yaw) {
  const R x = q[0], y = q[1], z = q[2], w = q[3];
  // the regular branch for every lane, the gimbal branches (|sarg| >= 0.99999) as a
  // wave-uniform fix-up
  const R sa = t.sarg < R(-1) ? R(-1) : (t.sarg > R(1) ? R(1) : t.sarg);
  if (GPD_OBS_ANGLES_F64 && sizeof(R) == 8) {
    pitch = (float)g_asin(sa);
    roll = (float)g_atan2(t.a, t.b);
    yaw = (float)g_atan2(R(2) * (x * y + w * z), w * w + x * x - y * y - z * z);
  } else {
    pitch = asinf((float)sa);
    roll = atan2f((float)t.a, (float)t.b);
    yaw = atan2f((float)(R(2) * (x * y + w * z)), (float)(w * w + x * x - y * y - z * z));
  }
  if (GPD_RARE(__ballot(t.gimbal) != 0ull)) {
    if (t.sarg <= R(-0.99999)) {
      pitch = -1.57079632679489661923f; roll = 0.0f; yaw = (float)(R(2) * g_atan2(x, -y));
    } else if (t.sarg >= R(0.99999)) {
      pitch = 1.57079632679489661923f; roll = 0.0f; yaw = (float)(R(2) * g_atan2(-x, y));
    }
  }
}

// float32 RPM from a float32 action exactly as numpy 1.x evaluates
// HOVER_RPM * (1 + 0.05*target) on a float32 array (BaseRLAviary.py:192, :225).
// hipcc would otherwise contract 1 + 0.05*a into one FMA (even through __fmul_rn/__fadd_rn),
// which differs from numpy's two separately rounded float32 ops by up to 2 ulps of the RPM.
__device__ __forceinline__ float action_to_rpm(float hover_f32, float a) {
#pragma clang fp contract(off)
  const float t = 0.05f * a;
  const float u = 1.0f + t;
  return hover_f32 * u;
}

// Thrust and body torques of the propellers (BaseAviary.py:838-851).  They depend on the RPMs
// only, so the step kernel evaluates them once per control step, outside the substep loop.
// Evaluated with FP contraction OFF, like numpy: with contraction hipcc fuses r^2*kf into the
// following add, so four equal RPMs (every ONE_D_RPM action, the hover equilibrium) would leave
// a residual roll/pitch torque instead of the reference's exact zero.
// W = {fz, tx, ty, tz} in the body frame.
template <typename R, int PF>
__device__ __forceinline__ void rpm_wrench(const R rpm[4], const DynK<R>& k, const Consts<R>& c, R W[4]) {
#pragma clang fp contract(off)
  R f[4], zt[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const R r2 = rpm[m] * rpm[m];
    f[m] = r2 * k.kf;                                  // :838
    zt[m] = r2 * k.km;                                 // :842
  }
  if (k.model == MODEL_RACE) {
#pragma unroll
    for (int m = 0; m < 4; ++m) zt[m] = -zt[m];        // :843-844
  }
  W[0] = ((f[0] + f[1]) + f[2]) + f[3];                // np.sum(forces) :839
  W[3] = ((-zt[0] + zt[1]) - zt[2]) + zt[3];           // :845
  if (pf_on<PF>(k.flags, F_GEOM)) {                   // _physics: forces at prop links :698-705
    R tx = R(0), ty = R(0);
#pragma unroll
    for (int m = 0; m < 4; ++m) { tx = tx + c.ry[m] * f[m]; ty = ty - c.rx[m] * f[m]; }
    W[1] = tx; W[2] = ty;
  } else if (k.model == MODEL_CF2P) {                  // :849-851
    W[1] = (f[1] - f[3]) * k.L;
    W[2] = (-f[0] + f[2]) * k.L;
  } else {                                             // CF2X / RACE :846-848 (roll-sign quirk kept)
    W[1] = (((f[0] + f[1]) - f[2]) - f[3]) * k.Ls2;
    W[2] = (((-f[0] + f[1]) + f[2]) - f[3]) * k.Ls2;
  }
}

// Body wrench of one substep: the propeller wrench W plus, with F_GND, the ground effect
// (_groundEffect :732-750) at the current pose.
template <typename R, int PF>
__device__ __forceinline__ void body_wrench(const Drone<R>& s, const R Rm[9], bool gnd_upright, const R rpm[4],
                                            const R W[4], const Consts<R>& c, const DynK<R>& kk, R& fz_out, R& tx_out,
                                            R& ty_out, R& tz_out) {
#pragma clang fp contract(off)
  R fz = W[0], tx = W[1], ty = W[2];
  if (pf_on<PF>(kk.flags, F_GND)) {
    // prop COM heights via forward kinematics, clipped, +z link force at each prop; applied only
    // while upright (a select, not a branch)
    R g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      R h = s.pz + ((Rm[6] * c.rx[k] + Rm[7] * c.ry[k]) + Rm[8] * c.rz[k]);
      h = h < c.ge_clip ? c.ge_clip : h;
      const R qq = c.prop_r * g_rcp(R(4) * h);   // h >= GND_EFF_H_CLIP > 0
      g[k] = ((rpm[k] * rpm[k]) * c.kf * c.ge_coeff) * (qq * qq);
    }
    const R gz = ((g[0] + g[1]) + g[2]) + g[3];
    R gx = R(0), gy = R(0);
#pragma unroll
    for (int k = 0; k < 4; ++k) { gx = gx + c.ry[k] * g[k]; gy = gy - c.rx[k] * g[k]; }
    fz = gnd_upright ? fz + gz : fz;
    tx = gnd_upright ? tx + gx : tx;
    ty = gnd_upright ? ty + gy : ty;
  }
  fz_out = fz;
  tx_out = tx;
  ty_out = ty;
  tz_out = W[3];
}

// ---------------------------------------------------------------- ground-plane contact (PYB*)
// The drone's collision cylinder (cf2x.urdf:31-35) against plane.urdf (BaseAviary.py:484; the
// collision filter at :500-503 is commented out), solved the way btMultiBodyConstraintSolver
// does inside p.stepSimulation(): after the unconstrained velocity update, before
// integrateTransforms, on the pose at the start of the step.  Restatement and its constants:
// oracle/bullet_mb.py plane_contact (parity unpinned: pybullet is absent).
//   * candidates: the rim points at body azimuth 0/90/180/270 deg of the cap facing down; a
//     point joins when its height is below the breaking threshold and it lies over the plane
//     box's top face;
//   * rows per point, in base-frame coordinates (M^-1 = diag(1/m, 1/I)): normal = world +z, two
//     friction directions (0,-1,0), (1,0,0) solved as a pair on the implicit cone;
//   * projected Gauss-Seidel: every normal row, then every friction pair, per iteration; stop
//     when the largest squared residual <= resid or after `iters` iterations.
// Inactive points carry rhs = jdi = 0, so their rows solve to a zero impulse without a branch.
// The caller gates the call on a wave ballot: a wave without a low drone never enters.
template <typename R>
__device__ __forceinline__ R pc_dot(R ax, R ay, R az, R bx, R by, R bz) { return (ax * bx + ay * by) + az * bz; }
constexpr int kWaveLanes = 64;

#ifdef GPD_CONTACT_STATS
// diagnostic build only: per solving wave, the iterations run [0..50] and the active lanes [51..115];
// 116..127 drone-contact totals (DcHook / dc_solve); 128..191 log2 histogram of a drone-contact
// solve's cycles; 192..242 its iteration histogram; 256 + b: block b's drone-contact cycles;
// 256 + 4096 + b: block b's step-kernel cycles; 256 + 8192 + b: block b's plane-solve cycles;
// 256 + 12288 + b: block b's drone-contact rare-path cycles (the hook's solve branch, call included)
constexpr int kPcHist = 256 + 4 * 4096 + 16;   // + 16: narrowphase phase cycles (dc_narrow_pass)
constexpr int kPcNp = 256 + 4 * 4096;
__device__ unsigned long long g_pc_hist[kPcHist];
#endif
// r_p x d for the rim point p (p = 0..3: (cr,0,zc), (0,cr,zc), (-cr,0,zc), (0,-cr,zc)), with the
// zero components dropped (exact: 0*x - y == -y).
template <int P, typename R>
__device__ __forceinline__ void pc_arm(R cr, R zc, R dx, R dy, R dz, R& ax, R& ay, R& az) {
  if (P == 0) { ax = -(zc * dy); ay = zc * dx - cr * dz; az = cr * dy; }
  if (P == 1) { ax = cr * dz - zc * dy; ay = zc * dx; az = -(cr * dx); }
  if (P == 2) { ax = -(zc * dy); ay = zc * dx + cr * dz; az = -(cr * dy); }
  if (P == 3) { ax = -(cr * dz) - zc * dy; ay = zc * dx; az = cr * dx; }
}

// skip: this lane's drone takes no part (its plane rows were solved in the drone <-> drone island)
template <typename R>
__device__ __forceinline__ void plane_contact(Drone<R>& s, const R Rm[9], const Consts<R>& c, const DynK<R>& k,
                                              bool skip = false) {
  // The rows' constants (rhs, 1/jacDiag, jacDiag) and impulses live in LDS, one column per lane
  // of the block's single wave (the run-time-flag kernels, which also serve non-contact configs,
  // and the multi-wave envs; the PYB flag-set kernels use plane_contact_regs below).  Kept in
  // registers with the point loops unrolled, the 12 rows' Jacobians would be hoisted out of the
  // iteration loop and raise the whole kernel's VGPR count for a path that only grounded drones take.
  enum { kRhs = 0, kJdi = 3, kJdn = 6, kLam = 7, kPer = 10 };
  __shared__ R pc[4 * kPer][64];
  const int ln = threadIdx.x & 63;
  const R nx = Rm[6], ny = Rm[7], nz = Rm[8];          // base-frame world +z
  const R ux = -Rm[3], uy = -Rm[4], uz = -Rm[5];       // (0,-1,0)
  const R ex = Rm[0], ey = Rm[1], ez = Rm[2];          // (1,0,0)
  const R zc = (-Rm[8] < R(0) ? -c.cyl_hh : c.cyl_hh) + c.cyl_zoff;
  const R cr = c.cyl_r;
  bool any = false;
  {
    // base-frame velocities
    const R vbx = pc_dot(Rm[0], Rm[3], Rm[6], s.vx, s.vy, s.vz);
    const R vby = pc_dot(Rm[1], Rm[4], Rm[7], s.vx, s.vy, s.vz);
    const R vbz = pc_dot(Rm[2], Rm[5], Rm[8], s.vx, s.vy, s.vz);
    const R wbx = pc_dot(Rm[0], Rm[3], Rm[6], s.wx, s.wy, s.wz);
    const R wby = pc_dot(Rm[1], Rm[4], Rm[7], s.wx, s.wy, s.wz);
    const R wbz = pc_dot(Rm[2], Rm[5], Rm[8], s.wx, s.wy, s.wz);
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      const R rx = p == 0 ? cr : (p == 2 ? -cr : R(0)), ry = p == 1 ? cr : (p == 3 ? -cr : R(0));
      const R dist = s.pz + pc_dot(nx, ny, nz, rx, ry, zc);
      const R wxp = s.px + pc_dot(Rm[0], Rm[1], Rm[2], rx, ry, zc);
      const R wyp = s.py + pc_dot(Rm[3], Rm[4], Rm[5], rx, ry, zc);
      const bool act = !skip && dist < c.brk && g_abs(wxp) <= c.plane_half && g_abs(wyp) <= c.plane_half;
      any = any || act;
      const R dx[3] = {nx, ux, ex}, dy[3] = {ny, uy, ey}, dz[3] = {nz, uz, ez};
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const R ax = ry * dz[j] - zc * dy[j], ay = zc * dx[j] - rx * dz[j], az = rx * dy[j] - ry * dx[j];
        const R jd = k.inv_m + ((ax * (ax * k.ijx) + ay * (ay * k.ijy)) + az * (az * k.ijz));
        const R inv = R(1) / jd;
        const R rel = pc_dot(dx[j], dy[j], dz[j], vbx, vby, vbz) + pc_dot(ax, ay, az, wbx, wby, wbz);
        R r;
        if (j == 0) {
          const R pen = dist + c.slop;
          r = pen > R(0) ? (-rel - pen / k.dt) * inv : (-pen * c.erp / k.dt - rel) * inv;
          pc[p * kPer + kJdn][ln] = act ? jd : R(0);
        } else {
          r = -rel * inv;
        }
        pc[p * kPer + kJdi + j][ln] = act ? inv : R(0);
        pc[p * kPer + kRhs + j][ln] = act ? r : R(0);
        pc[p * kPer + kLam + j][ln] = R(0);
      }
    }
  }
  const R nx_ = nx, ny_ = ny, nz_ = nz, ux_ = ux, uy_ = uy, uz_ = uz, ex_ = ex, ey_ = ey, ez_ = ez;
  const R zc_ = zc, cr_ = cr;
  R dl0 = R(0), dl1 = R(0), dl2 = R(0), da0 = R(0), da1 = R(0), da2 = R(0);
  bool done = !any;
  const R mu = vpin(c.mu), resid = vpin(c.resid);      // once, not a constant-block load per iteration
  const int iters = c.iters;
#ifdef GPD_CONTACT_STATS
  int it_used = 0;
  const unsigned long long nact = __ballot(any);
#endif
  for (int it = 0; it < iters; ++it) {
    if (__ballot(!done) == 0ull) break;
#ifdef GPD_CONTACT_STATS
    it_used = it + 1;
#endif
    if (!done) {
      // opaque per iteration: the row Jacobians are recomputed, not hoisted (see above)
      const R nx = vpin(nx_), ny = vpin(ny_), nz = vpin(nz_), ux = vpin(ux_), uy = vpin(uy_), uz = vpin(uz_);
      const R ex = vpin(ex_), ey = vpin(ey_), ez = vpin(ez_), zc = vpin(zc_), cr = vpin(cr_);
      R res = R(0);
#pragma unroll
      for (int p = 0; p < 4; ++p) {                  // normal rows
        R ax, ay, az;
        if (p == 0) pc_arm<0>(cr, zc, nx, ny, nz, ax, ay, az);
        if (p == 1) pc_arm<1>(cr, zc, nx, ny, nz, ax, ay, az);
        if (p == 2) pc_arm<2>(cr, zc, nx, ny, nz, ax, ay, az);
        if (p == 3) pc_arm<3>(cr, zc, nx, ny, nz, ax, ay, az);
        const R jv = pc_dot(nx, ny, nz, dl0, dl1, dl2) + pc_dot(ax, ay, az, da0, da1, da2);
        R delta = pc[p * kPer + kRhs][ln] - pc[p * kPer + kJdi][ln] * jv;
        const R lam = pc[p * kPer + kLam][ln];
        const R sum = lam + delta;
        const bool neg = sum < R(0);
        delta = neg ? -lam : delta;
        pc[p * kPer + kLam][ln] = neg ? R(0) : sum;
        const R dm = k.inv_m * delta;
        dl0 = dl0 + nx * dm; dl1 = dl1 + ny * dm; dl2 = dl2 + nz * dm;
        da0 = da0 + (ax * k.ijx) * delta; da1 = da1 + (ay * k.ijy) * delta; da2 = da2 + (az * k.ijz) * delta;
        const R rr = delta * pc[p * kPer + kJdn][ln];
        res = g_fmax(res, rr * rr);   // the oracle's max(res, x); x = rr^2 is never -0, NaN keeps res
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {                  // friction pairs on the cone
        R bx, by, bz, cx, cy, cz;
        if (p == 0) { pc_arm<0>(cr, zc, ux, uy, uz, bx, by, bz); pc_arm<0>(cr, zc, ex, ey, ez, cx, cy, cz); }
        if (p == 1) { pc_arm<1>(cr, zc, ux, uy, uz, bx, by, bz); pc_arm<1>(cr, zc, ex, ey, ez, cx, cy, cz); }
        if (p == 2) { pc_arm<2>(cr, zc, ux, uy, uz, bx, by, bz); pc_arm<2>(cr, zc, ex, ey, ez, cx, cy, cz); }
        if (p == 3) { pc_arm<3>(cr, zc, ux, uy, uz, bx, by, bz); pc_arm<3>(cr, zc, ex, ey, ez, cx, cy, cz); }
        const R lnrm = pc[p * kPer + kLam][ln];
        const bool on = lnrm > R(0);
        const R lim = mu * lnrm;
        const R l1 = pc[p * kPer + kLam + 1][ln], l2 = pc[p * kPer + kLam + 2][ln];
        const R j1 = pc_dot(ux, uy, uz, dl0, dl1, dl2) + pc_dot(bx, by, bz, da0, da1, da2);
        const R j2 = pc_dot(ex, ey, ez, dl0, dl1, dl2) + pc_dot(cx, cy, cz, da0, da1, da2);
        R s1 = l1 + (pc[p * kPer + kRhs + 1][ln] - pc[p * kPer + kJdi + 1][ln] * j1);
        R s2 = l2 + (pc[p * kPer + kRhs + 2][ln] - pc[p * kPer + kJdi + 2][ln] * j2);
        // onto the cone: (s1, s2) * lim / |s| when |s| > lim (a select: no branch, and the
        // Newton-refined rsqrt instead of a square root and a divide; within ~2 ulp of them)
        const R m2 = s1 * s1 + s2 * s2;
        const bool clip = m2 > lim * lim;
        const R f = clip ? lim * g_rsqrt(clip ? m2 : R(1)) : R(1);
        s1 = s1 * f;
        s2 = s2 * f;
        const R d1 = on ? s1 - l1 : R(0);
        const R d2 = on ? s2 - l2 : R(0);
        pc[p * kPer + kLam + 1][ln] = on ? s1 : l1;
        pc[p * kPer + kLam + 2][ln] = on ? s2 : l2;
        const R m1 = k.inv_m * d1, m2v = k.inv_m * d2;
        dl0 = dl0 + ux * m1; dl1 = dl1 + uy * m1; dl2 = dl2 + uz * m1;
        da0 = da0 + (bx * k.ijx) * d1; da1 = da1 + (by * k.ijy) * d1; da2 = da2 + (bz * k.ijz) * d1;
        dl0 = dl0 + ex * m2v; dl1 = dl1 + ey * m2v; dl2 = dl2 + ez * m2v;
        da0 = da0 + (cx * k.ijx) * d2; da1 = da1 + (cy * k.ijy) * d2; da2 = da2 + (cz * k.ijz) * d2;
        const R rr = (d1 + d2) * (d1 + d2);
        res = g_fmax(res, rr);
      }
      done = res <= resid;
    }
  }
#ifdef GPD_CONTACT_STATS
  if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
    atomicAdd(&g_pc_hist[it_used], 1ull);
    atomicAdd(&g_pc_hist[51 + __popcll(nact)], 1ull);
  }
#endif
  // back to world coordinates (rows of Rm: world = Rm . base); lanes without an active point
  // keep their velocities bit for bit, signed zeros included
  s.vx = any ? s.vx + pc_dot(Rm[0], Rm[1], Rm[2], dl0, dl1, dl2) : s.vx;
  s.vy = any ? s.vy + pc_dot(Rm[3], Rm[4], Rm[5], dl0, dl1, dl2) : s.vy;
  s.vz = any ? s.vz + pc_dot(Rm[6], Rm[7], Rm[8], dl0, dl1, dl2) : s.vz;
  s.wx = any ? s.wx + pc_dot(Rm[0], Rm[1], Rm[2], da0, da1, da2) : s.wx;
  s.wy = any ? s.wy + pc_dot(Rm[3], Rm[4], Rm[5], da0, da1, da2) : s.wy;
  s.wz = any ? s.wz + pc_dot(Rm[6], Rm[7], Rm[8], da0, da1, da2) : s.wz;
}

// plane_contact solved in WORLD coordinates with every row in VGPRs, for the kernels compiled for
// a PYB flag set (one-wave blocks; at the PYB configs' sizes a block is one thin wave per CU, so
// registers cost no occupancy).  The same projected Gauss-Seidel solve - same rows, order,
// projections and stopping rule - in the frame where the rows are sparse.  The row directions
// are the world axes (+z, (0,-1,0), (1,0,0)); with the solver's velocity changes kept in world
// coordinates (DL = R dl, DA = R da) a row's Jacobian product d.DL + (r x d).DA has ONE linear
// and TWO angular terms (r = the rim point's world arm), and a linear update touches one
// component.  Per row the base-frame products of the LDS solve (two 3-term dot products, three
// linear and three angular updates, the arm . I^-1 products) become 2 FMAs + 1 + 3 FMAs with
// g = I_w^-1 (r x d), I_w^-1 = R diag(1/I) R^T formed once per solve.  In exact arithmetic every
// quantity equals the base-frame one (R is orthonormal); the results differ by rounding only
// (tests/test_gpu_bullet.py's resynced and long-run contact gates).
//   * normal rows nobody in the wave touches are skipped (wave-uniform, decided once per solve);
//     a friction pair runs exec-masked on the lanes with a positive normal impulse at its point
//     (the others skip it, as the oracle does), and the cone projection on the lanes whose
//     impulse leaves the cone;
//   * a normal row's clamp at 0 applies new - old (== -old when clamped, the oracle's form);
//   * residual: the largest |row residual| is squared once per iteration (squaring is monotonic,
//     so this equals the largest squared residual exactly).
// (Round 6: a look-ahead form - unit k's row product as J_k v_{k-2} plus a per-solve coupling
// times d_{k-1}, one dependent FMA after its predecessor - measured 61.5 -> 72.1 us on the 4096-env
// PYB crash batch, branch-free and without the row skips: the loop is issue-bound, not chain-bound;
// profiles/r6/contact/probe_plane_lookahead_ab.log.)
// A solve holds its wave for (setup + iterations x ~300 instructions); a crashing
// batch's worst solve and the multi-drone batches' solves run into the iteration cap (50), so the
// per-iteration instruction count is what the PYB step time follows.  PK's park() / unpark()
// run after the setup and after the iterations: the caller moves what it keeps across the solve
// out of VGPRs for the iterations (bullet_substep).
#ifndef GPD_CONTACT_PARK
#define GPD_CONTACT_PARK 1   // 0: diagnostic builds (A/B of the parking)
#endif
// kStage: the drone <-> drone solve stages its sweeps' operands in LDS (gpd_kernels.h DcStage) -
// the parking callers are the compiled-in PYB flag-set kernels, whose LDS has the room
struct NoPark {
  static constexpr bool kStage = false;
  __device__ void park() const {}
  __device__ void unpark() const {}
};
template <class A, class B>
struct ParkFns {
  static constexpr bool kStage = true;
  A a;
  B b;
  __device__ void park() const { a(); }
  __device__ void unpark() const { b(); }
};
// max(r, |x|) for a running residual r that is already canonical: one v_max_f64 (fmax would add
// a canonicalising max of r per call).  A NaN x keeps r, as the oracle's max(res, x).
__device__ __forceinline__ double max_abs(double r, double x) {
  double o;
  asm("v_max_f64 %0, %1, |%2|" : "=v"(o) : "v"(r), "v"(x));
  return o;
}
__device__ __forceinline__ float max_abs(float r, float x) {
  float o;
  asm("v_max_f32 %0, %1, |%2|" : "=v"(o) : "v"(r), "v"(x));
  return o;
}
template <typename R, class PK = NoPark>
__device__ __forceinline__ void plane_contact_regs(Drone<R>& s, const R Rm[9], const Consts<R>& c, const DynK<R>& k,
                                                   const PK& pk = PK(), bool skip = false) {
#ifdef GPD_CONTACT_STATS
  const unsigned long long t_setup = __builtin_readcyclecounter();
#endif
  const R zc = (-Rm[8] < R(0) ? -c.cyl_hh : c.cyl_hh) + c.cyl_zoff;
  const R cr = c.cyl_r;
  // world inverse inertia I_w^-1 = R diag(1/I) R^T (symmetric)
  const R q00 = k.ijx * Rm[0], q01 = k.ijy * Rm[1], q02 = k.ijz * Rm[2];
  const R q10 = k.ijx * Rm[3], q11 = k.ijy * Rm[4], q12 = k.ijz * Rm[5];
  const R q20 = k.ijx * Rm[6], q21 = k.ijy * Rm[7], q22 = k.ijz * Rm[8];
  const R i00 = pc_dot(q00, q01, q02, Rm[0], Rm[1], Rm[2]);
  const R i01 = pc_dot(q00, q01, q02, Rm[3], Rm[4], Rm[5]);
  const R i02 = pc_dot(q00, q01, q02, Rm[6], Rm[7], Rm[8]);
  const R i11 = pc_dot(q10, q11, q12, Rm[3], Rm[4], Rm[5]);
  const R i12 = pc_dot(q10, q11, q12, Rm[6], Rm[7], Rm[8]);
  const R i22 = pc_dot(q20, q21, q22, Rm[6], Rm[7], Rm[8]);
  R rwx[4], rwy[4], rwz[4];              // world arms of the rim points
  R g[4][3][3];                          // I_w^-1 (r x d) per point and row
  R rhs[4][3], jdi[4][3], jdn[4], lam[4][3];
  const R idt = g_rcp(k.dt);
  bool act[4];
  bool any = false;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const R rx = p == 0 ? cr : (p == 2 ? -cr : R(0)), ry = p == 1 ? cr : (p == 3 ? -cr : R(0));
    rwx[p] = pc_dot(Rm[0], Rm[1], Rm[2], rx, ry, zc);
    rwy[p] = pc_dot(Rm[3], Rm[4], Rm[5], rx, ry, zc);
    rwz[p] = pc_dot(Rm[6], Rm[7], Rm[8], rx, ry, zc);
    const R dist = s.pz + rwz[p];
    act[p] = !skip && dist < c.brk && g_abs(s.px + rwx[p]) <= c.plane_half && g_abs(s.py + rwy[p]) <= c.plane_half;
    any = any || act[p];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      // world angular Jacobian a = r x d:  +z: (ry, -rx, 0);  (0,-1,0): (rz, 0, -rx);  (1,0,0): (0, rz, -ry)
      const R ax = j == 0 ? rwy[p] : (j == 1 ? rwz[p] : R(0));
      const R ay = j == 0 ? -rwx[p] : (j == 1 ? R(0) : rwz[p]);
      const R az = j == 0 ? R(0) : (j == 1 ? -rwx[p] : -rwy[p]);
      const R gx = pc_dot(i00, i01, i02, ax, ay, az);
      const R gy = pc_dot(i01, i11, i12, ax, ay, az);
      const R gz = pc_dot(i02, i12, i22, ax, ay, az);
      g[p][j][0] = gx; g[p][j][1] = gy; g[p][j][2] = gz;
      const R jd = k.inv_m + pc_dot(ax, ay, az, gx, gy, gz);
      // 1/jd and x/dt as Newton-refined reciprocals (jd >= 1/m > 0): ~1 ulp from the quotients,
      // a third of an f64 divide's instructions on the setup of every solve
      const R inv = g_rcp(jd);
      const R vl = j == 0 ? s.vz : (j == 1 ? -s.vy : s.vx);
      const R rel = vl + pc_dot(ax, ay, az, s.wx, s.wy, s.wz);
      R r;
      if (j == 0) {
        const R pen = dist + c.slop;
        r = pen > R(0) ? (-rel - pen * idt) * inv : (-pen * c.erp * idt - rel) * inv;
        jdn[p] = act[p] ? jd : R(0);
      } else {
        r = -rel * inv;
      }
      jdi[p][j] = act[p] ? inv : R(0);
      rhs[p][j] = act[p] ? r : R(0);
      lam[p][j] = R(0);
    }
  }
  R DLx = R(0), DLy = R(0), DLz = R(0), DAx = R(0), DAy = R(0), DAz = R(0);
  bool done = !any;
  const R mu = c.mu, resid = c.resid, im = k.inv_m;
  const int iters = c.iters;
  // normal rows some lane of the wave touches (a row that only finished lanes need runs with
  // them masked off and changes nothing)
  bool wrow[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) wrow[p] = __ballot(act[p]) != 0ull;
  pk.park();   // from here on only the solve's own values are live in this thread
#ifdef GPD_CONTACT_STATS
  int it_used = 0;
  const unsigned long long nact = __ballot(any);
  const unsigned long long t_loop = __builtin_readcyclecounter();
#endif
  for (int it = 0; it < iters; ++it) {
    if (__ballot(!done) == 0ull) break;
#ifdef GPD_CONTACT_STATS
    it_used = it + 1;
#endif
    if (!done) {
      R res = R(0);
#pragma unroll
      for (int p = 0; p < 4; ++p) {                  // normal rows
        if (!wrow[p]) continue;
        const R jv = DLz + (rwy[p] * DAx - rwx[p] * DAy);
        const R sum = lam[p][0] + (rhs[p][0] - jdi[p][0] * jv);
        const R ln = sum < R(0) ? R(0) : sum;
        const R d = ln - lam[p][0];
        lam[p][0] = ln;
        DLz = DLz + im * d;
        DAx = DAx + g[p][0][0] * d; DAy = DAy + g[p][0][1] * d; DAz = DAz + g[p][0][2] * d;
        res = max_abs(res, d * jdn[p]);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {                  // friction pairs on the cone
        const R lnrm = lam[p][0];
        if (lnrm > R(0)) {
          const R lim = mu * lnrm;
          const R l1 = lam[p][1], l2 = lam[p][2];
          const R j1 = (rwz[p] * DAx - rwx[p] * DAz) - DLy;
          const R j2 = (rwz[p] * DAy - rwy[p] * DAz) + DLx;
          R s1 = l1 + (rhs[p][1] - jdi[p][1] * j1);
          R s2 = l2 + (rhs[p][2] - jdi[p][2] * j2);
          const R m2 = s1 * s1 + s2 * s2;
          if (m2 > lim * lim) {                      // onto the cone: (s1, s2) * lim / |s|
            const R f = lim * g_rsqrt(m2);
            s1 = s1 * f;
            s2 = s2 * f;
          }
          const R d1 = s1 - l1, d2 = s2 - l2;
          lam[p][1] = s1;
          lam[p][2] = s2;
          DLy = DLy - im * d1;
          DLx = DLx + im * d2;
          DAx = DAx + g[p][1][0] * d1; DAy = DAy + g[p][1][1] * d1; DAz = DAz + g[p][1][2] * d1;
          DAx = DAx + g[p][2][0] * d2; DAy = DAy + g[p][2][1] * d2; DAz = DAz + g[p][2][2] * d2;
          res = max_abs(res, d1 + d2);
        }
      }
      done = res * res <= resid;
    }
  }
  pk.unpark();
#ifdef GPD_CONTACT_STATS
  const unsigned long long t_end = __builtin_readcyclecounter();
  if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
    atomicAdd(&g_pc_hist[it_used], 1ull);
    atomicAdd(&g_pc_hist[51 + __popcll(nact)], 1ull);
    atomicAdd(&g_pc_hist[120], t_loop - t_setup);   // setup cycles (s_memtime)
    atomicAdd(&g_pc_hist[121], t_end - t_loop);     // iteration-loop cycles (incl. the unpark)
    atomicAdd(&g_pc_hist[122], (unsigned long long)it_used);
    if (blockIdx.x < 4096) atomicAdd(&g_pc_hist[256 + 8192 + blockIdx.x], t_end - t_setup);
  }
#endif
  s.vx = any ? s.vx + DLx : s.vx;
  s.vy = any ? s.vy + DLy : s.vy;
  s.vz = any ? s.vz + DLz : s.vz;
  s.wx = any ? s.wx + DAx : s.wx;
  s.wy = any ? s.wy + DAy : s.wy;
  s.wz = any ? s.wz + DAz : s.wz;
}

// Lowest height of the contact candidates (the cap facing down, rim at 0/90/180/270 deg): the
// wave gate of plane_contact.
template <typename R>
__device__ __forceinline__ R contact_low(const Drone<R>& s, const R Rm[9], const Consts<R>& c) {
  const R zc = (-Rm[8] < R(0) ? -c.cyl_hh : c.cyl_hh) + c.cyl_zoff;
  const R h = g_abs(Rm[6]) > g_abs(Rm[7]) ? g_abs(Rm[6]) : g_abs(Rm[7]);
  return (s.pz + Rm[8] * zc) - c.cyl_r * h;
}

// ---------------------------------------------------------------- one Bullet (PYB*) substep
// Physics.PYB* (SURVEY.md §8 f3): the forces of _physics / _groundEffect / _drag / _downwash
// (BaseAviary.py:679-811) on the links of the URDF multibody, then ONE p.stepSimulation()
// (:369-370) of a free btMultiBody base without contacts, restated from Bullet3 (oracle:
// oracle/bullet_mb.py, which follows computeAccelerationsArticulatedBodyAlgorithmMultiDof /
// applyDeltaVeeMultiDof / stepPositionsMultiDof step by step).  Evaluated here in the
// world-frame form that the base-frame spatial algebra reduces to (the m w x v bias terms cancel
// and I^-1 I w = w; tests/test_oracle_bullet.py checks the two forms against each other):
//   w_b   = R^T w                                     (R = basis of the stored orientation)
//   wdot  = R J^-1 (tau - w_b x J w_b) - k_a (1 + |w|) w
//   vdot  = (R (0,0,T) [+ drag] - (0,0,M G)) / M - k_l (1 + |v|) v
//   w, v += dt * (wdot, vdot), each coordinate clamped to +-max_vel; p += dt * v
//   q_s'  = normalise((a, cos(f dt/2)) (x) q_s),  a = w sin(f dt/2)/f,  f = min(|w|, pi/4 / dt)
// with q_s = m_baseQuat^-1 (body -> world, what the readback round-trips).  The state's
// rpy_rates slots hold the world angular velocity (m_realBuf[0:3]); ang_v is its readback copy.
// The exponential map's half angle is clamped at pi/8 < 0.5, so the cos / sinc series always
// applies (a select, no branch; below Bullet's f < 0.001 Taylor switch the series agrees with
// Bullet's two-term expansion to ~1e-30).
// rpm / W / last / k are the caller's loop-carried values: a contact solve parks them in LDS and
// hands back the reloaded copies (see the contact block below).
// HK: the drone <-> drone contact of multi-drone envs (gpd_kernels.h DcHook), run on the
// unconstrained velocities before the ground-plane solve; NoDc elsewhere.
struct NoDc {
  template <typename R, class PK>
  __device__ bool operator()(Drone<R>&, R*, const Consts<R>&, const DynK<R>&, const PK&, bool) const { return false; }
};
template <typename R, int PF, bool ANGV, int CW = 1, class HK = NoDc>
__device__ __forceinline__ void bullet_substep(Drone<R>& s, R rpm[4], R W[4], R last[4], R dwsum,
                                               R q0[4], R d, const Consts<R>& c, DynK<R>& k, const HK& hk = HK()) {
  R inv, Rm[9];
  readback_unit<R, true, false>(q0[0], q0[1], q0[2], q0[3], d, inv, Rm);
  bool up = true;
  if (pf_on<PF>(k.flags, F_GND)) {   // |self.rpy[0,1]| < pi/2, :742
    const R qn[4] = {q0[0] * inv, q0[1] * inv, q0[2] * inv, q0[3] * inv};
    AttitudeArgs<R> t = attitude_args(qn);
    bool tilt_unused;
    attitude_decide<R, false, true>(s.qx, s.qy, s.qz, s.qw, t, tilt_unused, up);
  }
  R fz, tx, ty, tz;
  body_wrench<R, PF>(s, Rm, up, rpm, W, c, k, fz, tx, ty, tz);
  if (pf_on<PF>(k.flags, F_DW)) fz = fz + dwsum;
  // angular: base-frame rate, gyroscopic term, damping on the world rate
  const R wbx = (Rm[0] * s.wx + Rm[3] * s.wy) + Rm[6] * s.wz;
  const R wby = (Rm[1] * s.wx + Rm[4] * s.wy) + Rm[7] * s.wz;
  const R wbz = (Rm[2] * s.wx + Rm[5] * s.wy) + Rm[8] * s.wz;
  const R jwx = k.jx * wbx, jwy = k.jy * wby, jwz = k.jz * wbz;
  const R bx = k.ijx * (tx - (wby * jwz - wbz * jwy));
  const R by = k.ijy * (ty - (wbz * jwx - wbx * jwz));
  const R bz = k.ijz * (tz - (wbx * jwy - wby * jwx));
  const R kw = c.ang_damp + c.ang_damp * g_sqrt(s.wx * s.wx + s.wy * s.wy + s.wz * s.wz);
  const R dwx = ((Rm[0] * bx + Rm[1] * by) + Rm[2] * bz) - kw * s.wx;
  const R dwy = ((Rm[3] * bx + Rm[4] * by) + Rm[5] * bz) - kw * s.wy;
  const R dwz = ((Rm[6] * bx + Rm[7] * by) + Rm[8] * bz) - kw * s.wz;
  const R mv = c.max_vel;
  auto clampv = [mv](R x) { return x > mv ? mv : (x < -mv ? -mv : x); };
  s.wx = clampv(s.wx + k.dt * dwx);
  s.wy = clampv(s.wy + k.dt * dwy);
  s.wz = clampv(s.wz + k.dt * dwz);
  // linear
  R Fx = Rm[2] * fz, Fy = Rm[5] * fz, Fz = Rm[8] * fz;
  if (pf_on<PF>(k.flags, F_DRAG)) {   // _drag :773-781 with last_clipped_action, world force drag_factors * vel
    const R S = ((last[0] * c.rpm2rad + last[1] * c.rpm2rad) + last[2] * c.rpm2rad) + last[3] * c.rpm2rad;
    Fx = Fx + (-c.drag_xy * S) * s.vx;
    Fy = Fy + (-c.drag_xy * S) * s.vy;
    Fz = Fz + (-c.drag_z * S) * s.vz;
  }
  Fz = Fz - k.gravity;
  const R kv = c.lin_damp + c.lin_damp * g_sqrt(s.vx * s.vx + s.vy * s.vy + s.vz * s.vz);
  s.vx = clampv(s.vx + k.dt * (Fx * k.inv_m - kv * s.vx));
  s.vy = clampv(s.vy + k.dt * (Fy * k.inv_m - kv * s.vy));
  s.vz = clampv(s.vz + k.dt * (Fz * k.inv_m - kv * s.vz));
  // Everything this thread keeps across a contact solve (the caller's constants, RPMs and wrench,
  // the pose and velocities; for the drone <-> drone call also the basis) goes to per-lane LDS
  // columns for the solve and comes back after it: the solve's ~200 VGPRs then fit beside the
  // kernel's own state instead of spilling the row constants into AGPR round trips on the
  // Gauss-Seidel chain, and across the drone <-> drone call nothing of the substep loop is live,
  // so the loop's register allocation does not see it.  The reload goes through an opaque lane
  // offset, so nothing forwards the stored values past the solve; a memory clobber keeps the
  // stores ahead of it.
  // (the basis columns only where the drone <-> drone hook parks it: single-drone kernels keep
  // the 43 columns of the plane solve)
  constexpr bool kDcPark = !std::is_same<HK, NoDc>::value;
  constexpr int kPark = 15 + 12 + 4 + 12, kParkRm = kDcPark ? 9 : 0;
  __shared__ R pk[kPark + kParkRm][kWaveLanes];
  const int pl = threadIdx.x & (kWaveLanes - 1);
  auto each = [&](auto&& f) {
    f(k.dt); f(k.inv_m); f(k.gravity); f(k.jx); f(k.jy); f(k.jz); f(k.ijx); f(k.ijy); f(k.ijz);
    f(k.hdt); f(k.hdt2); f(k.kf); f(k.km); f(k.L); f(k.Ls2);
    f(s.px); f(s.py); f(s.pz); f(s.vx); f(s.vy); f(s.vz); f(s.wx); f(s.wy); f(s.wz);
    f(s.ax); f(s.ay); f(s.az);
#pragma unroll
    for (int j = 0; j < 4; ++j) f(q0[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) { f(rpm[j]); f(W[j]); f(last[j]); }
  };
  auto park = [&]() {
    int i = 0;
    each([&](R& x) { pk[i++][pl] = x; });
    asm volatile("" ::: "memory");
  };
  auto unpark = [&]() {
    int o = pl;
    asm volatile("" : "+v"(o));
    int i = 0;
    each([&](R& x) { x = pk[i++][o]; });
  };
  auto park_dc = [&]() {
    park();
#pragma unroll
    for (int j = 0; j < kParkRm; ++j) pk[kPark + j][pl] = Rm[j];
    asm volatile("" ::: "memory");
  };
  auto unpark_dc = [&]() {
    unpark();
    int o = pl;
    asm volatile("" : "+v"(o));
#pragma unroll
    for (int j = 0; j < kParkRm; ++j) Rm[j] = pk[kPark + j][o];
  };
  // island: this drone's plane rows were solved with its pair contacts (the hook's island solve)
  bool island = false;
  if (!pf_on<PF>(k.flags, F_NO_DC)) {
    // the run-time-flag kernels (a long observation tile may leave no LDS for the parked columns)
    // call the solve without parking
    const bool plane = !pf_on<PF>(k.flags, F_NO_PLANE);
    if (PF != kPfRuntime) island = hk(s, Rm, c, k, ParkFns<decltype(park_dc), decltype(unpark_dc)>{park_dc, unpark_dc}, plane);
    else island = hk(s, Rm, c, k, NoPark(), plane);
  }
  // ground-plane contact (solveConstraints, before integrateTransforms); the margin keeps the
  // gate conservative against the candidates' own rounding
  if (!pf_on<PF>(k.flags, F_NO_PLANE)) {
    const bool low = contact_low(s, Rm, c) < c.brk + R(1e-6) && !island;
    if (CW == 1) {
      // compiled-in PYB flag sets: the register-resident solve; run-time flags (every other
      // combination, whose kernels also serve non-contact configs) keep the LDS rows
      if (GPD_RARE(__ballot(low) != 0ull)) {
        if (PF != kPfRuntime) {
#if GPD_CONTACT_PARK
          plane_contact_regs<R>(s, Rm, c, k, ParkFns<decltype(park), decltype(unpark)>{park, unpark}, island);
#else
          plane_contact_regs<R>(s, Rm, c, k, NoPark(), island);
#endif
        } else {
          plane_contact<R>(s, Rm, c, k, island);
        }
      }
    } else {
      // multi-wave workgroups (envs of more than 64 drones, step_kernel_wide): the LDS rows hold
      // one wave's lanes, so the waves take turns (the whole workgroup runs this code)
      const int wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
      for (int w = 0; w < nw; ++w) {
        if (wv == w && __ballot(low) != 0ull) plane_contact<R>(s, Rm, c, k);
        __syncthreads();
      }
    }
  }
  s.px = s.px + k.dt * s.vx;
  s.py = s.py + k.dt * s.vy;
  s.pz = s.pz + k.dt * s.vz;
  // orientation: exponential map with the new world rate, clamped half angle
  const R t2 = (s.wx * s.wx + s.wy * s.wy + s.wz * s.wz) * k.hdt2;
  const bool clamp = t2 > c.ang_thr2;
  R co, sc;
  cos_sinc(clamp ? c.ang_thr2 : t2, co, sc);
  // axis = w sin(f dt/2)/f = w (dt/2) sinc(f dt/2), f clamped or not
  const R sh = k.hdt * sc;
  const R ax = s.wx * sh, ay = s.wy * sh, az = s.wz * sh;
  const R x = q0[0], y = q0[1], z = q0[2], w = q0[3];
  const R nx = ((co * x + ax * w) + ay * z) - az * y;
  const R ny = ((co * y + ay * w) + az * x) - ax * z;
  const R nz = ((co * z + az * w) + ax * y) - ay * x;
  const R nw = ((co * w - ax * x) - ay * y) - az * z;
  const R rn = g_rsqrt(nx * nx + ny * ny + nz * nz + nw * nw);   // btQuaternion::normalize
  s.qx = nx * rn; s.qy = ny * rn; s.qz = nz * rn; s.qw = nw * rn;
  if (ANGV) { s.ax = s.wx; s.ay = s.wy; s.az = s.wz; }   // getBaseVelocity: world rate
}

// ---------------------------------------------------------------- one DYN substep
// The readback that precedes the substep (BaseAviary.py:346-347 -> :517, :836) followed by
// BaseAviary._dynamics (:815-874) + _integrateQ (:876-889), evaluated on the readback
// snapshot (pos/vel from the client copy, qn = re-normalised orientation, rpy = its Euler
// angles, of which the ground effect only needs |roll|,|pitch| < pi/2 -> upright), optionally
// with the aero force terms of _groundEffect/_drag/_downwash added as a body wrench (see
// DESIGN.md §2 "new combination").
//   rpm  : this ctrl step's clipped action (current substep); W its propeller wrench
//   last : self.last_clipped_action (previous ctrl step's rpm on the first substep)
//   dwsum: summed downwash force along body z (already reduced over the env's drones)
// ANGV: also update the world-frame ang_v (write-only for the dynamics: only the value after the
// last substep of a control step is ever observed, so earlier substeps skip it).
// Schedule: the common path is ONE basic block.  With FAST (no aero terms) the torques do not
// depend on the attitude, so the rotation chain (omega, theta^2, the cos/sinc series) is
// written before the readback and the two dependency chains interleave.  Lanes with
// |theta| >= 0.5 (|omega| >= 240 rad/s at 240 Hz: library sin/cos) are redone in a
// wave-uniform branch at the end.
template <typename R, int PF, bool ANGV = true, int CW = 1, class HK = NoDc>
__device__ __forceinline__ void dyn_substep(Drone<R>& s, R rpm[4], R W[4], R last[4], R dwsum,
                                            const Consts<R>& c, DynK<R>& k, const HK& hk = HK()) {
  R q0[4] = {s.qx, s.qy, s.qz, s.qw};
  R d = q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3];
  // |q| = 1 +- eps for every quaternion _integrateQ produces from a unit one (its update matrix
  // is orthogonal); a lane that is not (a state set from outside, a NaN) is re-normalised here
  // in a wave-uniform branch that the substeps of a normal batch never take
  {
    const bool unit = g_abs(d - R(1)) < UnitTol<R>::v;
    if (GPD_RARE(__ballot(!unit) != 0ull)) {
      if (!unit) {
        const R r = g_rsqrt(d);
#pragma unroll
        for (int i = 0; i < 4; ++i) q0[i] = q0[i] * r;
        d = q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3];
      }
    }
  }
  if (pf_on<PF>(k.flags, F_BULLET)) {
    bullet_substep<R, PF, ANGV, CW, HK>(s, rpm, W, last, dwsum, q0, d, c, k, hk);
    return;
  }
  R inv, Rm[9];
  bool up = true;
  // the torques depend on the pose only through the ground effect (downwash and drag are forces):
  // without it the rotation chain goes ahead of the readback, as on the plain path
  constexpr bool kPoseFirst = PF == kPfRuntime || (PF & F_GND) != 0;
  auto readback = [&]() {
    readback_unit<R, ANGV || kPoseFirst, false>(q0[0], q0[1], q0[2], q0[3], d, inv, Rm);
    if (pf_on<PF>(k.flags, F_GND)) {   // |self.rpy[0,1]| < pi/2, :742
      const R qn[4] = {q0[0] * inv, q0[1] * inv, q0[2] * inv, q0[3] * inv};
      AttitudeArgs<R> t = attitude_args(qn);
      bool tilt_unused;
      attitude_decide<R, false, true>(s.qx, s.qy, s.qz, s.qw, t, tilt_unused, up);
    }
  };
  if (kPoseFirst) readback();
  R fz, tx, ty, tz;
  body_wrench<R, PF>(s, Rm, up, rpm, W, c, k, fz, tx, ty, tz);
  if (pf_on<PF>(k.flags, F_DW)) fz = fz + dwsum;      // _downwash :801-811 (body z)
  // torques - ω × (Jω); ω̇ = J⁻¹ τ                     :852-854
  const R jwx = k.jx * s.wx, jwy = k.jy * s.wy, jwz = k.jz * s.wz;
  const R cx = s.wy * jwz - s.wz * jwy;
  const R cy = s.wz * jwx - s.wx * jwz;
  const R cz = s.wx * jwy - s.wy * jwx;
  const R dwx = k.ijx * (tx - cx), dwy = k.ijy * (ty - cy), dwz = k.ijz * (tz - cz);
  s.wx = s.wx + k.dt * dwx;                            // :856
  s.wy = s.wy + k.dt * dwy;
  s.wz = s.wz + k.dt * dwz;
  // _integrateQ(quat, rpy_rates, dt)                  :876-889
  const R p = s.wx, q = s.wy, r = s.wz;
  const R n2 = p * p + q * q + r * r;
  // np.isclose(|omega|, 0) <=> |omega| <= 1e-8 <=> |omega|^2 <= 1e-16 (the two tests can only
  // disagree when |omega| lies within an ulp of 1e-8; numpy's BLAS norm itself rounds there)
  const bool rot = n2 > R(1e-16);
  // q' = (I cos(theta) + (2/|omega|) Lambda sin(theta)) q, theta = |omega| dt/2: the off-diagonal
  // weights (2/|omega|)(p/2) sin(theta) = p * (dt/2) * sin(theta)/theta.  Evaluated for every
  // lane and selected (no branch); the library sin/cos for |theta| >= 0.5 (|omega| >= 240 rad/s
  // at 240 Hz) is part of the rare-lane fix-up.
  const R t2 = n2 * k.hdt2;                            // theta^2
  R co, sc;                                            // cos(theta), sin(theta)/theta
  cos_sinc(t2, co, sc);
  const R sh = k.hdt * sc;                             // sin(theta)/|omega|
  const bool big = t2 >= R(0.25);
  if (!kPoseFirst) readback();
  // R·(0,0,fz) - (0,0,GRAVITY) [+ drag]                 :839-841
  R Fx = Rm[2] * fz, Fy = Rm[5] * fz, Fz = Rm[8] * fz;
  if (pf_on<PF>(k.flags, F_DRAG)) {                   // _drag :773-774 with last_clipped_action
    const R S = ((last[0] * c.rpm2rad + last[1] * c.rpm2rad) + last[2] * c.rpm2rad) + last[3] * c.rpm2rad;
    Fx = Fx + (-c.drag_xy * S) * s.vx;
    Fy = Fy + (-c.drag_xy * S) * s.vy;
    Fz = Fz + (-c.drag_z * S) * s.vz;
  }
  Fz = Fz - k.gravity;
  // semi-implicit Euler                                :855-859
  s.vx = s.vx + k.dt * (Fx * k.inv_m);
  s.vy = s.vy + k.dt * (Fy * k.inv_m);
  s.vz = s.vz + k.dt * (Fz * k.inv_m);
  s.px = s.px + k.dt * s.vx;
  s.py = s.py + k.dt * s.vy;
  s.pz = s.pz + k.dt * s.vz;
  // q' = M(omega) (inv q0) = M'(omega) q0 with the readback's 1/|q| folded into M's entries;
  // below the isclose threshold P = Q = R = 0 and co = 1 exactly (t2 <= 1e-16), so q' = inv q0,
  // the readback quaternion itself (up to Bullet's sign, see readback_unit), as the reference's
  // skip leaves it
  auto update = [&](R co_, R sh_) {
    const R shi = sh_ * inv;
    const R P = rot ? p * shi : R(0), Q = rot ? q * shi : R(0), Rr = rot ? r * shi : R(0);
    const R C = co_ * inv;
    const R x = q0[0], y = q0[1], z = q0[2], w = q0[3];
    s.qx = ((C * x + Rr * y) - Q * z) + P * w;
    s.qy = ((-Rr * x + C * y) + P * z) + Q * w;
    s.qz = ((Q * x - P * y) + C * z) + Rr * w;
    s.qw = ((-P * x - Q * y) - Rr * z) + C * w;
  };
  update(co, sh);
  // resetBaseVelocity(..., np.dot(rotation, rpy_rates))  :868-872
  if (ANGV) {
    s.ax = (Rm[0] * s.wx + Rm[1] * s.wy) + Rm[2] * s.wz;
    s.ay = (Rm[3] * s.wx + Rm[4] * s.wy) + Rm[5] * s.wz;
    s.az = (Rm[6] * s.wx + Rm[7] * s.wy) + Rm[8] * s.wz;
  }
  // keep the translation in the main block (it fills the latency of the rotation chain)
  asm volatile("" ::"v"(s.px), "v"(s.py), "v"(s.pz));
  if (GPD_RARE(__ballot(big) != 0ull)) {
    if (big) {
      const CoSh<R> cs = cold_cos_sinc(n2, k.hdt);
      update(cs.co, cs.sh);
    }
  }
}

// ---------------------------------------------------------------- FAST substep, split in two
// Without aero terms the body torques are the propeller wrench alone, so dyn_substep<R, true>
// falls into two dependency chains that meet once per substep: the body-rate chain (ω and the
// _integrateQ weights) reads nothing of the pose, and the pose chain (readback, v, p, q) needs
// only the rate chain's weights for its quaternion update.  step_kernel_duo runs them on two
// waves.  The operations and their order are dyn_substep's; results agree to rounding (hipcc
// contracts a few multiply-adds differently in the two code shapes: 1 ulp in f64).
//
// Rate half: ω' = ω + dt J⁻¹(τ − ω×Jω) (:852-856) and the weights of _integrateQ(q, ω', dt)
// (:876-889): h = {cos θ, sin θ/|ω'|, p, q, r} with (p, q, r) = ω' above the np.isclose threshold
// and 0 below it (then cos θ = 1 exactly: the pose half's update returns q/|q|).
template <typename R>
__device__ __forceinline__ void rate_half(R& wx, R& wy, R& wz, const R W[4], const DynK<R>& k, R h[5]) {
  const R jwx = k.jx * wx, jwy = k.jy * wy, jwz = k.jz * wz;
  const R cx = wy * jwz - wz * jwy;
  const R cy = wz * jwx - wx * jwz;
  const R cz = wx * jwy - wy * jwx;
  const R dwx = k.ijx * (W[1] - cx), dwy = k.ijy * (W[2] - cy), dwz = k.ijz * (W[3] - cz);
  wx = wx + k.dt * dwx;
  wy = wy + k.dt * dwy;
  wz = wz + k.dt * dwz;
  const R n2 = wx * wx + wy * wy + wz * wz;
  const bool rot = n2 > R(1e-16);
  const R t2 = n2 * k.hdt2;
  R co, sc;
  cos_sinc(t2, co, sc);
  R sh = k.hdt * sc;
  const bool big = t2 >= R(0.25);
  if (GPD_RARE(__ballot(big) != 0ull)) {
    if (big) {
      const CoSh<R> cs = cold_cos_sinc(n2, k.hdt);
      co = cs.co;
      sh = cs.sh;
    }
  }
  h[0] = co; h[1] = sh;
  h[2] = rot ? wx : R(0); h[3] = rot ? wy : R(0); h[4] = rot ? wz : R(0);
}

// Pose half: the readback of q (1/|q| and the thrust direction; with ANGV all nine entries for
// the world-frame ang_v of the rates w = ω'), semi-implicit Euler of v and p (:839-841,
// :855-859) and q' = M(ω') q/|q| from the rate half's weights h.
// CHECK: the |q|^2 ~ 1 test of dyn_substep (re-normalising a quaternion set from outside).  Only
// the first substep of a step needs it: from a quaternion with |d - 1| < UnitTol the update
// M(ω') q/|q| is orthogonal to rounding, so every later substep starts within a few ulp of 1.
template <typename R, bool ANGV, bool CHECK>
__device__ __forceinline__ void pose_half(Drone<R>& s, R fz, const R h[5], const R w[3], const DynK<R>& k) {
  R q0[4] = {s.qx, s.qy, s.qz, s.qw};
  R d = q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3];
  if (CHECK) {
    const bool unit = g_abs(d - R(1)) < UnitTol<R>::v;   // as in dyn_substep
    if (GPD_RARE(__ballot(!unit) != 0ull)) {
      if (!unit) {
        const R r = g_rsqrt(d);
#pragma unroll
        for (int i = 0; i < 4; ++i) q0[i] = q0[i] * r;
        d = q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3];
      }
    }
  }
  R inv, Rm[9];
  readback_unit<R, ANGV, false>(q0[0], q0[1], q0[2], q0[3], d, inv, Rm);
  R Fx = Rm[2] * fz, Fy = Rm[5] * fz, Fz = Rm[8] * fz;
  Fz = Fz - k.gravity;
  s.vx = s.vx + k.dt * (Fx * k.inv_m);
  s.vy = s.vy + k.dt * (Fy * k.inv_m);
  s.vz = s.vz + k.dt * (Fz * k.inv_m);
  s.px = s.px + k.dt * s.vx;
  s.py = s.py + k.dt * s.vy;
  s.pz = s.pz + k.dt * s.vz;
  const R shi = h[1] * inv;
  const R P = h[2] * shi, Q = h[3] * shi, Rr = h[4] * shi;
  const R C = h[0] * inv;
  const R x = q0[0], y = q0[1], z = q0[2], ww = q0[3];
  s.qx = ((C * x + Rr * y) - Q * z) + P * ww;
  s.qy = ((-Rr * x + C * y) + P * z) + Q * ww;
  s.qz = ((Q * x - P * y) + C * z) + Rr * ww;
  s.qw = ((-P * x - Q * y) - Rr * z) + C * ww;
  if (ANGV) {
    s.ax = (Rm[0] * w[0] + Rm[1] * w[1]) + Rm[2] * w[2];
    s.ay = (Rm[3] * w[0] + Rm[4] * w[1]) + Rm[5] * w[2];
    s.az = (Rm[6] * w[0] + Rm[7] * w[1]) + Rm[8] * w[2];
  }
}

// Summed downwash on drone (px,py,pz) from the env's D drones whose positions sit in LDS
// (BaseAviary._downwash :798-811).  A wave-wide ballot skips the α/β/exp block whenever no
// lane of the wave has an active pair (Δz > 0 ∧ Δxy < 10) for neighbour j.
// The downwash force on drone (px,py,pz) from drone (qx,qy,qz) (:798-811), 0 when the pair is
// culled (delta_z <= 0 or delta_xy >= 10).  alpha = DW1 (PROP_RADIUS/(4 dz))^2,
// beta = DW2 dz + DW3, f = -alpha exp(-0.5 (dxy/beta)^2); |dxy|^2 needs no square root, and
// beta = 0 keeps numpy's IEEE result (dxy^2/0 = inf -> exp(-inf) = 0; 0/0 = nan at dxy = 0).
// The ballot skips the exp block for a whole wave when no lane has an active pair.
template <typename R> struct DwCull;
template <> struct DwCull<double> { static constexpr double v = 99.999999999999985789145284797996282577514648437500; };
template <> struct DwCull<float> { static constexpr float v = 99.99999237060546875f; };

template <typename R>
__device__ __forceinline__ R dw_pair(R px, R py, R pz, R qx, R qy, R qz, const Consts<R>& c) {
  const R dz = qz - pz;
  const R ddx = qx - px, ddy = qy - py;
  const R dxy2 = ddx * ddx + ddy * ddy;
  // delta_z > 0 and delta_xy < 10 (:801).  sqrt is correctly rounded and monotonic, so
  // sqrt(s) < 10 <=> s < the smallest s' whose sqrt rounds to 10, which is the predecessor of
  // 100 in both double and float: the exact cull without a square root per pair
  const bool hit = (dz > R(0)) && (dxy2 < DwCull<R>::v);
  R f = R(0);
  if (__ballot(hit) != 0ull) {
    if (hit) {
      const R alpha = c.dwk1 / (dz * dz);
      const R beta = c.dw2 * dz + c.dw3;
      f = -alpha * g_exp(R(-0.5) * (dxy2 / (beta * beta)));
    }
  }
  return f;
}

// Summed downwash on one drone from its env's D drones (positions in LDS), neighbours in the
// reference's order j = 0..D-1 (culled pairs add +0, which changes no sum).
template <typename R>
__device__ __forceinline__ R downwash_sum(R px, R py, R pz, const R* sx, const R* sy, const R* sz,
                                          int base, int D, const Consts<R>& c) {
  R total = R(0);
  for (int j = 0; j < D; ++j) total = total + dw_pair(px, py, pz, sx[base + j], sy[base + j], sz[base + j], c);
  return total;
}

}  // namespace gpd
