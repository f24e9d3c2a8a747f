// gpd.hip — C ABI (include/gpd.h) of the batched quadrotor DYN path on MI355X (gfx950).
//
// Host side: validates the configuration (BaseAviary.__init__ checks, BaseAviary.py:79-80),
// derives the model constants in double exactly as BaseAviary.py:117-128 does, builds the
// reset template (INIT_XYZS / INIT_RPYS through the Bullet orientation round trip,
// BaseAviary.py:194-207, :486-491, :509-519), owns the SoA device state and launches the
// kernels of gpd_kernels.h on the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpd.h"
#include "gpd_kernels.h"
#include "gpd_handoff.h"

using namespace gpd;

static_assert(GPD_ACT_RPM == ACT_RPM && GPD_ACT_ONE_D_RPM == ACT_ONE_D_RPM && GPD_ACT_PID == ACT_PID &&
                  GPD_ACT_VEL == ACT_VEL && GPD_ACT_ONE_D_PID == ACT_ONE_D_PID,
              "action type codes of gpd.h and the kernels must agree");
constexpr int kCtrlComps = 9;
constexpr size_t kLdsBytes = 160 * 1024;   // LDS per workgroup on gfx950

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(GPD_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- host restatements of the Bullet helpers (double), for the reset template only
void h_quat_to_mat(const double q[4], double m[9]) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double d = x * x + y * y + z * z + w * w, s = 2.0 / d;
  const double xs = x * s, ys = y * s, zs = z * s;
  const double wx = w * xs, wy = w * ys, wz = w * zs, xx = x * xs, xy = x * ys, xz = x * zs;
  const double yy = y * ys, yz = y * zs, zz = z * zs;
  m[0] = 1.0 - (yy + zz); m[1] = xy - wz; m[2] = xz + wy;
  m[3] = xy + wz; m[4] = 1.0 - (xx + zz); m[5] = yz - wx;
  m[6] = xz - wy; m[7] = yz + wx; m[8] = 1.0 - (xx + yy);
}
void h_mat_to_quat(const double m[9], double q[4]) {
  const double tr = m[0] + m[4] + m[8];
  double t[4];
  if (tr > 0.0) {
    double s = std::sqrt(tr + 1.0);
    t[3] = s * 0.5; s = 0.5 / s;
    t[0] = (m[7] - m[5]) * s; t[1] = (m[2] - m[6]) * s; t[2] = (m[3] - m[1]) * s;
  } else {
    const int i = m[0] < m[4] ? (m[4] < m[8] ? 2 : 1) : (m[0] < m[8] ? 2 : 0);
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    double s = std::sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
    t[i] = s * 0.5; s = 0.5 / s;
    t[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
    t[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
    t[k] = (m[k * 3 + i] + m[i * 3 + k]) * s;
  }
  for (int a = 0; a < 4; ++a) q[a] = t[a];
}
void h_roundtrip(const double q[4], double out[4]) {
  double m[9];
  h_quat_to_mat(q, m);
  h_mat_to_quat(m, out);
}
void h_euler(const double q[4], double rpy[3]) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double sarg = -2.0 * (x * z - w * y);
  if (sarg <= -0.99999) {
    rpy[0] = 0.0; rpy[1] = -0.5 * M_PI; rpy[2] = 2.0 * std::atan2(x, -y);
  } else if (sarg >= 0.99999) {
    rpy[0] = 0.0; rpy[1] = 0.5 * M_PI; rpy[2] = 2.0 * std::atan2(-x, y);
  } else {
    rpy[1] = std::asin(std::fmin(1.0, std::fmax(-1.0, sarg)));
    rpy[0] = std::atan2(2.0 * (y * z + w * x), w * w - x * x - y * y + z * z);
    rpy[2] = std::atan2(2.0 * (x * y + w * z), w * w + x * x - y * y - z * z);
  }
}
void h_quat_from_euler(const double rpy[3], double q[4]) {  // btQuaternion::setEulerZYX
  const double hy = rpy[2] * 0.5, hp = rpy[1] * 0.5, hr = rpy[0] * 0.5;
  const double cy = std::cos(hy), sy = std::sin(hy), cp = std::cos(hp), sp = std::sin(hp);
  const double cr = std::cos(hr), sr = std::sin(hr);
  q[0] = sr * cp * cy - cr * sp * sy;
  q[1] = cr * sp * cy + sr * cp * sy;
  q[2] = cr * cp * sy - sr * sp * cy;
  q[3] = cr * cp * cy + sr * sp * sy;
}

}  // namespace

struct gpd_sim {
  gpd_drone_params P;
  gpd_pid_params pid;
  gpd_config cfg;
  gpd_constants K;
  int E, D, N, A, W, nsub, ring_len, prec, tpb;
  long long npad;
  void* d_state = nullptr;
  void* d_ctrl = nullptr;         // tiled [npad/64][9][64] DSLPIDControl state (PID action types)
  float* d_ring = nullptr;
  int2* d_ctr = nullptr;          // [E] {step_counter, ring head} + [E].x: last action in the ring
  void* d_init = nullptr;
  void* d_target = nullptr;
  void* d_consts = nullptr;       // Consts<real> in device memory
  int tile_bytes = 0;             // dynamic LDS of the step kernel
  int wt = 0;                     // SimView::wt (write-through store policy)
  int nc_magic = 0;               // SimView::nc_magic
  bool duo = false;               // step launches step_kernel_duo (two or three waves per block)
  bool wide = false;              // step_kernel_wide / integrate_kernel_wide, one env per workgroup: D > 64,
                                  // or an observation row too long for the one-wave kernels' LDS tile
  int step_waves = 1;             // waves per step block (1, 2, or 3 with the io wave)
  bool stream = false;            // streaming cache policies (step_kernel STREAM): batches past the MALL
  bool generic_pf = false;        // the run-time-flag step kernel even where a flag set is compiled in
                                  // (its static LDS + the observation tile would not fit: upload_tables)
  DwPairs dw_pairs{0, 0};         // SimView::dw_pairs
  // drone <-> drone contact (PYB*, 1 < D <= 64; SimView::dc*): pairs per env, p / P magic, the
  // [P] pair table, the row store of pairs past a block's first 64 (blocks x stride reals)
  int dcP = 0, dc_pmagic = 0;
  int* d_dc_tab = nullptr;
  void* d_dc_rows = nullptr;
  long long dc_row_stride = 0;
  double bound_xy;
  std::vector<double> init_tmpl;  // [D][10]
  std::vector<double> target;     // [D][3]
};

namespace {

template <typename R>
Consts<R> make_consts(const gpd_sim* s) {
  const gpd_drone_params& P = s->P;
  Consts<R> c;
  c.dt = (R)s->K.pyb_timestep;
  c.hdt = (R)(0.5 * s->K.pyb_timestep);
  c.hdt2 = (R)((0.5 * s->K.pyb_timestep) * (0.5 * s->K.pyb_timestep));
  c.m = (R)P.m;
  c.gravity = (R)s->K.gravity;
  c.kf = (R)P.kf;
  c.km = (R)P.km;
  c.L = (R)P.arm;
  c.Ls2 = (R)(P.arm / std::sqrt(2.0));
  c.jx = (R)P.ixx; c.jy = (R)P.iyy; c.jz = (R)P.izz;
  c.ijx = (R)(1.0 / P.ixx); c.ijy = (R)(1.0 / P.iyy); c.ijz = (R)(1.0 / P.izz);
  c.ge_coeff = (R)P.gnd_eff_coeff;
  c.prop_r = (R)P.prop_radius;
  c.ge_clip = (R)s->K.gnd_eff_h_clip;
  c.drag_xy = (R)P.drag_coeff_xy;
  c.drag_z = (R)P.drag_coeff_z;
  c.two_pi = (R)(2.0 * M_PI);
  c.dw1 = (R)P.dw_coeff_1; c.dw2 = (R)P.dw_coeff_2; c.dw3 = (R)P.dw_coeff_3;
  c.dwk1 = (R)(P.dw_coeff_1 * ((P.prop_radius / 4) * (P.prop_radius / 4)));
  c.inv_m = (R)(1.0 / P.m);
  c.rpm2rad = (R)(2.0 * M_PI / 60.0);
  for (int k = 0; k < 4; ++k) {
    c.rx[k] = (R)P.prop_pos[k][0];
    c.ry[k] = (R)P.prop_pos[k][1];
    c.rz[k] = (R)P.prop_pos[k][2];
  }
  for (int k = 0; k < 10; ++k) c.init0[k] = (R)s->init_tmpl[k];
  for (int k = 0; k < 3; ++k) c.target0[k] = (R)s->target[k];
  c.hover_f32 = (float)s->K.hover_rpm;
  c.model = P.model;
  // the Bullet integrator always places the thrust at the prop links (_physics :698-705)
  c.flags = s->cfg.physics_flags | ((s->cfg.physics_flags & GPD_F_BULLET) ? GPD_F_GEOM_WRENCH : 0);
  c.lin_damp = (R)0.04;      // btMultiBody() m_linearDamping (not removed: BaseAviary.py:492-494)
  c.ang_damp = (R)0.04;      // btMultiBody() m_angularDamping
  c.max_vel = (R)100.0;      // btMultiBody() m_maxCoordinateVelocity
  c.ang_thr2 = (R)((0.125 * M_PI) * (0.125 * M_PI));   // (ANGULAR_MOTION_THRESHOLD / 2)^2
  // ground-plane contact (plane_contact; constants restated in oracle/bullet_mb.py)
  c.cyl_r = (R)P.collision_r;
  c.cyl_hh = (R)(P.collision_h / 2);
  c.cyl_zoff = (R)P.collision_z_offset;
  {
    const double r = P.collision_r + 0.001, h = P.collision_h / 2 + 0.001;   // + URDF shape margin
    c.brk = (R)(0.02 * std::sqrt(r * r + r * r + h * h));                   // 0.02 x motion disc
  }
  c.slop = (R)1e-5;          // m_linearSlop (pybullet)
  c.erp = (R)0.08;           // m_erp2 (pybullet contactERP)
  c.mu = (R)(0.5 * 1.0);     // drone default friction x plane.urdf lateral_friction
  c.plane_half = (R)15.0;    // plane.urdf collision box 30 x 30
  c.resid = (R)1e-7;         // m_leastSquaresResidualThreshold (pybullet)
  {
    // drone <-> drone contact (drone_contact, gpd_kernels.h; oracle/bullet_mb.py drone_contact)
    const double bs = std::sqrt(P.collision_r * P.collision_r + (P.collision_h / 2) * (P.collision_h / 2));
    const double reach = 2.0 * bs + (double)c.brk;
    c.dd_reach2 = (R)(reach * reach);
    c.dd_mu = (R)(0.5 * 0.5);   // drone x drone default friction
  }
  c.iters = 50;              // m_numIterations (pybullet numSolverIterations)
  // setPhysicsEngineParameter(numSolverIterations=, solverResidualThreshold=) (gpd_config)
  if (s->cfg.solver_iterations > 0) c.iters = s->cfg.solver_iterations;
  if (s->cfg.solver_residual != 0.0) c.resid = (R)s->cfg.solver_residual;
#ifdef GPD_DIAG_RESID
  c.resid = (R)GPD_DIAG_RESID;   // diagnostic builds only (e.g. -1: every solve runs c.iters iterations)
#endif
  c.nsub = s->nsub;
  const gpd_pid_params& Q = s->pid;
  PidConsts<R>& k = c.pid;
  for (int i = 0; i < 3; ++i) {
    k.p_for[i] = (R)Q.p_coeff_for[i]; k.i_for[i] = (R)Q.i_coeff_for[i]; k.d_for[i] = (R)Q.d_coeff_for[i];
    k.p_tor[i] = (R)Q.p_coeff_tor[i]; k.i_tor[i] = (R)Q.i_coeff_tor[i]; k.d_tor[i] = (R)Q.d_coeff_tor[i];
  }
  k.pwm2rpm_scale = (R)Q.pwm2rpm_scale; k.pwm2rpm_const = (R)Q.pwm2rpm_const;
  k.min_pwm = (R)Q.min_pwm; k.max_pwm = (R)Q.max_pwm;
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 3; ++i) k.mixer[j * 3 + i] = (R)Q.mixer[j][i];
  k.gravity = (R)Q.gravity; k.kf = (R)Q.kf;
  k.ctrl_dt = (R)s->K.ctrl_timestep;
  k.speed_limit = 0.03 * P.max_speed_kmh * (1000.0 / 3600.0);
  return c;
}

template <typename R>
SimView<R> make_view(const gpd_sim* s) {
  SimView<R> v;
  v.state = (R*)s->d_state;
  v.ctrl = (R*)s->d_ctrl;
  v.ring = s->d_ring;
  v.ctr = s->d_ctr;
  v.init = (const R*)s->d_init;
  v.target = (const R*)s->d_target;
  v.npad = s->npad;
  v.N = s->N; v.D = s->D; v.A = s->A; v.W = s->W; v.tpb = s->tpb; v.ring_len = s->ring_len;
  v.task = s->cfg.task;
  v.autoreset = s->cfg.autoreset;
  v.trunc_sc = s->K.trunc_step_counter;
  v.wt = s->wt;
  v.nc_magic = s->nc_magic;
  v.dw_pairs = s->dw_pairs;
  v.bound_xy = (R)s->bound_xy;
  v.dcP = s->dcP;
  v.dc_pmagic = s->dc_pmagic;
  v.dc_tab = s->d_dc_tab;
  v.dc_rows = s->d_dc_rows;
  v.dc_row_stride = s->dc_row_stride;
  return v;
}

// The step_kernel instantiation of a sim: action type x (D > 1) x (plain DYN fast path).  The
// fast specialisation exists for the RPM action types only (the bench path).
// Physics-flag sets compiled into their own kernels (pf_on): the BASELINE configs' combinations
// (config 3: ground effect + drag; config 4: downwash) and Physics.PYB / PYB_GND_DRAG_DW (single-
// and multi-drone envs) for the RPM action types, plain DYN and Physics.PYB for the single-drone
// PID types; every other combination tests Consts::flags at run time.  The PYB flag sets run the
// register-resident contact solve (gpd_device.h plane_contact_regs), the run-time kernels the
// LDS one.
constexpr int kPfAero = F_GND | F_DRAG;
constexpr int kPfPyb = F_BULLET | F_GEOM;
constexpr int kPfPybAll = F_BULLET | F_GEOM | F_GND | F_DRAG | F_DW;
template <typename R, int ACT>
const void* step_fn_act(bool multi, int flags, bool stream) {
  if (multi) {
    switch (flags) {
      case 0: return (const void*)step_kernel<R, ACT, true, 0>;
      case F_DW: return (const void*)step_kernel<R, ACT, true, F_DW>;
      case kPfPyb: return (const void*)step_kernel<R, ACT, true, kPfPyb>;   // MultiHoverAviary's default physics
      case kPfPybAll: return (const void*)step_kernel<R, ACT, true, kPfPybAll>;
      // the same without the drone <-> drone contact (aero "no_drone_contact"): the kernels
      // compiled without it, as fast as before it existed
      case kPfPyb | F_NO_DC: return (const void*)step_kernel<R, ACT, true, kPfPyb | F_NO_DC>;
      case kPfPybAll | F_NO_DC: return (const void*)step_kernel<R, ACT, true, kPfPybAll | F_NO_DC>;
      default: return (const void*)step_kernel<R, ACT, true, kPfRuntime>;
    }
  }
  switch (flags) {
    case 0: return stream ? (const void*)step_kernel<R, ACT, false, 0, true> : (const void*)step_kernel<R, ACT, false, 0>;
    case kPfAero: return (const void*)step_kernel<R, ACT, false, kPfAero>;
    case kPfPyb: return (const void*)step_kernel<R, ACT, false, kPfPyb>;
    case kPfPybAll: return (const void*)step_kernel<R, ACT, false, kPfPybAll>;
    default: return (const void*)step_kernel<R, ACT, false, kPfRuntime>;
  }
}
template <typename R, int ACT>
const void* step_fn_pid(bool multi, int flags) {
  if (multi) return (const void*)step_kernel<R, ACT, true, kPfRuntime>;
  switch (flags) {
    case 0: return (const void*)step_kernel<R, ACT, false, 0>;
    case kPfPyb: return (const void*)step_kernel<R, ACT, false, kPfPyb>;
    default: return (const void*)step_kernel<R, ACT, false, kPfRuntime>;
  }
}
template <typename R>
const void* step_kernel_fn(const gpd_sim* s) {
  if (s->step_waves == 3)
    return s->cfg.act_type == GPD_ACT_RPM ? (const void*)step_kernel_duo<R, ACT_RPM, true>
                                          : (const void*)step_kernel_duo<R, ACT_ONE_D_RPM, true>;
  if (s->duo)
    return s->cfg.act_type == GPD_ACT_RPM ? (const void*)step_kernel_duo<R, ACT_RPM, false>
                                          : (const void*)step_kernel_duo<R, ACT_ONE_D_RPM, false>;
  const bool multi = s->D > 1;
  // the flags the kernel sees (Consts::flags, make_consts)
  const int pf = s->generic_pf ? kPfRuntime
                              : s->cfg.physics_flags | ((s->cfg.physics_flags & GPD_F_BULLET) ? GPD_F_GEOM_WRENCH : 0);
  switch (s->cfg.act_type) {
    case GPD_ACT_RPM: return step_fn_act<R, ACT_RPM>(multi, pf, s->stream);
    case GPD_ACT_ONE_D_RPM: return step_fn_act<R, ACT_ONE_D_RPM>(multi, pf, s->stream);
    case GPD_ACT_PID: return step_fn_pid<R, ACT_PID>(multi, pf);
    case GPD_ACT_VEL: return step_fn_pid<R, ACT_VEL>(multi, pf);
    default: return step_fn_pid<R, ACT_ONE_D_PID>(multi, pf);
  }
}

// static LDS of the run-time-flag step kernel of an action type (the one-wave kernel every sim
// that is not wide can fall back to: upload_tables)
template <typename R>
size_t runtime_step_lds(int act, bool multi) {
  const void* f;
  switch (act) {
    case GPD_ACT_RPM: f = step_fn_act<R, ACT_RPM>(multi, kPfRuntime, false); break;
    case GPD_ACT_ONE_D_RPM: f = step_fn_act<R, ACT_ONE_D_RPM>(multi, kPfRuntime, false); break;
    case GPD_ACT_PID: f = step_fn_pid<R, ACT_PID>(multi, kPfRuntime); break;
    case GPD_ACT_VEL: f = step_fn_pid<R, ACT_VEL>(multi, kPfRuntime); break;
    default: f = step_fn_pid<R, ACT_ONE_D_PID>(multi, kPfRuntime); break;
  }
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, f) != hipSuccess) {
    (void)hipGetLastError();
    return kLdsBytes;
  }
  return fa.sharedSizeBytes;
}

template <typename R>
int upload_tables(gpd_sim* s) {
  std::vector<R> ini(s->init_tmpl.begin(), s->init_tmpl.end());
  std::vector<R> tgt(s->target.begin(), s->target.end());
  const Consts<R> c = make_consts<R>(s);
  HIP_TRY(hipMemcpy(s->d_init, ini.data(), ini.size() * sizeof(R), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_target, tgt.data(), tgt.size() * sizeof(R), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_consts, &c, sizeof(c), hipMemcpyHostToDevice));
  if (s->wide) return GPD_OK;   // step_kernel_wide: no observation tile
  // the step kernel's static LDS (the PYB flag-set kernels park 44 KB of per-lane values around
  // the contact solve, gpd_device.h bullet_substep) beside the observation tile must fit the
  // workgroup's LDS; a long action history (high ctrl_freq) that leaves no room for it gets the
  // run-time-flag kernel, which solves the contact with its rows in 20 KB of LDS
  const void* f = step_kernel_fn<R>(s);
  hipFuncAttributes fa;
  HIP_TRY(hipFuncGetAttributes(&fa, f));
  if (fa.sharedSizeBytes + (size_t)s->tile_bytes > kLdsBytes && !s->generic_pf) {
    s->generic_pf = true;
    f = step_kernel_fn<R>(s);
    HIP_TRY(hipFuncGetAttributes(&fa, f));
  }
  if (fa.sharedSizeBytes + (size_t)s->tile_bytes > kLdsBytes)
    return fail(GPD_EUNSUPPORTED, "gpd_create: ctrl_freq too high for drone <-> drone contact (observation tile + "
                                  "the step kernel's LDS exceed 160 KiB; GPD_F_NO_DRONE_CONTACT lifts the limit)");
  // the observation tile can exceed the 64 KiB default dynamic-LDS limit for long histories
  if (s->tile_bytes > 65536)
    HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, s->tile_bytes));
  return GPD_OK;
}

inline unsigned grid_for(long long n, int tpb) { return (unsigned)((n + tpb - 1) / tpb); }
inline size_t real_size(const gpd_sim* s) { return s->prec == GPD_F64 ? sizeof(double) : sizeof(float); }
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

template <typename R, int MAXT, bool DC = false>
const void* step_wide_fn(int act) {
  switch (act) {
    case GPD_ACT_RPM: return (const void*)step_kernel_wide<R, ACT_RPM, MAXT, DC>;
    case GPD_ACT_ONE_D_RPM: return (const void*)step_kernel_wide<R, ACT_ONE_D_RPM, MAXT, DC>;
    case GPD_ACT_PID: return (const void*)step_kernel_wide<R, ACT_PID, MAXT, DC>;
    case GPD_ACT_VEL: return (const void*)step_kernel_wide<R, ACT_VEL, MAXT, DC>;
    default: return (const void*)step_kernel_wide<R, ACT_ONE_D_PID, MAXT, DC>;
  }
}
template <typename R, int MAXT>
const void* integrate_wide_fn(bool traj) {
  return traj ? (const void*)integrate_kernel_wide<R, true, MAXT> : (const void*)integrate_kernel_wide<R, false, MAXT>;
}

// last_clipped_action back from the ring (store_drone_step) before anything reads or replaces
// state[16..19]; a no-op launch when no step ran since the last settle
template <typename R>
int settle_last(gpd_sim* s, hipStream_t st) {
  if (!(s->wt & 4)) return GPD_OK;
  const SimView<R> v = make_view<R>(s);
  const Consts<R>* c = (const Consts<R>*)s->d_consts;
  hipLaunchKernelGGL((last_from_ring_kernel<R>), dim3(grid_for(s->N, 256)), dim3(256), 0, st, v, c);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemsetAsync(s->d_ctr + s->E, 0, sizeof(int2), st));
  return GPD_OK;
}
inline int settle_last_any(gpd_sim* s, hipStream_t st) {
  return s->prec == GPD_F64 ? settle_last<double>(s, st) : settle_last<float>(s, st);
}

template <typename R>
int launch_step(gpd_sim* s, const float* actions, float* obs, float* reward, uint8_t* term, uint8_t* trunc,
                float* terminal_obs, hipStream_t st) {
  StepIO<R> io;
  io.actions = actions; io.obs = obs; io.reward = reward; io.term = term; io.trunc = trunc;
  io.terminal_obs = terminal_obs;
  const SimView<R> v = make_view<R>(s);
  const Consts<R>* c = (const Consts<R>*)s->d_consts;
  if (s->wide) {
    // drone <-> drone contact: the one-wave instantiation with the contact solve (D <= 64)
    const bool dc = s->dcP > 0;
    const void* f = dc ? step_wide_fn<R, kWave, true>(s->cfg.act_type)
                    : s->D <= 256 ? step_wide_fn<R, 256>(s->cfg.act_type)
                    : (s->D <= 512 ? step_wide_fn<R, 512>(s->cfg.act_type) : step_wide_fn<R, 1024>(s->cfg.act_type));
    void* args[] = {(void*)&v, (void*)&io, (void*)&c};
    const int ge = s->tpb / s->D;   // envs per workgroup
    HIP_TRY(hipLaunchKernel(f, dim3((s->E + ge - 1) / ge), dim3((s->tpb + kWave - 1) / kWave * kWave), args, 0, st));
    return GPD_OK;
  }
  const unsigned grid = grid_for(s->N, s->tpb);
  const size_t lds = (size_t)s->tile_bytes;
  typedef void (*StepFn)(R*, const float*, int2*, const Consts<R>*, long long, int, int, SimView<R>, StepIO<R>);
  const StepFn f = (StepFn)step_kernel_fn<R>(s);
  hipLaunchKernelGGL(f, dim3(grid), dim3(s->step_waves * kWave), lds, st, v.state, io.actions, v.ctr, c, v.npad,
                     v.N, v.tpb, v, io);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

template <typename R>
int launch_integrate(gpd_sim* s, const void* rpm, int n_sub, void* traj, hipStream_t st) {
  const int rc = settle_last<R>(s, st);   // the raw substeps read and store last_clipped_action
  if (rc != GPD_OK) return rc;
  const SimView<R> v = make_view<R>(s);
  const Consts<R>* c = (const Consts<R>*)s->d_consts;
  const unsigned grid = grid_for(s->N, s->tpb);
  // plain DYN (the raw-integrator bench) compiled without flag tests; everything else at run time
  const bool plain = s->cfg.physics_flags == 0;
  const R* r = (const R*)rpm;
  R* tr = (R*)traj;
  if (s->wide && s->D > kWave) {   // (long-history envs of <= 64 drones: the one-wave kernels, no tile)
    const void* fw = s->D <= 256 ? integrate_wide_fn<R, 256>(tr != nullptr)
                     : (s->D <= 512 ? integrate_wide_fn<R, 512>(tr != nullptr) : integrate_wide_fn<R, 1024>(tr != nullptr));
    void* args[] = {(void*)&v, (void*)&c, (void*)&r, (void*)&n_sub, (void*)&tr};
    HIP_TRY(hipLaunchKernel(fw, dim3(s->E), dim3((s->D + kWave - 1) / kWave * kWave), args, 0, st));
    return GPD_OK;
  }
  const void* f;
  if (tr) {
    f = s->D > 1 ? (const void*)integrate_kernel<R, true, kPfRuntime, true>
                 : (const void*)integrate_kernel<R, false, kPfRuntime, true>;
  } else if (s->D > 1) {
    f = plain ? (const void*)integrate_kernel<R, true, 0, false> : (const void*)integrate_kernel<R, true, kPfRuntime, false>;
  } else {
    f = plain ? (s->N >= (1 << 19) ? (const void*)integrate_kernel<R, false, 0, false, true>
                                    : (const void*)integrate_kernel<R, false, 0, false>)
              : (const void*)integrate_kernel<R, false, kPfRuntime, false>;
  }
  void* args[] = {(void*)&v, (void*)&c, (void*)&r, (void*)&n_sub, (void*)&tr};
  HIP_TRY(hipLaunchKernel(f, dim3(grid), dim3(kWave), args, 0, st));
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

template <typename R>
int launch_reset(gpd_sim* s, const uint8_t* mask, float* obs, hipStream_t st) {
  const SimView<R> v = make_view<R>(s);
  hipLaunchKernelGGL((reset_kernel<R>), dim3(grid_for(s->N, 256)), dim3(256), 0, st, v, mask, obs);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

template <typename R>
int launch_state20(gpd_sim* s, void* out, int raw, hipStream_t st) {
  const int rc = settle_last<R>(s, st);
  if (rc != GPD_OK) return rc;
  const SimView<R> v = make_view<R>(s);
  hipLaunchKernelGGL((state20_kernel<R>), dim3(grid_for(s->N, 256)), dim3(256), 0, st, v, (R*)out, raw);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

template <typename R>
int launch_nonfinite(gpd_sim* s, uint8_t* flags, hipStream_t st) {
  const SimView<R> v = make_view<R>(s);
  HIP_TRY(hipMemsetAsync(flags, 0, (size_t)s->E, st));
  hipLaunchKernelGGL((nonfinite_kernel<R>), dim3(grid_for(s->N, 256)), dim3(256), 0, st, v, flags);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

template <typename R>
int launch_set_raw(gpd_sim* s, const void* in, hipStream_t st) {
  if (s->wt & 4) HIP_TRY(hipMemsetAsync(s->d_ctr + s->E, 0, sizeof(int2), st));   // all 20 replaced
  const SimView<R> v = make_view<R>(s);
  hipLaunchKernelGGL((set_raw_kernel<R>), dim3(grid_for(s->N, 256)), dim3(256), 0, st, v, (const R*)in);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

void free_sim(gpd_sim* s) {
  if (!s) return;
  if (s->d_state) (void)hipFree(s->d_state);
  if (s->d_ctrl) (void)hipFree(s->d_ctrl);
  if (s->d_ring) (void)hipFree(s->d_ring);
  if (s->d_ctr) (void)hipFree(s->d_ctr);
  if (s->d_init) (void)hipFree(s->d_init);
  if (s->d_target) (void)hipFree(s->d_target);
  if (s->d_consts) (void)hipFree(s->d_consts);
  if (s->d_dc_tab) (void)hipFree(s->d_dc_tab);
  if (s->d_dc_rows) (void)hipFree(s->d_dc_rows);
  delete s;
}

}  // namespace

extern "C" {

int gpd_abi_version(void) { return GPD_ABI_VERSION; }

const char* gpd_last_error(void) { return g_err.c_str(); }

int gpd_default_params(int model, gpd_drone_params* out) {
  if (!out) return fail(GPD_EINVAL, "gpd_default_params: out is NULL");
  gpd_drone_params p;
  std::memset(&p, 0, sizeof(p));
  p.model = model;
  // <properties> common to the three URDFs (cf2x.urdf:5)
  p.gnd_eff_coeff = 11.36859; p.drag_coeff_xy = 9.1785e-7; p.drag_coeff_z = 10.311e-7;
  p.dw_coeff_1 = 2267.18; p.dw_coeff_2 = .16; p.dw_coeff_3 = -.11;
  p.collision_h = .025; p.collision_r = .06; p.collision_z_offset = 0.0;  // collision cylinder
  double pp[4][3];
  if (model == GPD_MODEL_CF2X || model == GPD_MODEL_CF2P) {             // cf2x.urdf / cf2p.urdf
    p.arm = 0.0397; p.kf = 3.16e-10; p.km = 7.94e-12; p.thrust2weight = 2.25; p.max_speed_kmh = 30;
    p.prop_radius = 2.31348e-2; p.m = 0.027;
    if (model == GPD_MODEL_CF2X) {
      p.ixx = 1.4e-5; p.iyy = 1.4e-5; p.izz = 2.17e-5;
      const double c[4][3] = {{0.028, -0.028, 0}, {-0.028, -0.028, 0}, {-0.028, 0.028, 0}, {0.028, 0.028, 0}};
      std::memcpy(pp, c, sizeof(pp));
    } else {
      p.ixx = 2.3951e-5; p.iyy = 2.3951e-5; p.izz = 3.2347e-5;
      const double c[4][3] = {{0.0397, 0, 0}, {0, 0.0397, 0}, {-0.0397, 0, 0}, {0, -0.0397, 0}};
      std::memcpy(pp, c, sizeof(pp));
    }
  } else if (model == GPD_MODEL_RACE) {                                   // racer.urdf
    p.arm = 0.109; p.kf = 8.47e-9; p.km = 2.13e-11; p.thrust2weight = 4.17; p.max_speed_kmh = 200;
    p.prop_radius = 12.7e-2; p.m = 0.830; p.ixx = .003113; p.iyy = .003113; p.izz = .003113;
    const double c[4][3] = {{0.0850, 0.0675, 0}, {-0.0850, 0.0675, 0}, {-0.085, -0.0675, 0}, {0.085, -0.0675, 0}};
    std::memcpy(pp, c, sizeof(pp));
  } else {
    return fail(GPD_EINVAL, "gpd_default_params: unknown drone model");
  }
  std::memcpy(p.prop_pos, pp, sizeof(pp));
  *out = p;
  return GPD_OK;
}

int gpd_create(const gpd_drone_params* params, const gpd_config* cfg, gpd_sim** out) {
  if (!params || !cfg || !out) return fail(GPD_EINVAL, "gpd_create: NULL argument");
  *out = nullptr;
  const gpd_config& C = *cfg;
  if (C.n_envs < 1) return fail(GPD_EINVAL, "gpd_create: n_envs must be >= 1");
  if (C.drones_per_env < 1 || C.drones_per_env > kWideMax)
    return fail(GPD_EINVAL, "gpd_create: drones_per_env must be in [1, 1024]");
  if (C.pyb_freq < 1 || C.ctrl_freq < 1) return fail(GPD_EINVAL, "gpd_create: frequencies must be >= 1");
  if (C.pyb_freq % C.ctrl_freq != 0)
    return fail(GPD_EINVAL, "[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.");
  if (C.ctrl_freq / 2 < 1)
    return fail(GPD_EUNSUPPORTED, "gpd_create: ctrl_freq//2 == 0 gives an empty action buffer (unsupported)");
  if (C.act_type < GPD_ACT_RPM || C.act_type > GPD_ACT_ONE_D_PID) return fail(GPD_EINVAL, "gpd_create: bad act_type");
  const bool pid = act_is_pid(C.act_type);
  if (pid && params->model != GPD_MODEL_CF2X && params->model != GPD_MODEL_CF2P)  // BaseRLAviary.py:75-78
    return fail(GPD_EUNSUPPORTED,
                "[ERROR] in BaseRLAviary.__init()__, no controller is available for the specified drone_model");
  if (C.task < GPD_TASK_NONE || C.task > GPD_TASK_MULTIHOVER) return fail(GPD_EINVAL, "gpd_create: bad task");
  if (C.task == GPD_TASK_HOVER && C.drones_per_env != 1)
    return fail(GPD_EINVAL, "gpd_create: HoverAviary is single-drone (drones_per_env must be 1)");
  if (C.precision != GPD_F32 && C.precision != GPD_F64) return fail(GPD_EINVAL, "gpd_create: bad precision");
  if (C.solver_iterations < 0 || C.solver_iterations > 1000)
    return fail(GPD_EINVAL, "gpd_create: solver_iterations must be 0 (default) or in [1, 1000]");
  if (!std::isfinite(C.solver_residual)) return fail(GPD_EINVAL, "gpd_create: solver_residual must be finite");
  if ((C.physics_flags & GPD_F_BULLET) && C.drones_per_env > kWave && !(C.physics_flags & GPD_F_NO_DRONE_CONTACT))
    return fail(GPD_EUNSUPPORTED,
                "gpd_create: drone <-> drone contact is implemented for envs of up to 64 drones; pass "
                "GPD_F_NO_DRONE_CONTACT (aero 'no_drone_contact') for larger PYB* envs");
  if (C.physics_flags & ~(GPD_F_GND | GPD_F_DRAG | GPD_F_DW | GPD_F_GEOM_WRENCH | GPD_F_BULLET | GPD_F_NO_PLANE |
                          GPD_F_NO_DRONE_CONTACT))
    return fail(GPD_EINVAL, "gpd_create: unknown physics flag");
  if (params->model < GPD_MODEL_CF2X || params->model > GPD_MODEL_RACE)
    return fail(GPD_EINVAL, "gpd_create: unknown drone model");
  const long long Nll = (long long)C.n_envs * C.drones_per_env;
  if (Nll > (1LL << 31) - 64) return fail(GPD_EINVAL, "gpd_create: too many drones");

  gpd_sim* s = new gpd_sim();
  s->P = *params;
  s->cfg = C;
  s->cfg.init_xyzs_host = nullptr;
  s->cfg.init_rpys_host = nullptr;
  s->E = C.n_envs;
  s->D = C.drones_per_env;
  s->N = (int)Nll;
  s->A = act_width(C.act_type);
  gpd_default_pid_params(&s->pid);
  s->ring_len = C.ctrl_freq / 2;  // ACTION_BUFFER_SIZE = int(ctrl_freq//2)  BaseRLAviary.py:66
  s->W = 12 + s->ring_len * s->A;
  s->nsub = C.pyb_freq / C.ctrl_freq;
  s->prec = C.precision;
  // Drones per 64-lane block.  A wave's time is set by its serial instruction stream, not by
  // how many of its lanes are active, while a CU streams the observation rows of its blocks at
  // a limited store-issue rate; so when there are too few drones to give every CU a full wave,
  // blocks are thinned (down to 16 drones) to spread the rows over all 256 CUs.
  {
    const int full = (kWave / s->D) * s->D;
    const long long per_cu = (Nll + 255) / 256;
    int want = (int)std::min<long long>(full, std::max<long long>(16, per_cu));
    if (s->D > 1 && (C.physics_flags & GPD_F_DW)) {
      // downwash envs: the per-substep pair work is spread over a block's lanes, and about four
      // blocks per CU measured best (scripts/geom_probe_multi.py, D = 8, staggered init:
      // 512 envs 8 drones/block 13.2 us vs 16: 14.7; 2048 envs 16: 16.1 vs 64: 23.2;
      // 8192 envs 64: 27.3 vs 16: 50.3)
      want = (int)std::min<long long>(full, Nll / 1024);
    }
    want = std::max(s->D, (want / s->D) * s->D);
    if (C.drones_per_block > 0) want = std::max(s->D, std::min(full, (C.drones_per_block / s->D) * s->D));
    s->tpb = want;
    // envs of more than 64 drones: one env per multi-wave workgroup (step_kernel_wide).  Also an
    // observation row too long for the one-wave kernels (their LDS tile of 64 rows beside the
    // run-time-flag kernel's static LDS: a long action history, e.g. RPM actions at ctrl_freq 480):
    // the wide kernel copies the history columns without a tile (with the drone <-> drone contact
    // in its one-wave instantiation, D <= 64)
    const size_t tile = (size_t)step_tile_bytes(s->A, s->ring_len);
    const size_t lds_rt = s->D > kWave ? 0
                          : (C.precision == GPD_F64 ? runtime_step_lds<double>(C.act_type, s->D > 1)
                                                    : runtime_step_lds<float>(C.act_type, s->D > 1));
    s->wide = s->D > kWave || tile + lds_rt > (size_t)kLdsBytes;
    // envs of up to 32 drones share the wave, up to 64 / D of them, as many as leave ~2048
    // workgroups (the history copy's loads in flight: 4096 single-drone envs at ctrl_freq 480
    // 37.8 us per step with one env per workgroup, 86.7 with 64; 65536 envs 591 / 213 us);
    // gpd_config::drones_per_block overrides
    if (s->wide) {
      int ge = 1;
      if (s->D <= kWave / 2) {
        const int gmax = kWave / s->D;
        ge = C.drones_per_block > 0 ? C.drones_per_block / s->D : (int)std::min<long long>(gmax, C.n_envs / 2048);
        ge = std::max(1, std::min(gmax, ge));
      }
      s->tpb = ge * s->D;
    }
  }
  s->npad = ((long long)s->N + 63) / 64 * 64;
  {
    // downwash pairs over idle lanes: only for thin blocks whose pairs fit the LDS buffer
    const int D = s->D, n = s->tpb * D;
    if (D > 1 && (C.physics_flags & GPD_F_DW) && s->tpb < kWave && n <= kPairMax) {
      const int m = ((1 << 20) + D - 1) / D;
      bool ok = true;
      for (int p = 0; p < n && ok; ++p) ok = ((p * m) >> 20) == p / D;
      if (ok) s->dw_pairs = DwPairs{n, m};
    }
  }
  {
    // write-through (sc1) stores for the obs rows (bit 0) and the state (bit 1), default both:
    // measured on one MI355X, 4096 envs 8.60 -> 8.37 us/step and 65536 envs 15.3 -> 13.7 us,
    // large N unchanged (gpd_config::store_policy overrides).  State only while its byte
    // offsets fit the 32-bit buffer offset (re-applied after the wave-count policies below).
    s->wt = C.store_policy > 0 ? ((C.store_policy - 1) & 3) : 3;
    // bit 2: the step kernels leave last_clipped_action in the ring (store_drone_step) where
    // the step never reads it back: RPM action types (the ring holds the very actions it maps),
    // no drag (the only reader, on the first substep)
    if ((C.act_type == GPD_ACT_RPM || C.act_type == GPD_ACT_ONE_D_RPM) && !(C.physics_flags & GPD_F_DRAG)) s->wt |= 4;
  }
  s->bound_xy = C.task == GPD_TASK_MULTIHOVER ? 2.0 : 1.5;
  s->tile_bytes = step_tile_bytes(s->A, s->ring_len);
  {
    // division-free row/column split of the copy-out (t / NC for t <= 64)
    const int NC = s->A == 4 ? 3 + s->ring_len : 12 + s->ring_len * s->A;
    s->nc_magic = (65536 + NC - 1) / NC;
    for (int t = 0; t <= kWave && !s->wide; ++t)   // (the wide kernel has no tile copy-out)
      if ((t * s->nc_magic) >> 16 != t / NC) {
        delete s;
        return fail(GPD_EUNSUPPORTED, "gpd_create: observation width not supported by the tile copy-out");
      }
    // two-wave step (step_kernel_duo) for the plain-DYN single-drone RPM path while the launch
    // is latency-bound: up to 64K drones (<= 4 blocks per CU).  Measured on one MI355X
    // (scripts/geom_probe.py): 4096 envs 6.28 -> 5.71 us/step, 16384 envs 7.48 -> 6.49,
    // 65536 envs 10.45 -> 10.31, but 262144 envs 35.8 -> 38.1 (bandwidth-bound: the second
    // wave only adds occupancy pressure).  Its 128-lane copy-out needs t / NC for t <= 128.
    // A third (io) wave takes the history columns off the pose wave (step_waves = 3): measured
    // (scripts/geom_probe.py, gpurun_out r2n) 2048 envs 5.30 -> 5.24 us/step, 4096 envs 5.40 ->
    // 5.33, but 8192 envs 5.72 -> 5.90 and 16384 envs 6.23 -> 7.20: with fuller blocks the
    // two-wave copy-out overlaps other blocks' work anyway.
    // gpd_config::step_waves overrides (1, 2 or 3).
    const bool duo_ok = !s->wide && s->D == 1 && C.physics_flags == 0 &&
                        (C.act_type == GPD_ACT_RPM || C.act_type == GPD_ACT_ONE_D_RPM);
    int waves = !duo_ok || s->N > 65536 ? 1 : (s->N <= 4096 ? 3 : 2);
    if (C.step_waves > 0) waves = duo_ok ? std::min(3, C.step_waves) : 1;
    for (int t = 0; t <= 2 * kWave && waves == 2; ++t)
      if ((t * s->nc_magic) >> 16 != t / NC) waves = 1;
    s->step_waves = waves;
    s->duo = waves >= 2;
    // streaming cache policies for the single-wave plain-DYN kernel once a step's working set
    // (~820 B per drone: state, ring, rows) is well past the 256 MB Infinity Cache (>= 512K drones;
    // 262144 envs = 215 MB stay with the default policies, 1M envs 194 -> 145 us with STREAM,
    // 4096 envs 4.93 -> 6.31 us had it been used there)
    s->stream = !s->duo && !s->wide && s->D == 1 && C.physics_flags == 0 &&
                (C.act_type == GPD_ACT_RPM || C.act_type == GPD_ACT_ONE_D_RPM) && s->N >= (1 << 19);
    // the multi-wave kernels store their state plainly (measured 4096 envs 5.47 -> 5.37 us/step);
    // the single-wave kernel keeps write-through state stores (262144 envs 36.7 -> 35.9 us)
    if (s->duo && C.store_policy <= 0) s->wt &= ~2;
    // the io-wave kernel writes each observation row in two parts from two waves (12 state columns,
    // history columns): write-through row stores leave those lines partially written twice, +0.29 MB
    // of HBM writes per launch at 4096 envs (PMC/alg 1.232 -> 1.143 with plain row stores and
    // write-through state, store_policy 3; step time 4.93 vs 4.97 us, within the run-to-run spread:
    // profiles/r3/pmc4096, profiles/r3/policy_4096.log)
    if (waves == 3 && C.store_policy <= 0) s->wt = (s->wt & ~1) | 2;
    // write-through state stores address the whole state through one buffer resource with 32-bit
    // offsets (store_drone_wt): whatever the policy above chose, never past 2 GiB of state
    const size_t state_bytes = (size_t)kStateComps * s->npad * (C.precision == GPD_F64 ? 8 : 4);
    if (state_bytes >= 0x7fffffffULL) s->wt &= ~2;
  }
  if (s->tile_bytes > kLdsBytes && !s->wide) {
    delete s;
    return fail(GPD_EUNSUPPORTED, "gpd_create: ctrl_freq too high for drone <-> drone contact (observation tile "
                                  "exceeds 160 KiB of LDS; GPD_F_NO_DRONE_CONTACT lifts the limit)");
  }

  // derived constants (BaseAviary.py:117-128)
  const gpd_drone_params& P = *params;
  gpd_constants& K = s->K;
  std::memset(&K, 0, sizeof(K));
  K.gravity = 9.8 * P.m;
  K.hover_rpm = std::sqrt(K.gravity / (4 * P.kf));
  K.max_rpm = std::sqrt((P.thrust2weight * K.gravity) / (4 * P.kf));
  K.max_thrust = 4 * P.kf * (K.max_rpm * K.max_rpm);
  K.max_xy_torque = P.model == GPD_MODEL_CF2P ? P.arm * P.kf * (K.max_rpm * K.max_rpm)
                                              : (2 * P.arm * P.kf * (K.max_rpm * K.max_rpm)) / std::sqrt(2.0);
  K.max_z_torque = 2 * P.km * (K.max_rpm * K.max_rpm);
  K.gnd_eff_h_clip = 0.25 * P.prop_radius *
                     std::sqrt((15 * (K.max_rpm * K.max_rpm) * P.kf * P.gnd_eff_coeff) / K.max_thrust);
  K.pyb_timestep = 1.0 / C.pyb_freq;
  K.ctrl_timestep = 1.0 / C.ctrl_freq;
  K.pyb_steps_per_ctrl = s->nsub;
  K.action_buffer_size = s->ring_len;
  K.obs_width = s->W;
  K.act_width = s->A;
  K.n_drones = s->N;
  K.drones_per_block = s->tpb;
  K.lanes_per_block = s->step_waves * kWave;
  {  // truncated iff step_counter / PYB_FREQ > EPISODE_LEN_SEC  (HoverAviary.py:114)
    long long sc = (long long)std::floor(C.episode_len_sec * C.pyb_freq);
    if (sc < 0) sc = 0;
    while (sc > 0 && (double)(sc - 1) / C.pyb_freq > C.episode_len_sec) --sc;
    while (!((double)sc / C.pyb_freq > C.episode_len_sec)) ++sc;
    K.trunc_step_counter = (int)std::min<long long>(sc, 0x7fffffff);
  }

  // reset template: INIT_XYZS (BaseAviary.py:194-197) and the orientation the client stores
  s->init_tmpl.assign((size_t)s->D * 10, 0.0);
  s->target.assign((size_t)s->D * 3, 0.0);
  for (int d = 0; d < s->D; ++d) {
    double xyz[3], rpy[3] = {0, 0, 0};
    if (C.init_xyzs_host) {
      for (int k = 0; k < 3; ++k) xyz[k] = C.init_xyzs_host[d * 3 + k];
    } else {
      xyz[0] = d * 4 * P.arm;
      xyz[1] = d * 4 * P.arm;
      xyz[2] = P.collision_h / 2 - P.collision_z_offset + .1;
    }
    if (C.init_rpys_host)
      for (int k = 0; k < 3; ++k) rpy[k] = C.init_rpys_host[d * 3 + k];
    double q0[4], qraw[4], qn[4], e[3];
    h_quat_from_euler(rpy, q0);
    h_roundtrip(q0, qraw);  // loadURDF stores the orientation through a btTransform
    h_roundtrip(qraw, qn);  // readback (:517)
    h_euler(qn, e);         // :518
    double* t = &s->init_tmpl[(size_t)d * 10];
    t[0] = xyz[0]; t[1] = xyz[1]; t[2] = xyz[2];
    t[3] = qraw[0]; t[4] = qraw[1]; t[5] = qraw[2]; t[6] = qraw[3];
    t[7] = e[0]; t[8] = e[1]; t[9] = e[2];
    if (C.task == GPD_TASK_HOVER) {           // HoverAviary.py:51
      s->target[d * 3 + 2] = 1.0;
    } else if (C.task == GPD_TASK_MULTIHOVER) {  // MultiHoverAviary.py:71
      s->target[d * 3 + 0] = xyz[0];
      s->target[d * 3 + 1] = xyz[1];
      s->target[d * 3 + 2] = xyz[2] + 1.0 / (d + 1);
    }
  }

  const size_t rs = real_size(s);
  hipError_t e1 = hipMalloc(&s->d_state, (size_t)kStateComps * s->npad * rs);
  hipError_t e2 = hipMalloc((void**)&s->d_ring, (size_t)s->ring_len * s->npad * s->A * sizeof(float));
  hipError_t e3 = hipMalloc((void**)&s->d_ctr, (size_t)(s->E + 1) * sizeof(int2));
  hipError_t e4 = hipMalloc(&s->d_init, (size_t)s->D * 10 * rs);
  hipError_t e5 = hipMalloc(&s->d_target, (size_t)s->D * 3 * rs);
  hipError_t e6 = hipMalloc(&s->d_consts, s->prec == GPD_F64 ? sizeof(Consts<double>) : sizeof(Consts<float>));
  hipError_t e7 = pid ? hipMalloc(&s->d_ctrl, (size_t)kCtrlComps * s->npad * rs) : hipSuccess;
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess || e5 != hipSuccess ||
      e6 != hipSuccess || e7 != hipSuccess) {
    free_sim(s);
    (void)hipGetLastError();
    return fail(GPD_ENOMEM, "gpd_create: hipMalloc failed");
  }
  if ((C.physics_flags & GPD_F_BULLET) && s->D > 1 && !(C.physics_flags & GPD_F_NO_DRONE_CONTACT)) {
    // drone <-> drone contact (gpd_kernels.h DcHook / dc_solve): the pair table of an env and the
    // row store for a block's contacts past its first 64 (up to kDcPts per pair: the closest point
    // and the face manifold)
    const int D = s->D, P = D * (D - 1) / 2;
    const int npairs = (s->tpb / D) * P;
    s->dcP = P;
    s->dc_pmagic = ((1 << 24) + P - 1) / P;   // exact for p < npairs <= 32 (D - 1) <= 2016 (p P < 2^24)
    for (int p = 0; p < npairs; ++p)
      if (((p * s->dc_pmagic) >> 24) != p / P) {
        free_sim(s);
        return fail(GPD_EUNSUPPORTED, "gpd_create: drone contact pair layout not supported");
      }
    std::vector<int> tab;
    tab.reserve(P);
    for (int i = 0; i < D; ++i)
      for (int j = i + 1; j < D; ++j) tab.push_back(i | (j << 8));   // bullet_mb.drone_contacts' order
    if (hipMalloc((void**)&s->d_dc_tab, (size_t)P * sizeof(int)) != hipSuccess ||
        hipMemcpy(s->d_dc_tab, tab.data(), (size_t)P * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
      free_sim(s);
      (void)hipGetLastError();
      return fail(GPD_ENOMEM, "gpd_create: drone contact pair table");
    }
    if (npairs * kDcPts > kDcRegRows * kWave) {
      const int row_reals = s->prec == GPD_F64 ? dc_row_reals<double>() : dc_row_reals<float>();
      const int chunks = (npairs * kDcPts + kWave - 1) / kWave - kDcRegRows;
      s->dc_row_stride = (long long)chunks * kWave * row_reals;
      const long long blocks = ((long long)s->N + s->tpb - 1) / s->tpb;
      if (hipMalloc(&s->d_dc_rows, (size_t)(blocks * s->dc_row_stride) * rs) != hipSuccess) {
        free_sim(s);
        (void)hipGetLastError();
        return fail(GPD_ENOMEM, "gpd_create: drone contact row store");
      }
    }
  }
  int rc = s->prec == GPD_F64 ? upload_tables<double>(s) : upload_tables<float>(s);
  if (rc != GPD_OK) { free_sim(s); return rc; }
  if (hipMemset(s->d_state, 0, (size_t)kStateComps * s->npad * rs) != hipSuccess ||
      hipMemset(s->d_ring, 0, (size_t)s->ring_len * s->npad * s->A * sizeof(float)) != hipSuccess ||
      hipMemset(s->d_ctr, 0, (size_t)(s->E + 1) * sizeof(int2)) != hipSuccess ||
      (pid && hipMemset(s->d_ctrl, 0, (size_t)kCtrlComps * s->npad * rs) != hipSuccess)) {
    free_sim(s);
    return fail(GPD_EHIP, "gpd_create: hipMemset failed");
  }
  rc = s->prec == GPD_F64 ? launch_reset<double>(s, nullptr, nullptr, 0) : launch_reset<float>(s, nullptr, nullptr, 0);
  if (rc == GPD_OK && hipDeviceSynchronize() != hipSuccess) rc = fail(GPD_EHIP, "gpd_create: initial reset failed");
  if (rc != GPD_OK) { free_sim(s); return rc; }
  *out = s;
  return GPD_OK;
}

int gpd_destroy(gpd_sim* sim) {
  if (!sim) return fail(GPD_EINVAL, "gpd_destroy: NULL sim");
  (void)hipDeviceSynchronize();
  free_sim(sim);
  return GPD_OK;
}

int gpd_get_constants(const gpd_sim* sim, gpd_constants* out) {
  if (!sim || !out) return fail(GPD_EINVAL, "gpd_get_constants: NULL argument");
  *out = sim->K;
  return GPD_OK;
}

int gpd_reset(gpd_sim* sim, const uint8_t* env_mask, float* obs, void* stream) {
  if (!sim) return fail(GPD_EINVAL, "gpd_reset: NULL sim");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_reset<double>(sim, env_mask, obs, st) : launch_reset<float>(sim, env_mask, obs, st);
}

int gpd_step(gpd_sim* sim, const float* actions, float* obs, float* reward, uint8_t* terminated,
             uint8_t* truncated, float* terminal_obs, void* stream) {
  if (!sim || !actions || !obs || !reward || !terminated || !truncated)
    return fail(GPD_EINVAL, "gpd_step: NULL argument");
  if (sim->A == 4 && !aligned16(actions)) return fail(GPD_EINVAL, "gpd_step: actions must be 16-byte aligned");
  if (sim->A == 4 && (!aligned16(obs) || (terminal_obs && !aligned16(terminal_obs))))
    return fail(GPD_EINVAL, "gpd_step: obs buffers must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64
             ? launch_step<double>(sim, actions, obs, reward, terminated, truncated, terminal_obs, st)
             : launch_step<float>(sim, actions, obs, reward, terminated, truncated, terminal_obs, st);
}

int gpd_step_seq(gpd_sim* sim, const float* actions, int n_slots, int n_steps, float* obs, float* reward,
                 uint8_t* terminated, uint8_t* truncated, float* terminal_obs, void* stream) {
  if (!sim || !actions || !obs || !reward || !terminated || !truncated)
    return fail(GPD_EINVAL, "gpd_step_seq: NULL argument");
  if (n_slots < 1 || n_steps < 0) return fail(GPD_EINVAL, "gpd_step_seq: n_slots must be >= 1, n_steps >= 0");
  if (sim->A == 4 && !aligned16(actions)) return fail(GPD_EINVAL, "gpd_step_seq: actions must be 16-byte aligned");
  if (sim->A == 4 && (!aligned16(obs) || (terminal_obs && !aligned16(terminal_obs))))
    return fail(GPD_EINVAL, "gpd_step_seq: obs buffers must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const size_t slot = (size_t)sim->N * sim->A;
  for (int t = 0; t < n_steps; ++t) {
    const float* a = actions + (size_t)(t % n_slots) * slot;
    const int rc = sim->prec == GPD_F64
                       ? launch_step<double>(sim, a, obs, reward, terminated, truncated, terminal_obs, st)
                       : launch_step<float>(sim, a, obs, reward, terminated, truncated, terminal_obs, st);
    if (rc != GPD_OK) return rc;
  }
  return GPD_OK;
}

int gpd_integrate(gpd_sim* sim, const void* rpm, int n_sub, void* traj, void* stream) {
  if (!sim || !rpm) return fail(GPD_EINVAL, "gpd_integrate: NULL argument");
  if (n_sub < 0) return fail(GPD_EINVAL, "gpd_integrate: n_sub < 0");
  if (n_sub == 0) return GPD_OK;
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_integrate<double>(sim, rpm, n_sub, traj, st)
                              : launch_integrate<float>(sim, rpm, n_sub, traj, st);
}

int gpd_get_state20(gpd_sim* sim, void* out, void* stream) {
  if (!sim || !out) return fail(GPD_EINVAL, "gpd_get_state20: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_state20<double>(sim, out, 0, st) : launch_state20<float>(sim, out, 0, st);
}

int gpd_get_raw_state(gpd_sim* sim, void* out, void* stream) {
  if (!sim || !out) return fail(GPD_EINVAL, "gpd_get_raw_state: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_state20<double>(sim, out, 1, st) : launch_state20<float>(sim, out, 1, st);
}

int gpd_nonfinite(gpd_sim* sim, uint8_t* env_flags, void* stream) {
  if (!sim || !env_flags) return fail(GPD_EINVAL, "gpd_nonfinite: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_nonfinite<double>(sim, env_flags, st) : launch_nonfinite<float>(sim, env_flags, st);
}

int gpd_set_raw_state(gpd_sim* sim, const void* in, void* stream) {
  if (!sim || !in) return fail(GPD_EINVAL, "gpd_set_raw_state: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  return sim->prec == GPD_F64 ? launch_set_raw<double>(sim, in, st) : launch_set_raw<float>(sim, in, st);
}

int gpd_default_pid_params(gpd_pid_params* out) {
  if (!out) return fail(GPD_EINVAL, "gpd_default_pid_params: out is NULL");
  gpd_pid_params q;
  std::memset(&q, 0, sizeof(q));
  const double pf[3] = {.4, .4, 1.25}, iff[3] = {.05, .05, .05}, df[3] = {.2, .2, .5};       // :37-39
  const double pt[3] = {70000., 70000., 60000.}, it[3] = {.0, .0, 500.}, dtq[3] = {20000., 20000., 12000.};  // :40-42
  const double mix[4][3] = {{-.5, -.5, -1}, {-.5, .5, 1}, {.5, .5, -1}, {.5, -.5, 1}};     // :48-53 (CF2X)
  for (int i = 0; i < 3; ++i) {
    q.p_coeff_for[i] = pf[i]; q.i_coeff_for[i] = iff[i]; q.d_coeff_for[i] = df[i];
    q.p_coeff_tor[i] = pt[i]; q.i_coeff_tor[i] = it[i]; q.d_coeff_tor[i] = dtq[i];
  }
  q.pwm2rpm_scale = 0.2685; q.pwm2rpm_const = 4070.3; q.min_pwm = 20000; q.max_pwm = 65535;  // :43-46
  std::memcpy(q.mixer, mix, sizeof(mix));
  q.gravity = 9.8 * 0.027;  // g * m of cf2x.urdf:11 (BaseControl.py:35)
  q.kf = 3.16e-10;          // cf2x.urdf:5 (BaseControl.py:37)
  *out = q;
  return GPD_OK;
}

int gpd_set_pid_params(gpd_sim* sim, const gpd_pid_params* params) {
  if (!sim || !params) return fail(GPD_EINVAL, "gpd_set_pid_params: NULL argument");
  if (!act_is_pid(sim->cfg.act_type))
    return fail(GPD_EINVAL, "gpd_set_pid_params: the sim's action type has no controller");
  sim->pid = *params;
  HIP_TRY(hipDeviceSynchronize());
  return sim->prec == GPD_F64 ? upload_tables<double>(sim) : upload_tables<float>(sim);
}

int gpd_get_ctrl_state(gpd_sim* sim, void* out, void* stream) {
  if (!sim || !out) return fail(GPD_EINVAL, "gpd_get_ctrl_state: NULL argument");
  if (!sim->d_ctrl) return fail(GPD_EINVAL, "gpd_get_ctrl_state: the sim's action type has no controller");
  const unsigned g = grid_for(sim->N, 256);
  hipStream_t st = (hipStream_t)stream;
  if (sim->prec == GPD_F64)
    hipLaunchKernelGGL((soa_to_rows_kernel<double>), dim3(g), dim3(256), 0, st, (const double*)sim->d_ctrl, sim->npad,
                       kCtrlComps, sim->N, (double*)out);
  else
    hipLaunchKernelGGL((soa_to_rows_kernel<float>), dim3(g), dim3(256), 0, st, (const float*)sim->d_ctrl, sim->npad,
                       kCtrlComps, sim->N, (float*)out);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_set_ctrl_state(gpd_sim* sim, const void* in, void* stream) {
  if (!sim || !in) return fail(GPD_EINVAL, "gpd_set_ctrl_state: NULL argument");
  if (!sim->d_ctrl) return fail(GPD_EINVAL, "gpd_set_ctrl_state: the sim's action type has no controller");
  const unsigned g = grid_for(sim->N, 256);
  hipStream_t st = (hipStream_t)stream;
  if (sim->prec == GPD_F64)
    hipLaunchKernelGGL((rows_to_soa_kernel<double>), dim3(g), dim3(256), 0, st, (const double*)in, sim->npad, kCtrlComps,
                       sim->N, (double*)sim->d_ctrl);
  else
    hipLaunchKernelGGL((rows_to_soa_kernel<float>), dim3(g), dim3(256), 0, st, (const float*)in, sim->npad, kCtrlComps,
                       sim->N, (float*)sim->d_ctrl);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_get_step_counters(gpd_sim* sim, int32_t* out, void* stream) {
  if (!sim || !out) return fail(GPD_EINVAL, "gpd_get_step_counters: NULL argument");
  HIP_TRY(hipMemcpy2DAsync(out, sizeof(int32_t), sim->d_ctr, sizeof(int2), sizeof(int32_t), (size_t)sim->E,
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GPD_OK;
}

int gpd_set_step_counters(gpd_sim* sim, const int32_t* in, void* stream) {
  if (!sim || !in) return fail(GPD_EINVAL, "gpd_set_step_counters: NULL argument");
  const int rc = settle_last_any(sim, (hipStream_t)stream);   // the ring-derived value reads them
  if (rc != GPD_OK) return rc;
  HIP_TRY(hipMemcpy2DAsync(sim->d_ctr, sizeof(int2), in, sizeof(int32_t), sizeof(int32_t), (size_t)sim->E,
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GPD_OK;
}

namespace {
// checkpoint sections: state, controller state (PID types), action ring, counters
struct Section { void* dev; size_t bytes; };
// blob header: everything that fixes the section sizes and meaning
constexpr size_t kBlobHeader = 64;
void blob_header(const gpd_sim* sim, int64_t h[kBlobHeader / 8]) {
  const int64_t v[kBlobHeader / 8] = {(int64_t)GPD_ABI_VERSION, (int64_t)sim->N, (int64_t)sim->E, (int64_t)sim->D,
                                      (int64_t)sim->cfg.act_type, (int64_t)sim->prec, (int64_t)sim->ring_len,
                                      (int64_t)sim->npad};
  for (size_t i = 0; i < kBlobHeader / 8; ++i) h[i] = v[i];
}
int sections(gpd_sim* sim, Section out[4]) {
  out[0] = {sim->d_state, (size_t)kStateComps * sim->npad * real_size(sim)};
  out[1] = {sim->d_ctrl, sim->d_ctrl ? (size_t)kCtrlComps * sim->npad * real_size(sim) : 0};
  out[2] = {sim->d_ring, (size_t)sim->ring_len * sim->npad * sim->A * sizeof(float)};
  out[3] = {sim->d_ctr, (size_t)sim->E * sizeof(int2)};
  return 4;
}
}  // namespace

size_t gpd_state_bytes(const gpd_sim* sim) {
  if (!sim) return 0;
  Section sec[4];
  const int ns = sections(const_cast<gpd_sim*>(sim), sec);
  size_t total = kBlobHeader;
  for (int i = 0; i < ns; ++i) total += sec[i].bytes;
  return total;
}

int gpd_save_state(gpd_sim* sim, void* blob_host, void* stream) {
  if (!sim || !blob_host) return fail(GPD_EINVAL, "gpd_save_state: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  char* b = (char*)blob_host;
  int64_t hdr[kBlobHeader / 8];
  blob_header(sim, hdr);
  std::memcpy(b, hdr, kBlobHeader);
  const int rc = settle_last_any(sim, st);
  if (rc != GPD_OK) return rc;
  size_t off = kBlobHeader;
  Section sec[4];
  const int ns = sections(sim, sec);
  for (int i = 0; i < ns; ++i) {
    if (sec[i].bytes) HIP_TRY(hipMemcpyAsync(b + off, sec[i].dev, sec[i].bytes, hipMemcpyDeviceToHost, st));
    off += sec[i].bytes;
  }
  HIP_TRY(hipStreamSynchronize(st));
  return GPD_OK;
}

int gpd_load_state(gpd_sim* sim, const void* blob_host, void* stream) {
  if (!sim || !blob_host) return fail(GPD_EINVAL, "gpd_load_state: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  const char* b = (const char*)blob_host;
  int64_t hdr[kBlobHeader / 8], mine[kBlobHeader / 8];
  std::memcpy(hdr, b, kBlobHeader);
  blob_header(sim, mine);
  if (std::memcmp(hdr, mine, kBlobHeader) != 0)
    return fail(GPD_EINVAL, "gpd_load_state: blob does not match this sim");
  size_t off = kBlobHeader;
  Section sec[4];
  const int ns = sections(sim, sec);
  for (int i = 0; i < ns; ++i) {
    if (sec[i].bytes) HIP_TRY(hipMemcpyAsync(sec[i].dev, b + off, sec[i].bytes, hipMemcpyHostToDevice, st));
    off += sec[i].bytes;
  }
  if (sim->wt & 4) HIP_TRY(hipMemsetAsync(sim->d_ctr + sim->E, 0, sizeof(int2), st));   // saved settled
  HIP_TRY(hipStreamSynchronize(st));
  return GPD_OK;
}

// ---- config-5 learner hand-off (gpd_handoff.h; SURVEY §8(e), caller examples/learn.py:52-94)
namespace {
constexpr long long kPackAlign = 256;
inline long long align_up(long long n) { return (n + kPackAlign - 1) / kPackAlign * kPackAlign; }

int check_layout(const gpd_pack_layout* L, const char* fn) {
  if (!L) return fail(GPD_EINVAL, std::string(fn) + ": NULL layout");
  if (L->n_envs < 1 || L->drones_per_env < 1 || L->obs_width < kHandoffStateCols ||
      L->state_cols != kHandoffStateCols)
    return fail(GPD_EINVAL, std::string(fn) + ": layout not made by gpd_pack_layout_of");
  gpd_pack_layout ref;
  gpd_pack_layout_of(L->n_envs, L->drones_per_env, L->obs_width, &ref);
  if (std::memcmp(&ref, L, sizeof(ref)) != 0)
    return fail(GPD_EINVAL, std::string(fn) + ": layout offsets differ from gpd_pack_layout_of's");
  return GPD_OK;
}

HandoffView handoff_view(const gpd_pack_layout* L, long long stride, int n_ranks) {
  HandoffView v;
  v.obs = L->obs; v.reward = L->reward; v.term = L->terminated; v.trunc = L->truncated;
  v.tstate = L->terminal_state; v.tobs = L->terminal_obs; v.stride = stride;
  v.E = L->n_envs; v.D = L->drones_per_env; v.W = L->obs_width; v.G = n_ranks;
  return v;
}
}  // namespace

int gpd_pack_layout_of(int n_envs, int drones_per_env, int obs_width, gpd_pack_layout* out) {
  if (!out || n_envs < 1 || drones_per_env < 1 || obs_width < kHandoffStateCols)
    return fail(GPD_EINVAL, "gpd_pack_layout_of: invalid argument");
  const long long E = n_envs, D = drones_per_env, W = obs_width;
  gpd_pack_layout L;
  std::memset(&L, 0, sizeof(L));
  L.n_envs = n_envs; L.drones_per_env = drones_per_env; L.obs_width = obs_width;
  L.state_cols = kHandoffStateCols;
  long long off = 0;
  L.obs = off;            off += align_up(E * D * W * 4);
  L.reward = off;         off += align_up(E * 4);
  L.terminated = off;     off += align_up(E);
  L.truncated = off;
  L.prefix = off + E;
  L.prefix_aligned = align_up(L.prefix);
  off += align_up(E);
  L.terminal_state = off; off += align_up(E * D * kHandoffStateCols * 4);
  L.record = off;
  L.terminal_obs = off;   off += align_up(E * D * W * 4);
  L.total = off;
  *out = L;
  return GPD_OK;
}

int gpd_handoff_pack(uint8_t* pack, const gpd_pack_layout* layout, void* stream) {
  const int rc = check_layout(layout, "gpd_handoff_pack");
  if (rc != GPD_OK) return rc;
  if (!pack) return fail(GPD_EINVAL, "gpd_handoff_pack: NULL pack");
  const HandoffView v = handoff_view(layout, layout->record, 1);
  const long long n = (long long)v.E * v.D * kHandoffStateCols;
  if (n >= (1ll << 31)) return fail(GPD_EINVAL, "gpd_handoff_pack: shard too large");
  hipLaunchKernelGGL(handoff_pack_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, pack, v);
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_handoff_unpack(const uint8_t* gathered, int n_ranks, long long stride, const gpd_pack_layout* layout,
                       float* obs, float* reward, uint8_t* terminated, uint8_t* truncated, float* terminal_obs,
                       void* stream) {
  const int rc = check_layout(layout, "gpd_handoff_unpack");
  if (rc != GPD_OK) return rc;
  if (!gathered || !obs || !reward || !terminated || !truncated || n_ranks < 1)
    return fail(GPD_EINVAL, "gpd_handoff_unpack: NULL output or n_ranks < 1");
  if (stride != layout->prefix_aligned && stride != layout->record)
    return fail(GPD_EINVAL, "gpd_handoff_unpack: stride must be the layout's prefix_aligned or record");
  if (terminal_obs && stride != layout->record)
    return fail(GPD_EINVAL, "gpd_handoff_unpack: terminal rows need whole records (stride = record)");
  const HandoffView v = handoff_view(layout, stride, n_ranks);
  const long long rows = (long long)v.E * v.D;
  if (rows * v.W * n_ranks >= (1ll << 31))
    return fail(GPD_EINVAL, "gpd_handoff_unpack: gathered batch too large");
  hipStream_t st = (hipStream_t)stream;
  const bool vec4 = v.W % 4 == 0 && aligned16(obs) && (!terminal_obs || aligned16(terminal_obs)) && aligned16(gathered);
  const long long nvec = rows * v.W / (vec4 ? 4 : 1) * n_ranks;
  const long long nthr = std::max(nvec, (long long)v.E * n_ranks);
  const dim3 grid(grid_for(nthr, 256)), block(256);
  if (vec4) {
    if (terminal_obs)
      hipLaunchKernelGGL((handoff_unpack_kernel<4, true>), grid, block, 0, st, gathered, v, obs, reward, terminated,
                         truncated, terminal_obs);
    else
      hipLaunchKernelGGL((handoff_unpack_kernel<4, false>), grid, block, 0, st, gathered, v, obs, reward, terminated,
                         truncated, terminal_obs);
  } else {
    if (terminal_obs)
      hipLaunchKernelGGL((handoff_unpack_kernel<1, true>), grid, block, 0, st, gathered, v, obs, reward, terminated,
                         truncated, terminal_obs);
    else
      hipLaunchKernelGGL((handoff_unpack_kernel<1, false>), grid, block, 0, st, gathered, v, obs, reward, terminated,
                         truncated, terminal_obs);
  }
  HIP_TRY(hipGetLastError());
  return GPD_OK;
}

#ifdef GPD_STAMPS
// diagnostic build only: copy the phase stamps of the last step launches to the host
int gpd_debug_stamps(unsigned long long* out_host, int n_blocks) {
  if (n_blocks > 65536) n_blocks = 65536;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_stamps), (size_t)n_blocks * kStampPhases * 8, 0,
                              hipMemcpyDeviceToHost));
  return GPD_OK;
}
#endif

#ifdef GPD_CONTACT_STATS
// diagnostic build only: read and clear the contact-solve histogram (kPcHist counters)
int gpd_debug_contact_hist(unsigned long long* out_host) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_pc_hist), kPcHist * 8, 0, hipMemcpyDeviceToHost));
  static unsigned long long zero[kPcHist] = {};
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pc_hist), zero, kPcHist * 8, 0, hipMemcpyHostToDevice));
  return GPD_OK;
}
#endif

}  // extern "C"
