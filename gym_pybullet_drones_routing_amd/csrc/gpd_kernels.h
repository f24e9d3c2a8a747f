// gpd_kernels.h — the launch-level kernels of the batched DYN path (gfx950).
//
// HBM layout (owned by the sim):
//   state  real [20][npad]   SoA: pos(3) quat_raw(4) vel(3) rpy_rates(3) ang_v(3) last_rpm(4)
//   ring   float[15][npad*A] action history ring (BaseRLAviary.action_buffer), global head
//   steps  int32[E]          per-env step_counter
//   init   real [D][10]      per-drone reset template: pos(3) quat_raw(4) rpy(3)
//   target real [D][3]       task target positions
// One lane = one drone; one 64-lane block holds floor(64/D) whole envs so that the
// per-env exchange (downwash positions, reward/done reduction) stays inside a block.
#pragma once
#include "gpd_device.h"

namespace gpd {

constexpr int kStateComps = 20;
constexpr int kRing = 15;  // ACTION_BUFFER_SIZE = ctrl_freq//2 for the default 30 Hz; runtime value below
constexpr int kWave = 64;

enum : int { TASK_NONE = 0, TASK_HOVER = 1, TASK_MULTIHOVER = 2 };

template <typename R>
struct SimView {
  R* state;               // [20][npad]
  float* ring;            // [ring_len][npad*A]
  int32_t* steps;         // [E]
  const R* init;          // [D][10]
  const R* target;        // [D][3]
  long long npad;         // component stride of `state` (elements)
  int N, D, A, W, tpb, ring_len;
  int task, autoreset, trunc_sc;
  R bound_xy;             // 1.5 (Hover) or 2.0 (MultiHover)
};

template <typename R>
struct StepIO {
  const float* actions;   // [N][A]
  float* obs;             // [N][W]
  float* reward;          // [E]
  uint8_t* term;          // [E]
  uint8_t* trunc;         // [E]
  float* terminal_obs;    // [N][W] or null
  int head;               // ring slot receiving this step's action
};

template <typename R>
__device__ __forceinline__ void load_drone(const SimView<R>& v, long long n, Drone<R>& s, R last[4]) {
  const R* st = v.state;
  const long long p = v.npad;
  s.px = st[0 * p + n]; s.py = st[1 * p + n]; s.pz = st[2 * p + n];
  s.qx = st[3 * p + n]; s.qy = st[4 * p + n]; s.qz = st[5 * p + n]; s.qw = st[6 * p + n];
  s.vx = st[7 * p + n]; s.vy = st[8 * p + n]; s.vz = st[9 * p + n];
  s.wx = st[10 * p + n]; s.wy = st[11 * p + n]; s.wz = st[12 * p + n];
  s.ax = st[13 * p + n]; s.ay = st[14 * p + n]; s.az = st[15 * p + n];
  last[0] = st[16 * p + n]; last[1] = st[17 * p + n]; last[2] = st[18 * p + n]; last[3] = st[19 * p + n];
}

template <typename R>
__device__ __forceinline__ void store_drone(const SimView<R>& v, long long n, const Drone<R>& s, const R last[4]) {
  R* st = v.state;
  const long long p = v.npad;
  st[0 * p + n] = s.px; st[1 * p + n] = s.py; st[2 * p + n] = s.pz;
  st[3 * p + n] = s.qx; st[4 * p + n] = s.qy; st[5 * p + n] = s.qz; st[6 * p + n] = s.qw;
  st[7 * p + n] = s.vx; st[8 * p + n] = s.vy; st[9 * p + n] = s.vz;
  st[10 * p + n] = s.wx; st[11 * p + n] = s.wy; st[12 * p + n] = s.wz;
  st[13 * p + n] = s.ax; st[14 * p + n] = s.ay; st[15 * p + n] = s.az;
  st[16 * p + n] = last[0]; st[17 * p + n] = last[1]; st[18 * p + n] = last[2]; st[19 * p + n] = last[3];
}

// One physics substep of every drone of the block, including the readback that precedes it
// (BaseAviary.py:343-372 loop body).  MULTI: envs have D > 1 drones and may need downwash.
template <typename R, bool MULTI>
__device__ __forceinline__ void substep_block(Drone<R>& s, const R rpm[4], const R last[4], const Consts<R>& c,
                                              R* sx, R* sy, R* sz, int tid, int base, int D) {
  R qn[4], Rm[9];
  quat_readback(s.qx, s.qy, s.qz, s.qw, qn);   // :346-347 -> :517
  quat_to_mat(qn[0], qn[1], qn[2], qn[3], Rm); // :836
  R roll = R(0), pitch = R(0), yaw;
  if (c.flags & F_GND) quat_to_euler(qn, roll, pitch, yaw);  // self.rpy used by :742
  R dw = R(0);
  if (MULTI && (c.flags & F_DW)) {
    sx[tid] = s.px; sy[tid] = s.py; sz[tid] = s.pz;
    __syncthreads();
    dw = downwash_sum(s.px, s.py, s.pz, sx, sy, sz, base, D, c);
    __syncthreads();
  }
  dyn_substep(s, qn, Rm, roll, pitch, rpm, last, dw, c);
}

// ---------------------------------------------------------------------------------------
// gpd_step: one env.step() for every env (BaseAviary.py:259-383) in ONE launch.
template <typename R, int A, bool MULTI>
__global__ __launch_bounds__(kWave) void step_kernel(SimView<R> v, StepIO<R> io, Consts<R> c) {
  __shared__ R sx[2 * kWave], sy[2 * kWave], sz[2 * kWave];  // x2: inactive tail lanes may index past tpb
  __shared__ float srew[2 * kWave], sdist[2 * kWave];
  __shared__ int sflag[2 * kWave];
  const int tid = threadIdx.x;
  const int D = MULTI ? v.D : 1;
  const int d = MULTI ? tid % D : 0;
  const int base = tid - d;
  const long long n = (long long)blockIdx.x * v.tpb + tid;
  const bool active = tid < v.tpb && n < v.N;
  const long long nn = active ? n : 0;  // inactive lanes compute on drone 0 and store nothing
  const long long e = MULTI ? nn / D : nn;

  Drone<R> s;
  R last[4];
  load_drone(v, nn, s, last);
  const int sc = v.steps[e];

  // _preprocessAction: action_buffer.append(action); rpm = HOVER_RPM*(1+0.05*a)
  float a[A];
  if (A == 4) {
    const float4 a4 = *reinterpret_cast<const float4*>(io.actions + nn * 4);
    a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
  } else {
    a[0] = io.actions[nn];
  }
  R rpm[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) rpm[k] = (R)action_to_rpm(c.hover_f32, a[A == 4 ? k : 0]);

  for (int it = 0; it < c.nsub; ++it) {
    substep_block<R, MULTI>(s, rpm, last, c, sx, sy, sz, tid, base, D);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];   // self.last_clipped_action = clipped_action  :372
  }
  // final readback (:374) -> obs / reward / done
  R qn[4], roll, pitch, yaw;
  quat_readback(s.qx, s.qy, s.qz, s.qw, qn);
  quat_to_euler(qn, roll, pitch, yaw);

  // ---- task hooks, evaluated before step_counter += PYB_STEPS_PER_CTRL (:376-382)
  float reward = -1.0f;
  bool term = false, trunc = false;
  if (v.task != TASK_NONE) {
    const R tx = v.target[d * 3 + 0] - s.px, ty = v.target[d * 3 + 1] - s.py, tz = v.target[d * 3 + 2] - s.pz;
    const R dist = g_sqrt(tx * tx + ty * ty + tz * tz);
    const R d2 = dist * dist;
    R r = R(2) - d2 * d2;
    r = r > R(0) ? r : R(0);
    const bool oob = g_abs(s.px) > v.bound_xy || g_abs(s.py) > v.bound_xy || s.pz > R(2) ||
                     g_abs(roll) > R(0.4) || g_abs(pitch) > R(0.4);
    if (MULTI) {
      srew[tid] = (float)r;
      sdist[tid] = (float)dist;
      sflag[tid] = oob ? 1 : 0;
      __syncthreads();
      if (d == 0) {
        // MultiHoverAviary: summed reward, Σ dist < 1e-4, any drone out of bounds
        float rs = 0.0f, ds = 0.0f;
        int anyo = 0;
        for (int j = 0; j < D; ++j) { rs += srew[base + j]; ds += sdist[base + j]; anyo |= sflag[base + j]; }
        reward = rs;
        term = ds < 1e-4f;
        trunc = anyo != 0 || sc >= v.trunc_sc;
        sflag[tid] = (term ? 1 : 0) | (trunc ? 2 : 0);
        srew[tid] = reward;
      }
      __syncthreads();
      const int fl = sflag[base];
      term = fl & 1;
      trunc = (fl >> 1) & 1;
      reward = srew[base];
    } else {
      reward = (float)r;
      term = dist < R(1e-4);
      trunc = oob || sc >= v.trunc_sc;
    }
  }
  const bool done = term || trunc;
  const bool do_reset = done && v.autoreset;

  if (!active) return;

  // ---- observation row: [pos, rpy, vel, ang_v] then the 15-slot action history
  float row12[12] = {(float)s.px, (float)s.py, (float)s.pz, (float)roll, (float)pitch, (float)yaw,
                     (float)s.vx, (float)s.vy, (float)s.vz, (float)s.ax, (float)s.ay, (float)s.az};
  const long long slot_stride = v.npad * A;
  // current action into the ring (deque.append)
  float* ring_cur = v.ring + (long long)io.head * slot_stride + n * A;
  if (A == 4) *reinterpret_cast<float4*>(ring_cur) = make_float4(a[0], a[1], a[2], a[3]);
  else ring_cur[0] = a[0];

  float* orow = io.obs + n * v.W;
  float* trow = (do_reset && io.terminal_obs) ? io.terminal_obs + n * v.W : nullptr;
  // history: oldest first = slots head+1 .. head+ring_len-1, then the current action
  for (int k = 0; k < v.ring_len - 1; ++k) {
    int slot = io.head + 1 + k;
    slot -= slot >= v.ring_len ? v.ring_len : 0;
    const float* src = v.ring + (long long)slot * slot_stride + n * A;
    if (A == 4) {
      const float4 h = *reinterpret_cast<const float4*>(src);
      *reinterpret_cast<float4*>(orow + 12 + k * 4) = h;
      if (trow) *reinterpret_cast<float4*>(trow + 12 + k * 4) = h;
    } else {
      orow[12 + k] = src[0];
      if (trow) trow[12 + k] = src[0];
    }
  }
  const int kc = v.ring_len - 1;
  if (A == 4) {
    const float4 h = make_float4(a[0], a[1], a[2], a[3]);
    *reinterpret_cast<float4*>(orow + 12 + kc * 4) = h;
    if (trow) *reinterpret_cast<float4*>(trow + 12 + kc * 4) = h;
  } else {
    orow[12 + kc] = a[0];
    if (trow) trow[12 + kc] = a[0];
  }

  if (do_reset) {
    // terminal row -> terminal_obs; env back to INIT_XYZS / INIT_RPYS (_housekeeping :458-477)
    if (trow) {
#pragma unroll
      for (int k = 0; k < 12; ++k) trow[k] = row12[k];
    }
    const R* ini = v.init + d * 10;
    s.px = ini[0]; s.py = ini[1]; s.pz = ini[2];
    s.qx = ini[3]; s.qy = ini[4]; s.qz = ini[5]; s.qw = ini[6];
    s.vx = s.vy = s.vz = R(0);
    s.wx = s.wy = s.wz = R(0);
    s.ax = s.ay = s.az = R(0);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = R(0);
    row12[0] = (float)ini[0]; row12[1] = (float)ini[1]; row12[2] = (float)ini[2];
    row12[3] = (float)ini[7]; row12[4] = (float)ini[8]; row12[5] = (float)ini[9];
#pragma unroll
    for (int k = 6; k < 12; ++k) row12[k] = 0.0f;
  }
  if (A == 4) {
    *reinterpret_cast<float4*>(orow + 0) = make_float4(row12[0], row12[1], row12[2], row12[3]);
    *reinterpret_cast<float4*>(orow + 4) = make_float4(row12[4], row12[5], row12[6], row12[7]);
    *reinterpret_cast<float4*>(orow + 8) = make_float4(row12[8], row12[9], row12[10], row12[11]);
  } else {
#pragma unroll
    for (int k = 0; k < 12; ++k) orow[k] = row12[k];
  }
  store_drone(v, n, s, last);
  if (d == 0) {
    io.reward[e] = reward;
    io.term[e] = term ? 1 : 0;
    io.trunc[e] = trunc ? 1 : 0;
    v.steps[e] = do_reset ? 0 : sc + c.nsub;
  }
}

// ---------------------------------------------------------------------------------------
// gpd_integrate: n_sub raw substeps with explicit per-substep RPMs, each followed by a readback.
template <typename R, bool MULTI>
__global__ __launch_bounds__(kWave) void integrate_kernel(SimView<R> v, Consts<R> c, const R* __restrict__ rpm_in,
                                                          int n_sub, R* __restrict__ traj) {
  __shared__ R sx[2 * kWave], sy[2 * kWave], sz[2 * kWave];  // x2: inactive tail lanes may index past tpb
  const int tid = threadIdx.x;
  const int D = MULTI ? v.D : 1;
  const int d = MULTI ? tid % D : 0;
  const int base = tid - d;
  const long long n = (long long)blockIdx.x * v.tpb + tid;
  const bool active = tid < v.tpb && n < v.N;
  const long long nn = active ? n : 0;
  Drone<R> s;
  R last[4];
  load_drone(v, nn, s, last);
  const long long N = v.N;
  for (int t = 0; t < n_sub; ++t) {
    R rpm[4];
    const R* src = rpm_in + ((long long)t * N + nn) * 4;
    rpm[0] = src[0]; rpm[1] = src[1]; rpm[2] = src[2]; rpm[3] = src[3];
    substep_block<R, MULTI>(s, rpm, last, c, sx, sy, sz, tid, base, D);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];
    if (traj && active) {
      R qn[4], roll, pitch, yaw;
      quat_readback(s.qx, s.qy, s.qz, s.qw, qn);
      quat_to_euler(qn, roll, pitch, yaw);
      R* o = traj + ((long long)t * N + n) * 20;
      o[0] = s.px; o[1] = s.py; o[2] = s.pz;
      o[3] = qn[0]; o[4] = qn[1]; o[5] = qn[2]; o[6] = qn[3];
      o[7] = roll; o[8] = pitch; o[9] = yaw;
      o[10] = s.vx; o[11] = s.vy; o[12] = s.vz;
      o[13] = s.ax; o[14] = s.ay; o[15] = s.az;
      o[16] = last[0]; o[17] = last[1]; o[18] = last[2]; o[19] = last[3];
    }
  }
  if (active) store_drone(v, n, s, last);
}

// ---------------------------------------------------------------------------------------
// gpd_reset: masked re-initialisation (+ reset observation rows).
template <typename R>
__global__ __launch_bounds__(256) void reset_kernel(SimView<R> v, const uint8_t* __restrict__ mask, float* obs, int head) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  const long long e = n / v.D;
  const int d = (int)(n - e * v.D);
  if (mask && mask[e] == 0) return;
  const R* ini = v.init + d * 10;
  Drone<R> s;
  s.px = ini[0]; s.py = ini[1]; s.pz = ini[2];
  s.qx = ini[3]; s.qy = ini[4]; s.qz = ini[5]; s.qw = ini[6];
  s.vx = s.vy = s.vz = R(0);
  s.wx = s.wy = s.wz = R(0);
  s.ax = s.ay = s.az = R(0);
  R last[4] = {R(0), R(0), R(0), R(0)};
  store_drone(v, n, s, last);
  if (d == 0) v.steps[e] = 0;
  if (obs) {
    float* orow = obs + n * v.W;
    orow[0] = (float)ini[0]; orow[1] = (float)ini[1]; orow[2] = (float)ini[2];
    orow[3] = (float)ini[7]; orow[4] = (float)ini[8]; orow[5] = (float)ini[9];
    for (int k = 6; k < 12; ++k) orow[k] = 0.0f;
    const int A = v.A;
    const long long slot_stride = v.npad * A;
    for (int k = 0; k < v.ring_len; ++k) {   // oldest first: the slot about to be overwritten
      int slot = head + k;
      slot -= slot >= v.ring_len ? v.ring_len : 0;
      const float* src = v.ring + (long long)slot * slot_stride + n * A;
      for (int j = 0; j < A; ++j) orow[12 + k * A + j] = src[j];
    }
  }
}

// state20 (BaseAviary._getDroneStateVector :541-561) / raw state transposes
template <typename R>
__global__ __launch_bounds__(256) void state20_kernel(SimView<R> v, R* __restrict__ out, int raw) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  Drone<R> s;
  R last[4];
  load_drone(v, n, s, last);
  R* o = out + n * 20;
  if (raw) {
    const long long p = v.npad;
    for (int k = 0; k < 20; ++k) o[k] = v.state[k * p + n];
    return;
  }
  R qn[4], roll, pitch, yaw;
  quat_readback(s.qx, s.qy, s.qz, s.qw, qn);
  quat_to_euler(qn, roll, pitch, yaw);
  o[0] = s.px; o[1] = s.py; o[2] = s.pz;
  o[3] = qn[0]; o[4] = qn[1]; o[5] = qn[2]; o[6] = qn[3];
  o[7] = roll; o[8] = pitch; o[9] = yaw;
  o[10] = s.vx; o[11] = s.vy; o[12] = s.vz;
  o[13] = s.ax; o[14] = s.ay; o[15] = s.az;
  o[16] = last[0]; o[17] = last[1]; o[18] = last[2]; o[19] = last[3];
}

template <typename R>
__global__ __launch_bounds__(256) void set_raw_kernel(SimView<R> v, const R* __restrict__ in) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  const long long p = v.npad;
  for (int k = 0; k < 20; ++k) v.state[k * p + n] = in[n * 20 + k];
}

}  // namespace gpd
