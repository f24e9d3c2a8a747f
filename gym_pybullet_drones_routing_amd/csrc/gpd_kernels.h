// gpd_kernels.h — the launch-level kernels of the batched DYN path (gfx950).
//
// HBM layout (owned by the sim):
//   state  real [npad/64][20][64]  tiled SoA: pos(3) quat_raw(4) vel(3) rpy_rates(3) ang_v(3)
//                            last_rpm(4); each 64-drone tile keeps its 20 components contiguous
//   ring   float[npad/64][L][64*A]  action history ring (BaseRLAviary.action_buffer), tiled the
//                            same way, L = ACTION_BUFFER_SIZE = ctrl_freq//2
//   ctr    int2[E]           per-env {step_counter, ring head}: the head is the ring slot that
//                            receives the env's next action.  All envs advance it in lockstep,
//                            but keeping it per env (instead of a host-side launch argument)
//                            makes gpd_step a fixed-argument launch that a hipGraph can replay.
//   init   real [D][10]      per-drone reset template: pos(3) quat_raw(4) rpy(3)
//   target real [D][3]       task target positions
//   consts Consts<real>      model constants, read through a uniform pointer
// One lane = one drone; one 64-lane block (one wave) holds whole envs (up to floor(64/D); fewer
// "thin" blocks when there are too few drones to give every CU a wave) so that the per-env
// exchange (downwash positions, reward/done reduction) stays inside a block.
//
// Observation rows are [E][D][W] row-major (W = 12 + L*A, the Gym layout).  A lane's row is W
// floats, so writing rows straight from registers would scatter 16-byte pieces over 64
// different cache lines per store instruction.  Instead the wave assembles its 64 rows in an
// LDS tile stored column-major (tile[col][lane], one pad element per column so that the
// transposed reads are bank-conflict free):
//   * the L-1 history columns are DMA'd from the ring straight into the tile with
//     global_load_lds after the first substep, so their HBM latency hides under the physics;
//   * the 12 state columns and the current action are written from registers at the end;
//   * the tile is then streamed out with coalesced write-through 16-byte (A=4) / 4-byte
//     (A=1, 3) stores.
#pragma once
#include <type_traits>
#include "gpd_ctrl.h"
#include "gpd_device.h"

namespace gpd {

constexpr int kStateComps = 20;

// Minimum waves per SIMD the compiler must fit (register budget), for occupancy experiments
// (-DGPD_INTEGRATE_WPE=n / -DGPD_STEP_WPE=n).  1 = no constraint: forcing 4 waves on the
// integrate kernel spills to scratch and measured slower (scripts/ab_raw.sh).
#ifndef GPD_INTEGRATE_WPE
#define GPD_INTEGRATE_WPE 1
#endif
#ifndef GPD_STEP_WPE
#define GPD_STEP_WPE 1
#endif
constexpr int kWave = 64;
constexpr int kPad = kWave + 1;  // tile column stride (elements)

enum : int { TASK_NONE = 0, TASK_HOVER = 1, TASK_MULTIHOVER = 2 };

// Diagnostic build only (-DGPD_STAMPS, libgpd_stamps.so): lane 0 of every block records the
// shader clock at phase boundaries of step_kernel into g_stamps[block][phase].  The shipped
// library executes no stamp.
#ifdef GPD_STAMPS
constexpr int kStampPhases = 24;   // 0..10 shader clocks; 11 / 12: s_memrealtime (100 MHz) at entry / end;
                                   // 13: rate / io wave end (realtime); 14..16: HW_ID of waves 0..2;
                                   // 17..23: io wave phases (shader clocks)
__device__ unsigned long long g_stamps[65536 * kStampPhases];
#define GPD_STAMP(k)                                                                      \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + (k)] = t_; \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#define GPD_RSTAMP(k)                                                                     \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + (k)] = t_; \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#define GPD_IOSTAMP(k)                                                                    \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                           \
    if (tid == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + 17 + (k)] = t_; \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define GPD_IOSTAMP(k) do {} while (0)
#define GPD_STAMP(k) do {} while (0)
#define GPD_RSTAMP(k) do {} while (0)
#endif

// Write-through (sc1) stores through a buffer resource.  Every launch ends with a release that
// writes the XCD L2's dirty lines back; rows stored write-through are already on their way to
// memory when the wave stores them, so less of that write-back is left for the kernel's end.
typedef int gpd_v4i __attribute__((ext_vector_type(4)));
typedef unsigned gpd_v2u __attribute__((ext_vector_type(2)));
#ifndef GPD_WT_AUX
#define GPD_WT_AUX 16   // sc1 (write-through); diagnostic builds try other cache-policy bits
#endif
// Cache policies of the step kernel's streams: the default one for cache-resident batches (the
// state, ring and rows of the last step are re-read from L2 / Infinity Cache), and STREAM for
// batches far past the 256 MB Infinity Cache: nt (nontemporal) on the state loads and the
// history LDS-DMA, sc1|nt on the write-through stores.  Measured (scripts/large_n_ab2.sh,
// profiles/r3/large_n_ab_nt.log, U[-1,1] actions): 1M envs 194 -> 145 us, 4M envs 780 -> 608 us;
// at 4096 envs the same bits cost 4.93 -> 6.31 us, hence the size-dependent choice (gpd.hip).
constexpr int kAuxWt = GPD_WT_AUX, kAuxWtStream = 18, kAuxDmaStream = 2;
template <int AUX = kAuxWt>
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gpd_v4i, v), r, off, 0, AUX);
}
template <int AUX = kAuxWt>
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, AUX);
}
template <int AUX = kAuxWt>
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, int off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(gpd_v2u, v), r, off, 0, AUX);
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) void* gbl_void_ptr;

// Downwash work split for blocks with idle lanes: with n > 0, the block's n = tpb*D drone
// pairs are spread over all 64 lanes (pair k: drone k/D of the block, neighbour k%D of its
// env), each force goes to LDS, and the drone's lane sums its D forces in the reference's
// order.  k/D = (k*dmagic) >> 20 (host-checked for k < n).
struct DwPairs {
  int n, dmagic;
};
constexpr int kPairMax = 256;

template <typename R>
struct SimView {
  R* state;               // [npad/64][20][64]
  R* ctrl;                // [npad/64][9][64] DSLPIDControl state (PID action types only, else null)
  float* ring;            // [npad/64][ring_len][64*A]
  int2* ctr;              // [E] {step_counter, ring head}
  const R* init;          // [D][10]
  const R* target;        // [D][3]
  long long npad;         // drones rounded up to whole 64-drone tiles
  int N, D, A, W, tpb, ring_len;
  int task, autoreset, trunc_sc;
  int wt;                 // write-through stores: bit 0 obs/terminal rows, bit 1 state (see store_wt);
                          // bit 2: last_clipped_action lives in the ring (store_drone_step)
  int nc_magic;           // floor(t / NC) == (t * nc_magic) >> 16 for 0 <= t < 64 (host-checked)
  DwPairs dw_pairs;       // downwash pair split (n = 0: one lane per drone loops over its env)
  R bound_xy;             // 1.5 (Hover) or 2.0 (MultiHover)
  // drone <-> drone contact (PYB*, D > 1; DcPairs): pairs per env D(D-1)/2 (0 = off), p / P magic,
  // the [P] pair table, the per-block row store for pairs past the first 64 of a block
  int dcP, dc_pmagic;
  const int* dc_tab;
  void* dc_rows;
  long long dc_row_stride;   // row-store reals per block
};

template <typename R>
struct StepIO {
  const float* actions;   // [N][A]
  float* obs;             // [N][W]
  float* reward;          // [E]
  uint8_t* term;          // [E]
  uint8_t* trunc;         // [E]
  float* terminal_obs;    // [N][W] or null
};

// Tiled SoA: component k of drone n lives at tile(n) * C*64 + k*64 + lane(n).  Every wave
// load / store of one component is still 64 consecutive elements, while each 64-drone tile's
// state (and history) is one contiguous stretch of HBM: a block streams a few large runs
// instead of one 512-B run from each of 20 (+14) widely separated arrays.
__host__ __device__ __forceinline__ long long tidx(long long n, int k, int C) {
  return (n >> 6) * (64LL * C) + k * 64 + (n & 63);
}
// ring slot `slot` of drone n (units of float, A floats per drone)
__host__ __device__ __forceinline__ long long ridx(long long n, int slot, int L, int A) {
  return ((n >> 6) * L + slot) * (64LL * A) + (n & 63) * A;
}

// Only what the dynamics reads: ang_v is write-only, last_clipped_action is read only by drag.
template <bool NT, typename R>
__device__ __forceinline__ R ldst(const R* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <typename R, bool NT = false>
__device__ __forceinline__ void load_drone(const SimView<R>& v, long long n, Drone<R>& s, R last[4], bool need_last) {
  const R* st = v.state + tidx(n, 0, kStateComps);
  s.px = ldst<NT>(st + 0 * 64); s.py = ldst<NT>(st + 1 * 64); s.pz = ldst<NT>(st + 2 * 64);
  s.qx = ldst<NT>(st + 3 * 64); s.qy = ldst<NT>(st + 4 * 64); s.qz = ldst<NT>(st + 5 * 64); s.qw = ldst<NT>(st + 6 * 64);
  s.vx = ldst<NT>(st + 7 * 64); s.vy = ldst<NT>(st + 8 * 64); s.vz = ldst<NT>(st + 9 * 64);
  s.wx = ldst<NT>(st + 10 * 64); s.wy = ldst<NT>(st + 11 * 64); s.wz = ldst<NT>(st + 12 * 64);
  s.ax = s.ay = s.az = R(0);
  if (need_last) {
    last[0] = st[16 * 64]; last[1] = st[17 * 64]; last[2] = st[18 * 64]; last[3] = st[19 * 64];
  } else {
    last[0] = last[1] = last[2] = last[3] = R(0);
  }
}

template <typename R>
__device__ __forceinline__ void load_drone_full(const SimView<R>& v, long long n, Drone<R>& s, R last[4]) {
  load_drone(v, n, s, last, true);
  const R* st = v.state + tidx(n, 0, kStateComps);
  s.ax = st[13 * 64]; s.ay = st[14 * 64]; s.az = st[15 * 64];
}

template <typename R, int AUX = kAuxWt>
__device__ __forceinline__ void store_drone_wt(const SimView<R>& v, long long n, const Drone<R>& s, const R last[4]) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(v.state, 0, (int)(kStateComps * v.npad * (long long)sizeof(R)), 0x00020000);
  int o = (int)(tidx(n, 0, kStateComps) * sizeof(R));
  const R vals[20] = {s.px, s.py, s.pz, s.qx, s.qy, s.qz, s.qw, s.vx, s.vy, s.vz,
                      s.wx, s.wy, s.wz, s.ax, s.ay, s.az, last[0], last[1], last[2], last[3]};
  const bool skip_last = (v.wt & 4) != 0;   // store_drone_step
#pragma unroll
  for (int k = 0; k < 20; ++k, o += 64 * (int)sizeof(R))
    if (k < 16 || !skip_last) store_wt<AUX>(r, o, vals[k]);
}

template <typename R, bool NT = false>
__device__ __forceinline__ void store_drone(const SimView<R>& v, long long n, const Drone<R>& s, const R last[4]) {
  R* st = v.state + tidx(n, 0, kStateComps);
  const R vals[20] = {s.px, s.py, s.pz, s.qx, s.qy, s.qz, s.qw, s.vx, s.vy, s.vz,
                      s.wx, s.wy, s.wz, s.ax, s.ay, s.az, last[0], last[1], last[2], last[3]};
#pragma unroll
  for (int k = 0; k < 20; ++k) {
    if (NT) __builtin_nontemporal_store(vals[k], st + k * 64);
    else st[k * 64] = vals[k];
  }
}

// The step kernels' state store.  With SimView::wt bit 2 (RPM / ONE_D_RPM action types without
// drag, where nothing in the step reads it) last_clipped_action is not stored: it equals
// action_to_rpm of the ring's newest slot, or 0 in an env that has not stepped since its reset,
// and last_from_ring_kernel writes it back before any reader of state[16..19] (32 B per drone
// and step less HBM traffic in f64).  The kernel marks that with ctr[E].x = 1 (mark_last_in_ring).
template <typename R, int AUX = kAuxWt>
__device__ __forceinline__ void store_drone_step(const SimView<R>& v, long long n, const Drone<R>& s,
                                                 const R last[4]) {
  if (v.wt & 2) {
    store_drone_wt<R, AUX>(v, n, s, last);
    return;
  }
  R* st = v.state + tidx(n, 0, kStateComps);
  st[0 * 64] = s.px; st[1 * 64] = s.py; st[2 * 64] = s.pz;
  st[3 * 64] = s.qx; st[4 * 64] = s.qy; st[5 * 64] = s.qz; st[6 * 64] = s.qw;
  st[7 * 64] = s.vx; st[8 * 64] = s.vy; st[9 * 64] = s.vz;
  st[10 * 64] = s.wx; st[11 * 64] = s.wy; st[12 * 64] = s.wz;
  st[13 * 64] = s.ax; st[14 * 64] = s.ay; st[15 * 64] = s.az;
  if (!(v.wt & 4)) {
    st[16 * 64] = last[0]; st[17 * 64] = last[1]; st[18 * 64] = last[2]; st[19 * 64] = last[3];
  }
}

// drone 0's lane of a step launch: the state's last_clipped_action columns are stale from here on
template <typename R>
__device__ __forceinline__ void mark_last_in_ring(const SimView<R>& v, long long n) {
  if ((v.wt & 4) && n == 0) v.ctr[v.N / v.D] = make_int2(1, 0);
}

// Workgroup barrier for LDS exchanges within a block (between its waves, or its lanes): waits for this wave's own
// LDS operations only.  __syncthreads() (a workgroup release fence) would also wait for every
// vector-memory operation in flight, including an LDS-DMA that nobody reads until much later.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS exchange among the lanes of ONE wave (the step / integrate kernels' blocks are one wave):
// a wave's LDS instructions execute in order, so a later ds_read sees an earlier ds_write of
// any lane without a wait or a hardware barrier; the fence only keeps the compiler from
// reordering the accesses.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------- drone <-> drone contact (PYB*, D > 1)
// MultiHoverAviary's drones are colliding Bullet bodies (BaseAviary.py:486-491) stepped together
// by p.stepSimulation() (:369-370).  Restatement (oracle/bullet_mb.py drone_contact; parity
// unpinned like the plane's: Bullet's GJK / EPA and its persistent manifold are not restated):
//   * broadphase (pair_near): pairs (i, j > i) of an env whose bounding spheres come within the
//     breaking threshold and that no separating axis (the two cylinder axes, the centre line)
//     keeps farther apart than it;
//   * narrowphase: Bullet's margin scheme, the CONVERGED closest points of the margin-shrunk core
//     cylinders (core_pair: cap centres, lateral surfaces, the four rims by trust-region Newton)
//     give the normal (B -> A) and distance core - 2 x margin, with thicker margins for deeper
//     overlaps (up to ~2 cm), beyond that the least overlap over the centre line and the two axes;
//   * a cap-to-cap contact adds its face manifold (face_points: four points spanning the caps'
//     overlap), each point below the breaking threshold a contact of the pair; at most four points
//     per pair (Bullet's MANIFOLD_CACHE_SIZE): with four face points the closest point replaces the
//     one sortCachedPoints would (manifold_replace);
//   * EVERY pair whose distance is below the breaking threshold is in contact (up to kDcPts
//     contacts per pair), solved in (i, j) order;
//   * rows (normal, btPlaneSpace1 friction pair) between two bodies: effective mass
//     2/m + a_A.I_A^-1 a_A + a_B.I_B^-1 a_B; the plane's rhs rules and cone (mu 0.25); projected
//     Gauss-Seidel over the env's normal rows, then friction pairs, in contact order; the env stops
//     at its largest squared residual <= resid or after `iters` iterations;
//   * island: a drone in a pair contact that touches the ground plane brings its plane rows into
//     the env's loop (plane normal rows, pair normal rows, plane friction, pair friction per
//     iteration, as Bullet solves an island), and skips its own plane solve.
// GPU layout.  The pairs of a block's whole envs are numbered p = env * P + q (P = D(D-1)/2, q the
// (i, j) index of bullet_mb.drone_contacts' order) and lane ln handles pairs ln, ln + 64, ... (chunk
// ch = p / 64).  The hot part (DcHook, every substep): the drones' centre / axis columns into LDS,
// the broadphase of every pair (the sphere test; the separating-axis tests only for pairs in
// reach), one ballot per chunk.  A wave with a pair in reach calls dc_solve (rare): its near pairs
// compacted over the lanes (in pair order, whatever chunk they come from), the narrowphase of up to
// 64 of them per pass in parallel, their contacts (closest point + face points) numbered in order
// and each set up by lane c % 64 - the first 64 in registers, later ones in a per-block global row
// store - then the Gauss-Seidel sweeps: round r solves the level-r contacts of every env at once
// (contacts of one level touch different drones), the drones' velocity deltas in LDS.  When no env
// of the wave has more than one contact (no face manifold, no island) the owner lane keeps its two
// drones' deltas in registers for the whole solve and the sweep needs no LDS at all.
template <typename R>
__device__ __forceinline__ R cyl_extent_cos(R ua, R r, R hh) {
  const R s2 = R(1) - ua * ua;
  return hh * g_abs(ua) + r * g_sqrt(s2 > R(0) ? s2 : R(0));
}
// btPlaneSpace1
template <typename R>
__device__ __forceinline__ void plane_space(const R n[3], R p[3], R q[3]) {
  if (g_abs(n[2]) > R(0.7071067811865475244008443621048490)) {
    const R a = n[1] * n[1] + n[2] * n[2];
    const R k = g_rsqrt(a);   // ~2 ulp from 1 / sqrt(a), a third of the instructions
    p[0] = R(0); p[1] = -n[2] * k; p[2] = n[1] * k;
    q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
  } else {
    const R a = n[0] * n[0] + n[1] * n[1];
    const R k = g_rsqrt(a);
    p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = R(0);
    q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
  }
}

// ---- narrowphase (oracle/bullet_mb.py core_pair / rim_newton / rim_closest / pair_geometry / face_points)
// The closest points of the margin-shrunk cores, converged: the near caps' centres, the lateral
// surfaces along the axes' closest points (closed forms), and the four rim circles against the other
// cylinder - 5 trust-region Newton steps on the rim angle from each of 16 start azimuths (k x 22.5
// deg), the smallest squared distance per rim; the first candidate within the tie of the closest
// wins.  Everything in B's frame (btPlaneSpace1(aB), aB); B's rims in A's frame (btPlaneSpace1 of A).
// A pass's near pairs split into 64 tasks each (4 rims x 16 starts) over the wave's lanes
// (dc_narrow_pass): a sparse wave (one near pair, the common case) runs ONE Newton chain of 6
// evaluations per lane (round 5: 4 starts x 8 steps, 9 evaluations).
template <typename R> struct NpTol;
template <> struct NpTol<double> { static constexpr double accept = 1e-10, same = 1e-4, tie = 1e-7; };   // RIM_ACCEPT, RIM_SAME, PAIR_TIE
template <> struct NpTol<float> { static constexpr float accept = 1e-5f, same = 1e-4f, tie = 1e-7f; };
constexpr int kRimSamples = 16, kRimIters = 5;   // RIM_SAMPLES, RIM_ITERS
template <typename R>
__device__ __forceinline__ void axial_project(R x, R y, R z, R r, R h, R& qx, R& qy, R& qz) {
  const R rho2 = x * x + y * y;
  const R f = rho2 > r * r ? r / g_sqrt(rho2) : R(1);
  qx = x * f; qy = y * f; qz = g_max1(g_min1(z, h), -h);
}
template <typename R>
__device__ __forceinline__ R axial_extent(R az, R r, R h) {
  const R s2 = R(1) - az * az;
  return h * g_abs(az) + r * g_sqrt(s2 > R(0) ? s2 : R(0));
}
// the rim point C + r (c e1 + s e2) against the axial cylinder: squared distance f, f'/2 = g and
// f''/2 = hh in the rim angle (bullet_mb._rim_eval), the point P and its projection Q
template <typename R>
struct RimEval {
  R f, g, hh, P[3], Q[3];
};
template <typename R>
__device__ __forceinline__ void rim_eval(const R C[3], const R e1[3], const R e2[3], R c, R s, R r, R h, RimEval<R>& o) {
  const R u0 = c * e1[0] + s * e2[0], u1 = c * e1[1] + s * e2[1], u2 = c * e1[2] + s * e2[2];
  const R d0 = r * (c * e2[0] - s * e1[0]), d1 = r * (c * e2[1] - s * e1[1]), d2 = r * (c * e2[2] - s * e1[2]);
  o.P[0] = C[0] + r * u0; o.P[1] = C[1] + r * u1; o.P[2] = C[2] + r * u2;
  const R rho2 = o.P[0] * o.P[0] + o.P[1] * o.P[1];
  const bool out_r = rho2 > r * r;
  const R ir = g_rsqrt(out_r ? rho2 : R(1));
  const R k = out_r ? r * ir : R(1);
  o.Q[0] = o.P[0] * k; o.Q[1] = o.P[1] * k; o.Q[2] = g_max1(g_min1(o.P[2], h), -h);
  const R e0 = o.P[0] - o.Q[0], e1_ = o.P[1] - o.Q[1], e2_ = o.P[2] - o.Q[2];
  o.f = pc_dot(e0, e1_, e2_, e0, e1_, e2_);
  o.g = pc_dot(e0, e1_, e2_, d0, d1, d2);
  const R rt = (o.P[0] * d0 + o.P[1] * d1) * (ir * ir);
  const R m0 = out_r ? d0 - k * (d0 - rt * o.P[0]) : R(0);
  const R m1 = out_r ? d1 - k * (d1 - rt * o.P[1]) : R(0);
  const R m2 = g_abs(o.P[2]) > h ? d2 : R(0);
  o.hh = pc_dot(m0, m1, m2, d0, d1, d2) - r * pc_dot(e0, e1_, e2_, u0, u1, u2);
}
// bullet_mb.rim_newton: kRimIters trust-region Newton steps on the rim angle from (c, s)
template <typename R>
__device__ __forceinline__ void rim_newton(const R C[3], const R e1[3], const R e2[3], R r, R h, R c, R s, RimEval<R>& cur) {
  constexpr R kAcc = NpTol<R>::accept;
  rim_eval(C, e1, e2, c, s, r, h, cur);
  R rad = R(0.19634954084936207);   // pi / RIM_SAMPLES
#pragma unroll 1
  for (int it = 0; it < kRimIters; ++it) {
    // -g / hh and 1 / sqrt as Newton-refined reciprocals (~1 ulp; the oracle divides)
    R d = cur.hh > R(0) ? -cur.g * g_rcp(cur.hh > R(0) ? cur.hh : R(1)) : -copysign(rad, cur.g);
    d = g_max1(g_min1(d, rad), -rad);
    R c2 = c - d * s, s2 = s + d * c;
    const R kn = g_rsqrt(c2 * c2 + s2 * s2);
    c2 = c2 * kn; s2 = s2 * kn;
    RimEval<R> nx;
    rim_eval(C, e1, e2, c2, s2, r, h, nx);
    const bool acc = nx.f < cur.f * (R(1) - kAcc);
    if (acc) { c = c2; s = s2; cur = nx; }
    rad = acc ? g_min1(R(2) * rad, R(1)) : g_abs(d) * R(0.25);
  }
}
// closest point of the cylinder (centre c, unit axis a) to x (bullet_mb.cyl_project)
template <typename R>
__device__ __forceinline__ void cyl_project(const R c[3], const R a[3], R r, R h, const R x[3], R o[3]) {
  const R dx = x[0] - c[0], dy = x[1] - c[1], dz = x[2] - c[2];
  const R t = pc_dot(dx, dy, dz, a[0], a[1], a[2]);
  const R tc = g_max1(g_min1(t, h), -h);
  R rx = dx - t * a[0], ry = dy - t * a[1], rz = dz - t * a[2];
  const R rho2 = pc_dot(rx, ry, rz, rx, ry, rz);
  const R f = rho2 > r * r ? r / g_sqrt(rho2) : R(1);
  o[0] = (c[0] + tc * a[0]) + rx * f; o[1] = (c[1] + tc * a[1]) + ry * f; o[2] = (c[2] + tc * a[2]) + rz * f;
}
// a pair in B's frame: A's centre L and axis A, B's world basis (bp, bq, ab); A's frame (ap, aq, A)
// with B's centre Lb and axis Bz in it and B's rim basis (bp2, bq2) there; the facing caps and
// which far rims (and the lateral pair) are needed (bullet_mb.core_pair)
template <typename R>
struct NpPair {
  R L[3], A[3], bp[3], bq[3], ap[3], aq[3], Lb[3], Bz[3], bp2[3], bq2[3];
  R la, sa, sb;
};
template <typename R>
__device__ __forceinline__ void np_pair(const R ca[3], const R aa[3], const R cb[3], const R ab[3], NpPair<R>& q) {
  plane_space(ab, q.bp, q.bq);
  const R lx = ca[0] - cb[0], ly = ca[1] - cb[1], lz = ca[2] - cb[2];
  q.L[0] = pc_dot(q.bp[0], q.bp[1], q.bp[2], lx, ly, lz); q.L[1] = pc_dot(q.bq[0], q.bq[1], q.bq[2], lx, ly, lz);
  q.L[2] = pc_dot(ab[0], ab[1], ab[2], lx, ly, lz);
  q.A[0] = pc_dot(q.bp[0], q.bp[1], q.bp[2], aa[0], aa[1], aa[2]); q.A[1] = pc_dot(q.bq[0], q.bq[1], q.bq[2], aa[0], aa[1], aa[2]);
  q.A[2] = pc_dot(ab[0], ab[1], ab[2], aa[0], aa[1], aa[2]);
  plane_space(q.A, q.ap, q.aq);
  q.Lb[0] = -pc_dot(q.ap[0], q.ap[1], q.ap[2], q.L[0], q.L[1], q.L[2]);
  q.Lb[1] = -pc_dot(q.aq[0], q.aq[1], q.aq[2], q.L[0], q.L[1], q.L[2]);
  q.Lb[2] = -pc_dot(q.A[0], q.A[1], q.A[2], q.L[0], q.L[1], q.L[2]);
  q.Bz[0] = q.ap[2]; q.Bz[1] = q.aq[2]; q.Bz[2] = q.A[2];
  plane_space(q.Bz, q.bp2, q.bq2);
  q.la = -q.Lb[2];
  q.sa = q.la > R(0) ? R(-1) : R(1);
  q.sb = q.L[2] >= R(0) ? R(1) : R(-1);
}
template <typename R>
__device__ __forceinline__ void np_far(const NpPair<R>& q, R r, R h, bool& far_a, bool& far_b) {
  far_a = -q.sa * q.la - h < axial_extent(q.sa * q.A[2], r, h);
  far_b = q.sb * q.L[2] - h < axial_extent(q.A[2], r, h);
}
template <typename R>
__device__ __forceinline__ void np_to_b(const NpPair<R>& q, const R v[3], R o[3]) {   // A's frame -> B's: Ma^T v + L
  o[0] = ((q.ap[0] * v[0] + q.aq[0] * v[1]) + q.A[0] * v[2]) + q.L[0];
  o[1] = ((q.ap[1] * v[0] + q.aq[1] * v[1]) + q.A[1] * v[2]) + q.L[1];
  o[2] = ((q.ap[2] * v[0] + q.aq[2] * v[1]) + q.A[2] * v[2]) + q.L[2];
}
// one rim task: rim 0/2 = A's near / far rim against B, 1/3 = B's near / far rim against A, from
// start azimuth k (k x 22.5 deg); (x on A, y on B) in B's frame and the squared distance
template <typename R>
__device__ __forceinline__ void np_rim_task(const NpPair<R>& q, int rim, int k, R r, R h, R& f, R x[3], R y[3]) {
  // bullet_mb.RIM_COS / RIM_SIN: the first quadrant's (cos, sin) turned by k / 4 quarter turns,
  // negations as 0 - x (+0.0 where the oracle's table has it)
  const R H = R(0.7071067811865475244008443621048490), C1 = R(0.92387953251128674), S1 = R(0.38268343236508978);
  const int qd = k & 3, qt = k >> 2;
  const R qc = qd == 0 ? R(1) : (qd == 1 ? C1 : (qd == 2 ? H : S1));
  const R qs = qd == 0 ? R(0) : (qd == 1 ? S1 : (qd == 2 ? H : C1));
  const R c0 = qt == 0 ? qc : (qt == 1 ? R(0) - qs : (qt == 2 ? R(0) - qc : qs));
  const R s0 = qt == 0 ? qs : (qt == 1 ? qc : (qt == 2 ? R(0) - qs : R(0) - qc));
  const bool on_a = (rim & 1) == 0;
  const R sg = on_a ? (rim < 2 ? q.sa : -q.sa) : (rim < 2 ? q.sb : -q.sb);
  const R* base = on_a ? q.L : q.Lb;
  const R* ax = on_a ? q.A : q.Bz;
  const R* e1 = on_a ? q.ap : q.bp2;
  const R* e2 = on_a ? q.aq : q.bq2;
  const R C[3] = {base[0] + sg * h * ax[0], base[1] + sg * h * ax[1], base[2] + sg * h * ax[2]};
  RimEval<R> o;
  rim_newton(C, e1, e2, r, h, c0, s0, o);
  f = o.f;
  if (on_a) {
    x[0] = o.P[0]; x[1] = o.P[1]; x[2] = o.P[2];
    y[0] = o.Q[0]; y[1] = o.Q[1]; y[2] = o.Q[2];
  } else {   // B's rim point P and A's point Q, both in A's frame
    np_to_b(q, o.Q, x);
    np_to_b(q, o.P, y);
  }
}
// the closed-form candidates 0..2 of bullet_mb.core_pair: the near caps' centres and the lateral pair
// (d = +inf where the lateral pair is not a candidate)
template <typename R>
__device__ __forceinline__ void np_closed(const NpPair<R>& q, R r, R h, bool far_a, bool far_b, R x[3][3], R y[3][3],
                                          R d[3]) {
  const R inf = R(INFINITY);
  x[0][0] = q.L[0] + q.sa * h * q.A[0]; x[0][1] = q.L[1] + q.sa * h * q.A[1]; x[0][2] = q.L[2] + q.sa * h * q.A[2];
  axial_project(x[0][0], x[0][1], x[0][2], r, h, y[0][0], y[0][1], y[0][2]);
  {
    const R yb[3] = {q.Lb[0] + q.sb * h * q.Bz[0], q.Lb[1] + q.sb * h * q.Bz[1], q.Lb[2] + q.sb * h * q.Bz[2]};
    R xa[3];
    axial_project(yb[0], yb[1], yb[2], r, h, xa[0], xa[1], xa[2]);
    np_to_b(q, xa, x[1]);
    np_to_b(q, yb, y[1]);
  }
  {
    const R b = q.A[2], dd = q.la, e = q.L[2];
    const R den = R(1) - b * b;
    R s = den > R(1e-12) ? (b * e - dd) / den : R(0);
    s = g_max1(g_min1(s, h), -h);
    const R t = g_max1(g_min1(b * s + e, h), -h);
    s = g_max1(g_min1(b * t - dd, h), -h);
    const R pa[3] = {q.L[0] + s * q.A[0], q.L[1] + s * q.A[1], q.L[2] + s * q.A[2]};
    const R wx = pa[0], wy = pa[1], wz = pa[2] - t;
    const R wn = g_sqrt(pc_dot(wx, wy, wz, wx, wy, wz));
    const bool ok = far_a && far_b && wn > R(1e-12);
    const R wd = ok ? wn : R(1);
    const R ux = wx / wd, uy = wy / wd, uz = wz / wd;
    const R xq[3] = {pa[0] - r * ux, pa[1] - r * uy, pa[2] - r * uz};
    cyl_project(q.L, q.A, r, h, xq, x[2]);
    axial_project(r * ux, r * uy, t + r * uz, r, h, y[2][0], y[2][1], y[2][2]);
    d[2] = ok ? R(0) : inf;
  }
  for (int c = 0; c < 3; ++c) {
    if (c == 2 && !(d[2] == R(0))) continue;
    const R dx = x[c][0] - y[c][0], dy = x[c][1] - y[c][1], dz = x[c][2] - y[c][2];
    d[c] = g_sqrt(pc_dot(dx, dy, dz, dx, dy, dz));
  }
}
// the least-overlap fallback of bullet_mb.pair_geometry (cores overlapping at every margin level)
template <typename R>
__device__ __forceinline__ void np_fallback(const R ca[3], const R aa[3], const R cb[3], const R ab[3], R r, R hh,
                                            R n[3], R& dist) {
  const R lx = ca[0] - cb[0], ly = ca[1] - cb[1], lz = ca[2] - cb[2];
  const R c2 = pc_dot(lx, ly, lz, lx, ly, lz);
  R best = R(0);
  bool have = false;
  for (int u = 0; u < 3; ++u) {
    R ux, uy, uz;
    if (u == 0) {
      if (!(c2 > R(1e-24))) continue;
      const R l = g_sqrt(c2);
      ux = lx / l; uy = ly / l; uz = lz / l;
    } else {
      const R* a = u == 1 ? aa : ab;
      ux = a[0]; uy = a[1]; uz = a[2];
    }
    if (pc_dot(ux, uy, uz, lx, ly, lz) < R(0)) { ux = -ux; uy = -uy; uz = -uz; }
    const R ov = (cyl_extent_cos(pc_dot(ux, uy, uz, aa[0], aa[1], aa[2]), r, hh) +
                  cyl_extent_cos(pc_dot(ux, uy, uz, ab[0], ab[1], ab[2]), r, hh)) -
                 pc_dot(ux, uy, uz, lx, ly, lz);
    if (!have || ov < best) {
      have = true;
      best = ov;
      n[0] = ux; n[1] = uy; n[2] = uz;
    }
  }
  dist = -best;
}
// bullet_mb.face_points: the face manifold of a cap-to-cap contact - four points spanning the
// overlap of the two near caps (the lens's tips on the line of the cap centres and its corners),
// each carried along n to B's and A's cap planes: point on B fp[k] and distance fd[k]; returns
// false (no points) unless the caps face each other and overlap.
template <typename R>
__device__ __forceinline__ bool face_points(const R ca[3], const R aa[3], const R cb[3], const R ab[3], const R n[3],
                                            R radius, R half_height, R mg, R fp[4][3], R fd[4]) {
  const R r = radius - mg, h = half_height - mg;
  const R sa = pc_dot(cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2], aa[0], aa[1], aa[2]) >= R(0) ? R(1) : R(-1);
  const R sb = pc_dot(ca[0] - cb[0], ca[1] - cb[1], ca[2] - cb[2], ab[0], ab[1], ab[2]) >= R(0) ? R(1) : R(-1);
  const R nuA[3] = {sa * aa[0], sa * aa[1], sa * aa[2]}, nuB[3] = {sb * ab[0], sb * ab[1], sb * ab[2]};
  const R cB[3] = {cb[0] + sb * h * ab[0], cb[1] + sb * h * ab[1], cb[2] + sb * h * ab[2]};
  const R cab[3] = {(ca[0] + sa * h * aa[0]) - cB[0], (ca[1] + sa * h * aa[1]) - cB[1], (ca[2] + sa * h * aa[2]) - cB[2]};
  const R nb = pc_dot(n[0], n[1], n[2], nuB[0], nuB[1], nuB[2]), na = -pc_dot(n[0], n[1], n[2], nuA[0], nuA[1], nuA[2]);
  const R kf = R(0.7071067811865475244008443621048490);   // FACE_COS
  const R cn = pc_dot(cab[0], cab[1], cab[2], n[0], n[1], n[2]);
  const R dl[3] = {cab[0] - cn * n[0], cab[1] - cn * n[1], cab[2] - cn * n[2]};
  const R s2 = pc_dot(dl[0], dl[1], dl[2], dl[0], dl[1], dl[2]);
  if (!(nb >= kf && na >= kf && s2 < R(4) * r * r)) return false;
  const R s = g_sqrt(s2);
  R u[3];
  if (s > R(1e-9)) {
    u[0] = dl[0] / s; u[1] = dl[1] / s; u[2] = dl[2] / s;
  } else {
    R t2[3];
    plane_space(n, u, t2);
  }
  const R v[3] = {n[1] * u[2] - n[2] * u[1], n[2] * u[0] - n[0] * u[2], n[0] * u[1] - n[1] * u[0]};
  const R w2 = r * r - R(0.25) * s2;
  const R w = g_sqrt(w2 > R(0) ? w2 : R(0));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const R cu = k == 0 ? s - r : (k == 1 ? r : R(0.5) * s);
    const R cv = k == 2 ? w : (k == 3 ? -w : R(0));
    const R p0 = cu * u[0] + cv * v[0], p1 = cu * u[1] + cv * v[1], p2 = cu * u[2] + cv * v[2];
    const R tb = -pc_dot(p0, p1, p2, nuB[0], nuB[1], nuB[2]) / nb;
    const R ta = pc_dot(cab[0] - p0, cab[1] - p1, cab[2] - p2, nuA[0], nuA[1], nuA[2]) / -na;
    const R tm = tb + mg;
    fp[k][0] = cB[0] + p0 + tm * n[0]; fp[k][1] = cB[1] + p1 + tm * n[1]; fp[k][2] = cB[2] + p2 + tm * n[2];
    fd[k] = (ta - tb) - R(2) * mg;
  }
  return true;
}
// bullet_mb.manifold_replace (btPersistentManifold::sortCachedPoints): the slot of the full cache
// (the four face points: point on B fp, distance fd) the closest point (pb, dist) replaces - never
// a cached point deeper than it, else the slot whose replacement spans the largest quad (Bullet's
// pairing of the cached points on A), the first of a tie; the ties (depth, area) keep rounding
// from deciding a symmetric manifold
template <typename R> struct MfTol;
template <> struct MfTol<double> { static constexpr double depth = 1e-6, area = 1e-4; };   // MANIFOLD_*_TIE
template <> struct MfTol<float> { static constexpr float depth = 1e-6f, area = 1e-4f; };
template <typename R>
__device__ __forceinline__ int manifold_replace(const R pb[3], R dist, const R n[3], const R fp[4][3], const R fd[4]) {
  const R nw[3] = {pb[0] + n[0] * dist, pb[1] + n[1] * dist, pb[2] + n[2] * dist};
  R ca[4][3];
  R maxpen = dist;
  int imax = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ca[k][0] = fp[k][0] + n[0] * fd[k]; ca[k][1] = fp[k][1] + n[1] * fd[k]; ca[k][2] = fp[k][2] + n[2] * fd[k];
    if (fd[k] < maxpen - MfTol<R>::depth) { maxpen = fd[k]; imax = k; }
  }
  R res[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // res_k = |(new - c_a) x (c_b - c_c)|^2, (a, b, c) = (1,3,2) (0,3,2) (0,3,1) (0,2,1)
    const int a = k == 0 ? 1 : 0, b = k < 3 ? 3 : 2, c = k < 2 ? 2 : 1;
    const R x0 = nw[0] - ca[a][0], x1 = nw[1] - ca[a][1], x2 = nw[2] - ca[a][2];
    const R y0 = ca[b][0] - ca[c][0], y1 = ca[b][1] - ca[c][1], y2 = ca[b][2] - ca[c][2];
    const R z0 = x1 * y2 - x2 * y1, z1 = x2 * y0 - x0 * y2, z2 = x0 * y1 - x1 * y0;
    res[k] = k == imax ? R(0) : pc_dot(z0, z1, z2, z0, z1, z2);
  }
  const R top = g_max1(g_max1(res[0], res[1]), g_max1(res[2], res[3])) * (R(1) - MfTol<R>::area);
  return res[0] >= top ? 0 : (res[1] >= top ? 1 : (res[2] >= top ? 2 : 3));
}
#ifndef GPD_DC_DIAG
#define GPD_DC_DIAG 0   // diagnostic builds only: 1 = broadphase only (no solve compiled),
                        // 3 = no drone contact, 6 = the solve compiled but never entered, 7 = the
                        // solve called but returning at once, 8 = narrowphase and rows, no iterations
#endif
enum { DC_CX, DC_CY, DC_CZ, DC_AX, DC_AY, DC_AZ, DC_PX, DC_PY, DC_PZ, DC_VX, DC_VY, DC_VZ, DC_WX, DC_WY, DC_WZ,
       DC_I00, DC_I01, DC_I02, DC_I11, DC_I12, DC_I22, DC_DLX, DC_DLY, DC_DLZ, DC_DAX, DC_DAY, DC_DAZ,
       DC_R0, DC_R1, DC_R3, DC_R4, DC_R6, DC_R7, DC_N };   // DC_R*: the basis entries beside the axis (Rm[2,5,8])
constexpr int kDcChunks = 32;   // pair chunks of a block: <= 64 (D-1) / 2 / 64 + 1 for D <= 64
constexpr int kDcPts = 4;       // contacts per pair: Bullet's MANIFOLD_CACHE_SIZE (bullet_mb.pair_manifold)
constexpr int kDcConPasses = kDcPts * kDcChunks;   // 64-contact passes of a block
// a near pair's narrowphase, staged for the lanes that set up its contacts' rows
enum { DS_N = 0, DS_PB = 3, DS_D = 6, DS_FP = 7, DS_FD = 19, DS_NUM = 23 };
// an island drone's plane rows (bullet_mb._plane_rows_world): world arms, rhs, 1/jacDiag, jacDiag, impulses
enum { DI_RW = 0, DI_RHS = 12, DI_JDI = 24, DI_JDN = 36, DI_LAM = 40, DI_NUM = 52 };
template <typename R>
struct DcLds {
  R dc[DC_N][kWave];                  // drone columns
  // one area, three uses at different times: a pass's narrowphases (st: normal, point, distance,
  // face points per near slot; rim: per near slot and rim the best start's (x, y) and whether the
  // rim is needed), then, after the last pass, the island drones' plane rows (isl)
  R u[DI_NUM][kWave];
  unsigned long long nearw[kDcChunks], contw[kDcConPasses];   // pairs in reach (by chunk) / contacts (by pass)
  R eres[kWave];                      // per env: this iteration's largest squared residual
  int edone[kWave];                   // per env: solve finished
  int stouch[kWave];                  // drone in a contact
  int island[kWave];                  // drone whose plane rows the solve takes (its own plane solve skipped)
  int cij[kWave], clev[kWave];        // contacts 0..63: the lane's contact (i | j << 8) and its level
  int cij1[kWave], clev1[kWave];      // contacts 64..127 (the lanes' second register row)
  int dlev[kWave];                    // per drone: the level of its last contact (level pass)
  int nsp[kWave], nsij[kWave];        // this pass's near pairs: pair index, i | j << 8
  int qmap[kDcPts * kWave];           // this pass's contacts: near slot | point << 8 (0 closest, 1..4 face)
  int npdone[kWave];                  // narrowphase: near slot resolved at an earlier margin level
  int ecnt[kWave], ek0[kWave], ek1[kWave];   // per env: contacts, their contact-index range [ek0, ek1)
};
// The Gauss-Seidel sweeps' staging (the compiled-in PYB flag-set kernels, STAGE = true; the
// run-time-flag kernels, which serve the long observation tiles, recompute instead): operands that
// do not change over a solve's iterations, formed once at the setup - the same operations on the
// same operands as the recomputation, so the same bits.
//   ig: an island drone's plane points: the inverse-inertia images of the angular Jacobians, per
//       point p: normal G (3 p ..), friction along (0,-1,0) H, along (1,0,0) K;
//   pj: a first register row's (contacts 0..63) angular Jacobians and images per direction q (n,
//       t1, t2): pj[12 q + x][contact], x = A 0..2 (r_A x d), B 3..5 (r_B x d), gA 6..8, gB 9..11.
enum { DG_G = 0, DG_H = 12, DG_K = 24, DG_NUM = 36 };
constexpr int kPj = 36;
template <typename R>
struct DcStage {
  R ig[DG_NUM][kWave];
  R pj[kPj][kWave];
};
template <typename R>
__device__ __forceinline__ DcStage<R>& dc_stage() {
  __shared__ DcStage<R> x;
  return x;
}
static_assert(DS_NUM + 4 * 7 <= DI_NUM, "narrowphase staging fits the island rows' area");
#define DC_ST(k) u[k]
#define DC_RIM(m, e) u[DS_NUM + 7 * (m) + (e)]
#define DC_ISL(k) u[k]
// one LDS block per instantiation, shared by the hook (inlined) and the solve (a call)
template <typename R>
__device__ __forceinline__ DcLds<R>& dc_lds() {
  __shared__ DcLds<R> x;
  return x;
}
// the per-block layout a kernel hands to the hook (its prologue computes it once)
struct DcPairs {
  int npairs, P, D, nch;   // pairs of the block's whole envs, per env, drones per env, chunks
  int pij[4];              // chunks 0..3: this lane's pair as (lane i) | (lane j) << 8, -1 = none
  int pmagic;              // p / P == (p * pmagic) >> 24 for p < npairs (host-checked)
  const int* tab;          // [P] pair q -> i | j << 8 (env-local drones), for chunks >= 4
  void* rows;              // this block's row store (chunks >= 1), or null
};
__device__ __forceinline__ DcPairs dc_pairs_none() {
  DcPairs dp;
  dp.npairs = dp.P = dp.nch = dp.pmagic = 0;
  dp.D = 1;
  dp.pij[0] = dp.pij[1] = dp.pij[2] = dp.pij[3] = -1;
  dp.tab = nullptr;
  dp.rows = nullptr;
  return dp;
}
// whether a kernel of flag set PF runs the drone <-> drone contact (multi-drone PYB* envs)
template <bool MULTI, int PF>
__device__ __forceinline__ bool dc_enabled(int flags) {
  return MULTI && pf_on<PF>(flags, F_BULLET) && !pf_on<PF>(flags, F_NO_DC);
}
__device__ __forceinline__ int dc_pair_lanes(const DcPairs& dp, int p);
// this lane's pair of chunk ch (registers for chunks 0..3, selects rather than a dynamic index)
__device__ __forceinline__ int dc_pair_of(const DcPairs& dp, int ch, int p) {
  if (ch >= 4) return dc_pair_lanes(dp, p);
  return ch == 0 ? dp.pij[0] : (ch == 1 ? dp.pij[1] : (ch == 2 ? dp.pij[2] : dp.pij[3]));
}
__device__ __forceinline__ int dc_pair_lanes(const DcPairs& dp, int p) {
  const int e = (p * dp.pmagic) >> 24;
  const int t = dp.tab[p - e * dp.P];
  return ((t & 255) + e * dp.D) | (((t >> 8) + e * dp.D) << 8);
}
template <typename R>
__device__ __forceinline__ DcPairs dc_pairs_for(const SimView<R>& v, int tid, int nact) {
  DcPairs dp;
  dp.P = v.dcP;
  dp.D = v.D;
  dp.npairs = v.dcP > 0 ? (nact / v.D) * v.dcP : 0;
  dp.nch = (dp.npairs + kWave - 1) / kWave;
  dp.pmagic = v.dc_pmagic;
  dp.tab = v.dc_tab;
  dp.rows = v.dc_rows ? (void*)((R*)v.dc_rows + (long long)blockIdx.x * v.dc_row_stride) : nullptr;
#pragma unroll
  for (int ch = 0; ch < 4; ++ch) {
    const int p = tid + kWave * ch;
    dp.pij[ch] = p < dp.npairs ? dc_pair_lanes(dp, p) : -1;
  }
  return dp;
}
// broadphase of the pair (i, j) (oracle/bullet_mb.py pair_near): the sphere test, then the
// separating-axis rejects; the centre / axis columns written
template <typename R>
__device__ __forceinline__ bool dc_near(const DcLds<R>& L, int i, int j, const Consts<R>& c) {
  const R ex = L.dc[DC_CX][i] - L.dc[DC_CX][j], ey = L.dc[DC_CY][i] - L.dc[DC_CY][j],
          ez = L.dc[DC_CZ][i] - L.dc[DC_CZ][j];
  const R e2 = pc_dot(ex, ey, ez, ex, ey, ez);
  if (GPD_RARE(e2 < c.dd_reach2)) {
    const R ax = L.dc[DC_AX][i], ay = L.dc[DC_AY][i], az = L.dc[DC_AZ][i];
    const R bx = L.dc[DC_AX][j], by = L.dc[DC_AY][j], bz = L.dc[DC_AZ][j];
    const R r = c.cyl_r, hh = c.cyl_hh, lim = c.brk + R(1e-9);
    const R tilt = cyl_extent_cos(pc_dot(ax, ay, az, bx, by, bz), r, hh);   // one along the other's axis
    const R ea = pc_dot(ex, ey, ez, ax, ay, az), eb = pc_dot(ex, ey, ez, bx, by, bz);
    if (g_abs(ea) - (hh + tilt) > lim) return false;
    if (g_abs(eb) - (hh + tilt) > lim) return false;
    if (e2 > R(0)) {
      const R l = g_sqrt(e2);
      const R ext = cyl_extent_cos(ea / l, r, hh) + cyl_extent_cos(eb / l, r, hh);
      if (l - ext > lim) return false;
    }
    return true;
  }
  return false;
}
// a contact's rows: directions (n, t1, t2), the arms of A (= i) and B (= j) from their COMs, rhs,
// 1/jacDiag, the normal row's jacDiag, impulses - 25 reals (the angular Jacobians r x d and their
// I_w^-1 images are formed at each use from the arms and the drones' inverse inertias, the same
// operations as at the setup, so the values are the same bit for bit)
template <typename R>
struct DcRow {
  R d[3][3], ra[3], rb[3], rhs[3], jdi[3], jdn, lam[3];
  int i, j, env, rank;
};
constexpr int kRowReal = 25, kRowLam = 22;   // reals of a row; offset of lam
// the world inverse inertias (symmetric: 00 01 02 11 12 22) of a row's two drones
template <typename R>
struct DcInv {
  R a[6], b[6];
};
template <typename R>
__device__ __forceinline__ void dc_inv(const DcLds<R>& L, int i, int j, DcInv<R>& I) {
#pragma unroll
  for (int x = 0; x < 6; ++x) { I.a[x] = L.dc[DC_I00 + x][i]; I.b[x] = L.dc[DC_I00 + x][j]; }
}
template <typename R>
__device__ __forceinline__ void dc_cross(const R r[3], const R d[3], R o[3]) {
  o[0] = r[1] * d[2] - r[2] * d[1]; o[1] = r[2] * d[0] - r[0] * d[2]; o[2] = r[0] * d[1] - r[1] * d[0];
}
template <typename R>
__device__ __forceinline__ void dc_symv(const R m[6], const R v[3], R o[3]) {
  o[0] = pc_dot(m[0], m[1], m[2], v[0], v[1], v[2]);
  o[1] = pc_dot(m[1], m[3], m[4], v[0], v[1], v[2]);
  o[2] = pc_dot(m[2], m[4], m[5], v[0], v[1], v[2]);
}
template <bool STAGE, typename R>
__device__ __forceinline__ void dc_row_setup(const DcLds<R>& L, int i, int j, const R n[3], const R pb[3], R dist,
                                             const Consts<R>& c, R inv_m, R idt, DcRow<R>& w, int slot) {
  const R pa[3] = {pb[0] + n[0] * dist, pb[1] + n[1] * dist, pb[2] + n[2] * dist};
  w.ra[0] = pa[0] - L.dc[DC_PX][i]; w.ra[1] = pa[1] - L.dc[DC_PY][i]; w.ra[2] = pa[2] - L.dc[DC_PZ][i];
  w.rb[0] = pb[0] - L.dc[DC_PX][j]; w.rb[1] = pb[1] - L.dc[DC_PY][j]; w.rb[2] = pb[2] - L.dc[DC_PZ][j];
  R t1[3], t2[3];
  plane_space(n, t1, t2);
  DcInv<R> I;
  dc_inv(L, i, j, I);
  const R dvx = L.dc[DC_VX][i] - L.dc[DC_VX][j], dvy = L.dc[DC_VY][i] - L.dc[DC_VY][j], dvz = L.dc[DC_VZ][i] - L.dc[DC_VZ][j];
  const R wa[3] = {L.dc[DC_WX][i], L.dc[DC_WY][i], L.dc[DC_WZ][i]};
  const R wb[3] = {L.dc[DC_WX][j], L.dc[DC_WY][j], L.dc[DC_WZ][j]};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const R* d = q == 0 ? n : (q == 1 ? t1 : t2);
    w.d[q][0] = d[0]; w.d[q][1] = d[1]; w.d[q][2] = d[2];
    R A[3], B[3], gA[3], gB[3];
    dc_cross(w.ra, d, A);
    dc_cross(w.rb, d, B);
    dc_symv(I.a, A, gA);
    dc_symv(I.b, B, gB);
    if (STAGE && slot >= 0) {   // a first register row: the sweeps read these instead of recomputing them
      DcStage<R>& G = dc_stage<R>();
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        G.pj[12 * q + e][slot] = A[e]; G.pj[12 * q + 3 + e][slot] = B[e];
        G.pj[12 * q + 6 + e][slot] = gA[e]; G.pj[12 * q + 9 + e][slot] = gB[e];
      }
    }
    const R jd = (inv_m + inv_m + pc_dot(A[0], A[1], A[2], gA[0], gA[1], gA[2])) + pc_dot(B[0], B[1], B[2], gB[0], gB[1], gB[2]);
    const R rel = (pc_dot(d[0], d[1], d[2], dvx, dvy, dvz) + pc_dot(A[0], A[1], A[2], wa[0], wa[1], wa[2])) -
                  pc_dot(B[0], B[1], B[2], wb[0], wb[1], wb[2]);
    // 1/jd and x/dt as Newton-refined reciprocals (jd >= 2/m > 0): ~1 ulp from the quotients
    const R inv = g_rcp(jd);
    if (q == 0) {
      const R pen = dist + c.slop;
      w.rhs[0] = pen > R(0) ? (-rel - pen * idt) * inv : (-pen * c.erp * idt - rel) * inv;
      w.jdn = jd;
    } else {
      w.rhs[q] = -rel * inv;
    }
    w.jdi[q] = inv;
    w.lam[q] = R(0);
  }
  w.i = i;
  w.j = j;
}
// a row's angular Jacobians A = r_A x d_q, B = r_B x d_q and their images I_A^-1 A, I_B^-1 B: recomputed
// from the arms and the drones' inverse inertias (rows in the row store), or read from the setup's
// staging (register rows, L.pj) - the same operations on the same operands, so the same bits
template <typename R>
struct DcJacRow {
  const DcRow<R>& w;
  const DcInv<R>& I;
  __device__ __forceinline__ void operator()(int q, R A[3], R B[3], R gA[3], R gB[3]) const {
    dc_cross(w.ra, w.d[q], A);
    dc_cross(w.rb, w.d[q], B);
    dc_symv(I.a, A, gA);
    dc_symv(I.b, B, gB);
  }
};
template <typename R>
struct DcJacLds {
  const DcStage<R>& G;
  int slot;
  __device__ __forceinline__ void operator()(int q, R A[3], R B[3], R gA[3], R gB[3]) const {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      A[e] = G.pj[12 * q + e][slot]; B[e] = G.pj[12 * q + 3 + e][slot];
      gA[e] = G.pj[12 * q + 6 + e][slot]; gB[e] = G.pj[12 * q + 9 + e][slot];
    }
  }
};
// the rows' Jacobian products and impulse application (vi / vj: the two drones' deltas, linear
// then angular)
template <typename R>
__device__ __forceinline__ R dc_jv(const DcRow<R>& w, int q, const R A[3], const R B[3], const R vi[6], const R vj[6]) {
  return (pc_dot(w.d[q][0], w.d[q][1], w.d[q][2], vi[0] - vj[0], vi[1] - vj[1], vi[2] - vj[2]) +
          pc_dot(A[0], A[1], A[2], vi[3], vi[4], vi[5])) -
         pc_dot(B[0], B[1], B[2], vj[3], vj[4], vj[5]);
}
template <typename R>
__device__ __forceinline__ void dc_apply(const DcRow<R>& w, int q, R delta, R inv_m, const R gA[3], const R gB[3], R vi[6],
                                         R vj[6]) {
  const R dm = inv_m * delta;
  vi[0] = vi[0] + w.d[q][0] * dm; vi[1] = vi[1] + w.d[q][1] * dm; vi[2] = vi[2] + w.d[q][2] * dm;
  vi[3] = vi[3] + gA[0] * delta; vi[4] = vi[4] + gA[1] * delta; vi[5] = vi[5] + gA[2] * delta;
  vj[0] = vj[0] - w.d[q][0] * dm; vj[1] = vj[1] - w.d[q][1] * dm; vj[2] = vj[2] - w.d[q][2] * dm;
  vj[3] = vj[3] - gB[0] * delta; vj[4] = vj[4] - gB[1] * delta; vj[5] = vj[5] - gB[2] * delta;
}
// one normal row (bullet_mb.drone_contact's normal loop); returns the row's squared residual
template <typename R, typename J>
__device__ __forceinline__ R dc_normal(DcRow<R>& w, R inv_m, R vi[6], R vj[6], const J& jac) {
  R A[3], B[3], gA[3], gB[3];
  jac(0, A, B, gA, gB);
  R delta = w.rhs[0] - w.jdi[0] * dc_jv(w, 0, A, B, vi, vj);
  const R sum = w.lam[0] + delta;
  const bool neg = sum < R(0);
  delta = neg ? -w.lam[0] : delta;
  w.lam[0] = neg ? R(0) : sum;
  dc_apply(w, 0, delta, inv_m, gA, gB, vi, vj);
  const R rr = delta * w.jdn;
  return rr * rr;
}
// one friction pair on the cone (only while the normal impulse is positive); squared residual
template <typename R, typename J>
__device__ __forceinline__ R dc_friction(DcRow<R>& w, R mu, R inv_m, R vi[6], R vj[6], const J& jac) {
  if (!(w.lam[0] > R(0))) return R(0);
  R A1[3], B1[3], gA1[3], gB1[3], A2[3], B2[3], gA2[3], gB2[3];
  jac(1, A1, B1, gA1, gB1);
  jac(2, A2, B2, gA2, gB2);
  const R lim = mu * w.lam[0];
  R s1 = w.lam[1] + (w.rhs[1] - w.jdi[1] * dc_jv(w, 1, A1, B1, vi, vj));
  R s2 = w.lam[2] + (w.rhs[2] - w.jdi[2] * dc_jv(w, 2, A2, B2, vi, vj));
  const R m2 = s1 * s1 + s2 * s2;
  if (m2 > lim * lim) {
    const R f = lim * g_rsqrt1(m2);   // one Newton step: ~1e-14 relative on the projected impulse
    s1 = s1 * f;
    s2 = s2 * f;
  }
  const R e1 = s1 - w.lam[1], e2 = s2 - w.lam[2];
  w.lam[1] = s1;
  w.lam[2] = s2;
  dc_apply(w, 1, e1, inv_m, gA1, gB1, vi, vj);
  dc_apply(w, 2, e2, inv_m, gA2, gB2, vi, vj);
  const R rr = e1 + e2;
  return rr * rr;
}
// the row store: per chunk, element x of lane ln at chunk[x * 64 + ln] (kRowReal reals), then the
// four ints (i, j, env, rank) at ints[k * 64 + ln] behind them
template <typename R>
__device__ __forceinline__ void dc_row_store(R* chunk, int ln, const DcRow<R>& w) {
  const R* src = &w.d[0][0];
#pragma unroll
  for (int x = 0; x < kRowReal; ++x) chunk[x * kWave + ln] = src[x];
  int* di = reinterpret_cast<int*>(chunk + kRowReal * kWave);
  di[ln] = w.i; di[kWave + ln] = w.j; di[2 * kWave + ln] = w.env; di[3 * kWave + ln] = w.rank;
}
template <typename R>
__device__ __forceinline__ void dc_row_load(const R* chunk, int ln, DcRow<R>& w) {
  R* dst = &w.d[0][0];
#pragma unroll
  for (int x = 0; x < kRowReal; ++x) dst[x] = chunk[x * kWave + ln];
  const int* si = reinterpret_cast<const int*>(chunk + kRowReal * kWave);
  w.i = si[ln]; w.j = si[kWave + ln]; w.env = si[2 * kWave + ln]; w.rank = si[3 * kWave + ln];
}
// R elements of one row in the store: kRowReal reals + 4 ints, column-major over the chunk's 64 lanes
template <typename R>
__host__ __device__ constexpr int dc_row_reals() { return kRowReal + (4 * 4 + (int)sizeof(R) - 1) / (int)sizeof(R); }
constexpr int kDcRegRows = 2;   // contacts 0..127 of a block in the lanes' registers (two rows a lane)

// the setup and solve: a call, so that its registers stay out of the substep loop that almost
// never enters it (the caller parks its own values in LDS around it: bullet_substep)
#ifndef GPD_DC_INLINE
#define GPD_DC_INLINE 0   // A/B builds: 1 = the solve inlined at each substep call site
#endif
#if GPD_DC_INLINE
#define GPD_DC_ATTR __forceinline__
#else
#define GPD_DC_ATTR __noinline__
#endif
// wave-wide exclusive prefix sum of small non-negative ints (and the total)
__device__ __forceinline__ int wave_excl_scan(int x, int ln, int& total) {
  int v = x;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(v, o);
    if (ln >= o) v += y;
  }
  total = __shfl(v, kWave - 1);
  return v - x;
}
// an island drone's plane rows (bullet_mb._plane_rows_world; plane_contact_regs' world form): lane ln's
// columns of L.isl; returns whether any of its four points is active
template <bool STAGE, typename R>
__device__ __forceinline__ bool island_rows(DcLds<R>& L, int ln, const Consts<R>& c, R inv_m, R idt) {
  const R Rm[9] = {L.dc[DC_R0][ln], L.dc[DC_R1][ln], L.dc[DC_AX][ln], L.dc[DC_R3][ln], L.dc[DC_R4][ln],
                   L.dc[DC_AY][ln], L.dc[DC_R6][ln], L.dc[DC_R7][ln], L.dc[DC_AZ][ln]};
  const R i00 = L.dc[DC_I00][ln], i01 = L.dc[DC_I01][ln], i02 = L.dc[DC_I02][ln], i11 = L.dc[DC_I11][ln],
          i12 = L.dc[DC_I12][ln], i22 = L.dc[DC_I22][ln];
  const R px = L.dc[DC_PX][ln], py = L.dc[DC_PY][ln], pz = L.dc[DC_PZ][ln];
  const R vx = L.dc[DC_VX][ln], vy = L.dc[DC_VY][ln], vz = L.dc[DC_VZ][ln];
  const R wx = L.dc[DC_WX][ln], wy = L.dc[DC_WY][ln], wz = L.dc[DC_WZ][ln];
  const R zc = (-Rm[8] < R(0) ? -c.cyl_hh : c.cyl_hh) + c.cyl_zoff;
  const R cr = c.cyl_r;
  bool any = false;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const R rx = p == 0 ? cr : (p == 2 ? -cr : R(0)), ry = p == 1 ? cr : (p == 3 ? -cr : R(0));
    const R rwx = pc_dot(Rm[0], Rm[1], Rm[2], rx, ry, zc);
    const R rwy = pc_dot(Rm[3], Rm[4], Rm[5], rx, ry, zc);
    const R rwz = pc_dot(Rm[6], Rm[7], Rm[8], rx, ry, zc);
    L.DC_ISL(DI_RW + 3 * p)[ln] = rwx; L.DC_ISL(DI_RW + 3 * p + 1)[ln] = rwy; L.DC_ISL(DI_RW + 3 * p + 2)[ln] = rwz;
    const R dist = pz + rwz;
    const bool act = dist < c.brk && g_abs(px + rwx) <= c.plane_half && g_abs(py + rwy) <= c.plane_half;
    any = any || act;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const R ax = j == 0 ? rwy : (j == 1 ? rwz : R(0));
      const R ay = j == 0 ? -rwx : (j == 1 ? R(0) : rwz);
      const R az = j == 0 ? R(0) : (j == 1 ? -rwx : -rwy);
      const R gx = pc_dot(i00, i01, i02, ax, ay, az), gy = pc_dot(i01, i11, i12, ax, ay, az),
              gz = pc_dot(i02, i12, i22, ax, ay, az);
      if (STAGE) {
        DcStage<R>& G = dc_stage<R>();
        const int gk = (j == 0 ? DG_G : (j == 1 ? DG_H : DG_K)) + 3 * p;
        G.ig[gk][ln] = gx; G.ig[gk + 1][ln] = gy; G.ig[gk + 2][ln] = gz;
      }
      const R jd = inv_m + pc_dot(ax, ay, az, gx, gy, gz);
      const R inv = g_rcp(jd);
      const R vl = j == 0 ? vz : (j == 1 ? -vy : vx);
      const R rel = vl + pc_dot(ax, ay, az, wx, wy, wz);
      R r;
      if (j == 0) {
        const R pen = dist + c.slop;
        r = pen > R(0) ? (-rel - pen * idt) * inv : (-pen * c.erp * idt - rel) * inv;
        L.DC_ISL(DI_JDN + p)[ln] = act ? jd : R(0);
      } else {
        r = -rel * inv;
      }
      L.DC_ISL(DI_JDI + 3 * p + j)[ln] = act ? inv : R(0);
      L.DC_ISL(DI_RHS + 3 * p + j)[ln] = act ? r : R(0);
      L.DC_ISL(DI_LAM + 3 * p + j)[ln] = R(0);
    }
  }
  return any;
}
// one sweep of an island drone's plane rows (normal rows or friction pairs) on its LDS deltas;
// returns the largest squared residual.  Branch-free: every operand is loaded before the chain
// starts, and a point the oracle skips (inactive: no row; a friction pair whose normal impulse is
// not positive) takes a zero step - the same values bit for bit (x + 0 * y == x for finite y).
template <bool STAGE, typename R>
__device__ __forceinline__ R island_sweep(DcLds<R>& L, int ln, bool friction, R mu, R inv_m) {
  const DcStage<R>& G = dc_stage<R>();
  R dl0 = L.dc[DC_DLX][ln], dl1 = L.dc[DC_DLY][ln], dl2 = L.dc[DC_DLZ][ln];
  R da0 = L.dc[DC_DAX][ln], da1 = L.dc[DC_DAY][ln], da2 = L.dc[DC_DAZ][ln];
  const R i00 = L.dc[DC_I00][ln], i01 = L.dc[DC_I01][ln], i02 = L.dc[DC_I02][ln], i11 = L.dc[DC_I11][ln],
          i12 = L.dc[DC_I12][ln], i22 = L.dc[DC_I22][ln];
  R rw[4][3], lam[4][3], rhs[4][3], jdi[4][3], jdn[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      rw[p][e] = L.DC_ISL(DI_RW + 3 * p + e)[ln];
      lam[p][e] = L.DC_ISL(DI_LAM + 3 * p + e)[ln];
      rhs[p][e] = L.DC_ISL(DI_RHS + 3 * p + e)[ln];
      jdi[p][e] = L.DC_ISL(DI_JDI + 3 * p + e)[ln];
    }
    jdn[p] = L.DC_ISL(DI_JDN + p)[ln];
  }
  R res = R(0);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    // a point no island lane of the wave has a row for (inactive, or a friction pair whose normal
    // impulse is not positive) is skipped by the whole wave: its zero step changes nothing
    if (__ballot(friction ? lam[p][0] > R(0) : jdn[p] > R(0)) == 0ull) continue;
    const R rwx = rw[p][0], rwy = rw[p][1], rwz = rw[p][2];
    if (!friction) {
      // an inactive point has rhs = jdi = jdn = 0 and lam = 0: delta = 0
      const R ax = rwy, ay = -rwx;
      const R g0 = STAGE ? G.ig[DG_G + 3 * p][ln] : pc_dot(i00, i01, i02, ax, ay, R(0));
      const R g1 = STAGE ? G.ig[DG_G + 3 * p + 1][ln] : pc_dot(i01, i11, i12, ax, ay, R(0));
      const R g2 = STAGE ? G.ig[DG_G + 3 * p + 2][ln] : pc_dot(i02, i12, i22, ax, ay, R(0));
      const R jv = dl2 + (ax * da0 + ay * da1);
      R delta = rhs[p][0] - jdi[p][0] * jv;
      const R sum = lam[p][0] + delta;
      const bool neg = sum < R(0);
      delta = neg ? -lam[p][0] : delta;
      lam[p][0] = neg ? R(0) : sum;
      dl2 = dl2 + inv_m * delta;
      da0 = da0 + g0 * delta;
      da1 = da1 + g1 * delta;
      da2 = da2 + g2 * delta;
      const R rr = delta * jdn[p];
      res = g_fmax(res, rr * rr);
    } else {
      const R lnrm = lam[p][0];
      const bool act = lnrm > R(0);
      const R lim = mu * lnrm;
      const R l1 = lam[p][1], l2 = lam[p][2];
      // (0,-1,0): a = (rz, 0, -rx); (1,0,0): a = (0, rz, -ry)
      const R h0 = STAGE ? G.ig[DG_H + 3 * p][ln] : pc_dot(i00, i01, i02, rwz, R(0), -rwx);
      const R h1 = STAGE ? G.ig[DG_H + 3 * p + 1][ln] : pc_dot(i01, i11, i12, rwz, R(0), -rwx);
      const R h2 = STAGE ? G.ig[DG_H + 3 * p + 2][ln] : pc_dot(i02, i12, i22, rwz, R(0), -rwx);
      const R k0 = STAGE ? G.ig[DG_K + 3 * p][ln] : pc_dot(i00, i01, i02, R(0), rwz, -rwy);
      const R k1 = STAGE ? G.ig[DG_K + 3 * p + 1][ln] : pc_dot(i01, i11, i12, R(0), rwz, -rwy);
      const R k2 = STAGE ? G.ig[DG_K + 3 * p + 2][ln] : pc_dot(i02, i12, i22, R(0), rwz, -rwy);
      const R j1 = (rwz * da0 - rwx * da2) - dl1;
      const R j2 = (rwz * da1 - rwy * da2) + dl0;
      R s1 = l1 + (rhs[p][1] - jdi[p][1] * j1);
      R s2 = l2 + (rhs[p][2] - jdi[p][2] * j2);
      const R m2 = s1 * s1 + s2 * s2;
      const bool cap = m2 > lim * lim;
      const R f = cap ? lim * g_rsqrt1(cap ? m2 : R(1)) : R(1);
      s1 = s1 * f;
      s2 = s2 * f;
      const R d1 = act ? s1 - l1 : R(0), d2 = act ? s2 - l2 : R(0);
      lam[p][1] = act ? s1 : l1;
      lam[p][2] = act ? s2 : l2;
      dl1 = dl1 - inv_m * d1;
      dl0 = dl0 + inv_m * d2;
      da0 = da0 + h0 * d1;
      da1 = da1 + h1 * d1;
      da2 = da2 + h2 * d1;
      da0 = da0 + k0 * d2;
      da1 = da1 + k1 * d2;
      da2 = da2 + k2 * d2;
      const R rr = d1 + d2;
      res = g_fmax(res, rr * rr);
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (!friction) {
      L.DC_ISL(DI_LAM + 3 * p)[ln] = lam[p][0];
    } else {
      L.DC_ISL(DI_LAM + 3 * p + 1)[ln] = lam[p][1];
      L.DC_ISL(DI_LAM + 3 * p + 2)[ln] = lam[p][2];
    }
  }
  L.dc[DC_DLX][ln] = dl0; L.dc[DC_DLY][ln] = dl1; L.dc[DC_DLZ][ln] = dl2;
  L.dc[DC_DAX][ln] = da0; L.dc[DC_DAY][ln] = da1; L.dc[DC_DAZ][ln] = da2;
  return res;
}
template <typename R>
__device__ __forceinline__ void eres_max(DcLds<R>& L, int env, R rr) {
  // the max through an LDS atomic on the bit pattern (non-negative floats order as unsigned integers)
  if (sizeof(R) == 8)
    atomicMax(reinterpret_cast<unsigned long long*>(&L.eres[env]), (unsigned long long)__double_as_longlong((double)rr));
  else
    atomicMax(reinterpret_cast<unsigned int*>(&L.eres[env]), (unsigned int)__float_as_uint((float)rr));
}
// The narrowphases of a pass's nthis near pairs (L.nsij[0..nthis)): bullet_mb.pair_geometry per pair,
// its 4 x 16 rim Newton chains as 64 tasks over the lanes (task t: slot t / 64, rim (t / 16) % 4,
// start t % 16; the best start per rim by a butterfly over 16 lanes, ties to the lower start), the
// closed-form candidates and the selection by the pair's own lane (lane = slot), margin level by
// margin level while some pair's cores overlap; then the fallback and the face manifold.  Lane
// ln < nthis stages its pair's result in L.st and its face-point mask in L.nsp[ln] and returns its
// contact count.  dc_narrow_pass: a call, so its registers stay out of dc_solve's Gauss-Seidel
// loops; dc_solve_body<.., INL = true> inlines it (see DcHookT).
template <typename R>
__device__ __forceinline__ int dc_narrow_pass_body(const Consts<R>* cp, int ln, int nthis) {
  DcLds<R>& L = dc_lds<R>();
  const Consts<R>& c = *cp;
#ifdef GPD_CONTACT_STATS
  unsigned long long tn0 = __builtin_readcyclecounter(), tn_task = 0, tn_sel = 0;
#endif
  const R margins[4] = {R(0.001), R(0.003), R(0.006), R(0.011)};
  const bool mine = ln < nthis;
  const int pij = mine ? L.nsij[ln] : 0;
  const int mi = pij & 255, mj = pij >> 8;
  const R ca[3] = {L.dc[DC_CX][mi], L.dc[DC_CY][mi], L.dc[DC_CZ][mi]}, aa[3] = {L.dc[DC_AX][mi], L.dc[DC_AY][mi], L.dc[DC_AZ][mi]};
  const R cb[3] = {L.dc[DC_CX][mj], L.dc[DC_CY][mj], L.dc[DC_CZ][mj]}, ab[3] = {L.dc[DC_AX][mj], L.dc[DC_AY][mj], L.dc[DC_AZ][mj]};
  NpPair<R> own;
  np_pair(ca, aa, cb, ab, own);
  bool found = !mine;
  R n[3] = {R(0), R(0), R(1)}, pb[3] = {R(0), R(0), R(0)}, dist = R(0), mgf = R(-1);
  R yl[3] = {R(0), R(0), R(0)};
  L.npdone[ln] = found ? 1 : 0;
  wave_lds_sync();
  const int ntask = nthis * 64;
#pragma unroll 1
  for (int lv = 0; lv < 4; ++lv) {
    if (__ballot(!found) == 0ull) break;
    const R mg = margins[lv], r = c.cyl_r - mg, h = c.cyl_hh - mg;
#pragma unroll 1
    for (int t0 = 0; t0 < ntask; t0 += kWave) {
      const int t = t0 + ln;
      // task t: slot t / 64, rim (t / 16) % 4, start t % 16 (bullet_mb.RIM_STARTS)
      const int slot = (t >> 6) & 63, rim = (t >> 4) & 3, k = t & 15;
      R f = R(INFINITY), x[3] = {R(0), R(0), R(0)}, y[3] = {R(0), R(0), R(0)};
      bool need = false;
      if (t < ntask && !L.npdone[slot]) {
        const int pj = L.nsij[slot];
        const int ti = pj & 255, tj = pj >> 8;
        const R tca[3] = {L.dc[DC_CX][ti], L.dc[DC_CY][ti], L.dc[DC_CZ][ti]};
        const R taa[3] = {L.dc[DC_AX][ti], L.dc[DC_AY][ti], L.dc[DC_AZ][ti]};
        const R tcb[3] = {L.dc[DC_CX][tj], L.dc[DC_CY][tj], L.dc[DC_CZ][tj]};
        const R tab[3] = {L.dc[DC_AX][tj], L.dc[DC_AY][tj], L.dc[DC_AZ][tj]};
        NpPair<R> q;
        np_pair(tca, taa, tcb, tab, q);
        bool far_a, far_b;
        np_far(q, r, h, far_a, far_b);
        need = rim < 2 || (rim == 2 ? far_a : far_b);
        if (need) np_rim_task(q, rim, k, r, h, f, x, y);
      }
      // the rim's result: the lowest start within RIM_SAME of the group's smallest f (bullet_mb.rim_closest)
      R fmin = f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) fmin = g_min1(fmin, __shfl_xor(fmin, o));
      const unsigned long long near = __ballot(f <= fmin * (R(1) + NpTol<R>::same));
      const int g0 = ln & ~15;
      const int src = g0 + __builtin_ctz((unsigned)((near >> g0) & 0xffffull) | 0x10000u);
#pragma unroll
      for (int e = 0; e < 3; ++e) { x[e] = __shfl(x[e], src); y[e] = __shfl(y[e], src); }
      if (t < ntask && (t & 15) == 0) {
#pragma unroll
        for (int e = 0; e < 3; ++e) { L.DC_RIM(rim, e)[slot] = x[e]; L.DC_RIM(rim, 3 + e)[slot] = y[e]; }
        L.DC_RIM(rim, 6)[slot] = need ? R(0) : R(INFINITY);   // a rim the pair does not need
      }
    }
    wave_lds_sync();
#ifdef GPD_CONTACT_STATS
    const unsigned long long tn1 = __builtin_readcyclecounter();
    tn_task += tn1 - tn0;
#endif
    if (!found) {
      bool far_a, far_b;
      np_far(own, r, h, far_a, far_b);
      R cx[3][3], cy[3][3], cd[3];
      np_closed(own, r, h, far_a, far_b, cx, cy, cd);
      R ds[7];
      ds[0] = cd[0]; ds[1] = cd[1]; ds[2] = cd[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const R dx = L.DC_RIM(m, 0)[ln] - L.DC_RIM(m, 3)[ln], dy = L.DC_RIM(m, 1)[ln] - L.DC_RIM(m, 4)[ln],
                dz = L.DC_RIM(m, 2)[ln] - L.DC_RIM(m, 5)[ln];
        ds[3 + m] = L.DC_RIM(m, 6)[ln] == R(0) ? g_sqrt(pc_dot(dx, dy, dz, dx, dy, dz)) : R(INFINITY);
      }
      R dmin = ds[0];
#pragma unroll
      for (int m = 1; m < 7; ++m) dmin = g_min1(dmin, ds[m]);
      const R lim = dmin + NpTol<R>::tie;
      int w = 6;
#pragma unroll
      for (int m = 6; m >= 0; --m) w = ds[m] <= lim ? m : w;
      R bx[3], by[3], bd = ds[0];
#pragma unroll
      for (int e = 0; e < 3; ++e) { bx[e] = cx[0][e]; by[e] = cy[0][e]; }
#pragma unroll
      for (int m = 1; m < 7; ++m) {
        if (w == m) {
          bd = ds[m];
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            bx[e] = m < 3 ? cx[m < 3 ? m : 0][e] : L.DC_RIM(m >= 3 ? m - 3 : 0, e)[ln];
            by[e] = m < 3 ? cy[m < 3 ? m : 0][e] : L.DC_RIM(m >= 3 ? m - 3 : 0, 3 + e)[ln];
          }
        }
      }
      yl[0] = by[0]; yl[1] = by[1]; yl[2] = by[2];
      if (bd > R(1e-4)) {
        found = true;
        mgf = mg;
        const R ux = (bx[0] - by[0]) / bd, uy = (bx[1] - by[1]) / bd, uz = (bx[2] - by[2]) / bd;
        n[0] = (ux * own.bp[0] + uy * own.bq[0]) + uz * ab[0];
        n[1] = (ux * own.bp[1] + uy * own.bq[1]) + uz * ab[1];
        n[2] = (ux * own.bp[2] + uy * own.bq[2]) + uz * ab[2];
        const R wx = (by[0] * own.bp[0] + by[1] * own.bq[0]) + by[2] * ab[0],
                wy = (by[0] * own.bp[1] + by[1] * own.bq[1]) + by[2] * ab[1],
                wz = (by[0] * own.bp[2] + by[1] * own.bq[2]) + by[2] * ab[2];
        pb[0] = cb[0] + (wx + n[0] * mg); pb[1] = cb[1] + (wy + n[1] * mg); pb[2] = cb[2] + (wz + n[2] * mg);
        dist = bd - R(2) * mg;
#ifdef GPD_CONTACT_STATS
        atomicAdd(&g_pc_hist[249 + lv], 1ull);   // narrowphases ending at margin level lv
#endif
      }
    }
    L.npdone[ln] = found ? 1 : 0;
    wave_lds_sync();
#ifdef GPD_CONTACT_STATS
    tn0 = __builtin_readcyclecounter();
    tn_sel += tn0 - tn1;
#endif
  }
#ifdef GPD_CONTACT_STATS
  const unsigned long long tn2 = __builtin_readcyclecounter();
#endif
  if (!found) {   // cores overlapping at every level: the least-overlap fallback at the last level's point
    pb[0] = cb[0] + ((yl[0] * own.bp[0] + yl[1] * own.bq[0]) + yl[2] * ab[0]);
    pb[1] = cb[1] + ((yl[0] * own.bp[1] + yl[1] * own.bq[1]) + yl[2] * ab[1]);
    pb[2] = cb[2] + ((yl[0] * own.bp[2] + yl[1] * own.bq[2]) + yl[2] * ab[2]);
    np_fallback(ca, aa, cb, ab, c.cyl_r, c.cyl_hh, n, dist);
#ifdef GPD_CONTACT_STATS
    atomicAdd(&g_pc_hist[253], 1ull);   // narrowphases ending in the least-overlap fallback
#endif
  }
#ifdef GPD_CONTACT_STATS
  if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
    atomicAdd(&g_pc_hist[kPcNp + 0], 1ull);          // passes
    atomicAdd(&g_pc_hist[kPcNp + 1], tn_task);       // rim-task phases (all levels)
    atomicAdd(&g_pc_hist[kPcNp + 2], tn_sel);        // selections (all levels)
    atomicAdd(&g_pc_hist[kPcNp + 3], (unsigned long long)nthis);
    atomicAdd(&g_pc_hist[kPcNp + 4], __builtin_readcyclecounter() - tn2);   // fallback + face points (to here)
  }
#endif
  if (!mine) return 0;
  const R brk = c.brk;
  const bool con = dist < brk;
  R fp[4][3], fd[4];
  const bool face = con && mgf > R(0) && face_points(ca, aa, cb, ab, n, c.cyl_r, c.cyl_hh, mgf, fp, fd);
  int fmask = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m) fmask |= (face && fd[m] < brk) ? (1 << m) : 0;
  // at most four points per pair, Bullet's MANIFOLD_CACHE_SIZE (bullet_mb.pair_manifold): with all
  // four face points the closest point takes the slot btPersistentManifold::sortCachedPoints frees
  const int rep = fmask == 15 ? manifold_replace(pb, dist, n, fp, fd) : -1;
  L.DC_ST(DS_N)[ln] = n[0]; L.DC_ST(DS_N + 1)[ln] = n[1]; L.DC_ST(DS_N + 2)[ln] = n[2];
  L.DC_ST(DS_PB)[ln] = pb[0]; L.DC_ST(DS_PB + 1)[ln] = pb[1]; L.DC_ST(DS_PB + 2)[ln] = pb[2];
  L.DC_ST(DS_D)[ln] = dist;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    L.DC_ST(DS_FP + 3 * m)[ln] = fp[m][0]; L.DC_ST(DS_FP + 3 * m + 1)[ln] = fp[m][1]; L.DC_ST(DS_FP + 3 * m + 2)[ln] = fp[m][2];
    L.DC_ST(DS_FD + m)[ln] = fd[m];
  }
  L.nsp[ln] = fmask | ((rep + 1) << 4);   // reused (the pair index is no longer needed): face-point
                                          // mask, and 1 + the slot the closest point replaces (0: none)
  return con ? (rep >= 0 ? 4 : 1 + __popc(fmask)) : 0;
}
template <typename R>
__device__ __noinline__ int dc_narrow_pass(const Consts<R>* cp, int ln, int nthis) {
  return dc_narrow_pass_body<R>(cp, ln, nthis);
}
// plane: the ground plane is on (the island solve takes the plane rows of drones in a pair contact
// that touch it, bullet_mb.drone_contact(plane=True)); nact: the block's drones
template <typename R, bool STAGE, bool INL>
__device__ __forceinline__ void dc_solve_body(const Consts<R>* cp, R inv_m, R dt, int ln, DcPairs dp, bool plane) {
#ifdef GPD_CONTACT_STATS
  const unsigned long long t0 = __builtin_readcyclecounter();
  unsigned long long t1 = t0, t2 = t0, t_np = t0;
  int n_near = 0;
#endif
  DcLds<R>& L = dc_lds<R>();
  const Consts<R>& c = *cp;
  const R idt = g_rcp(dt);
  const int nenv = dp.P > 0 ? dp.npairs / dp.P : 0;
  L.dc[DC_DLX][ln] = R(0); L.dc[DC_DLY][ln] = R(0); L.dc[DC_DLZ][ln] = R(0);
  L.dc[DC_DAX][ln] = R(0); L.dc[DC_DAY][ln] = R(0); L.dc[DC_DAZ][ln] = R(0);
  L.stouch[ln] = 0;
  L.island[ln] = 0;
#if GPD_DC_DIAG == 7
  wave_lds_sync();
  return;   // diagnostic build: the call entered, nothing solved
#endif
  // ---- narrowphases: the near pairs compacted (pair order kept), near pair k to lane k % 64 of
  // pass k / 64; each contact pair emits its closest point and its face manifold's points below the
  // breaking threshold as consecutive contacts.  Contact c's rows are set up by lane c % 64: the
  // first 128 contacts in the lanes' registers (two rows a lane), later ones in the block's global
  // row store.
  int nnear = 0;
  for (int ch = 0; ch < dp.nch; ++ch) nnear += __popcll(L.nearw[ch]);
  if (ln < nenv) { L.ecnt[ln] = 0; L.ek0[ln] = 0x7fffffff; L.ek1[ln] = 0; }
  const int npass = (nnear + kWave - 1) / kWave;
  DcRow<R> w0, w1;
  bool have0 = false, have1 = false;
  w0.i = w0.j = w1.i = w1.j = 0;
  w0.rank = w1.rank = 0;
  R* rows = reinterpret_cast<R*>(dp.rows);
  constexpr int kRowR = dc_row_reals<R>();
  int ncon = 0;   // contacts emitted so far (wave-uniform)
  for (int ps = 0; ps < npass; ++ps) {
    int base = -ps * kWave;
    for (int ch = 0; ch < dp.nch; ++ch) {
      const unsigned long long nw = L.nearw[ch];
      if ((nw >> ln) & 1ull) {
        const int k = base + __popcll(nw & ((1ull << ln) - 1ull));
        if (k >= 0 && k < kWave) {
          const int p = ln + kWave * ch;
          L.nsp[k] = p;
          L.nsij[k] = dc_pair_of(dp, ch, p);
        }
      }
      base += __popcll(nw);
    }
    wave_lds_sync();
    const int nthis = nnear - ps * kWave < kWave ? nnear - ps * kWave : kWave;
#ifdef GPD_CONTACT_STATS
    n_near += ln < nthis ? 1 : 0;
#endif
    const int cnt = INL ? dc_narrow_pass_body<R>(cp, ln, nthis) : dc_narrow_pass<R>(cp, ln, nthis);
    int total;
    const int off = wave_excl_scan(cnt, ln, total);
    if (cnt > 0) {
      const int fmask = L.nsp[ln] & 15, rep = (L.nsp[ln] >> 4) - 1;
      int q = off;
      if (rep < 0) L.qmap[q++] = ln;          // the closest point first, then the face points
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if ((fmask >> m) & 1) L.qmap[q++] = m == rep ? ln : ln | ((m + 1) << 8);
    }
    wave_lds_sync();
#ifdef GPD_CONTACT_STATS
    if (ps == 0) t_np = __builtin_readcyclecounter();   // narrowphases of pass 0 done
#endif
    // the pass's contacts: contact c = ncon + q set up by lane c % 64
    for (int t = 0; t * kWave < total; ++t) {
      const int q = ((ln - ncon) & (kWave - 1)) + kWave * t;
      if (q < total) {
        const int cc = ncon + q;
        const int qm = L.qmap[q];
        const int sl = qm & 255, m = qm >> 8;
        const int pj = L.nsij[sl];
        const int i = pj & 255, j = pj >> 8;
        const R n[3] = {L.DC_ST(DS_N)[sl], L.DC_ST(DS_N + 1)[sl], L.DC_ST(DS_N + 2)[sl]};
        R pb[3], dist;
        if (m == 0) {
          pb[0] = L.DC_ST(DS_PB)[sl]; pb[1] = L.DC_ST(DS_PB + 1)[sl]; pb[2] = L.DC_ST(DS_PB + 2)[sl];
          dist = L.DC_ST(DS_D)[sl];
        } else {
          pb[0] = L.DC_ST(DS_FP + 3 * (m - 1))[sl]; pb[1] = L.DC_ST(DS_FP + 3 * (m - 1) + 1)[sl];
          pb[2] = L.DC_ST(DS_FP + 3 * (m - 1) + 2)[sl];
          dist = L.DC_ST(DS_FD + (m - 1))[sl];
        }
        DcRow<R> w;
        dc_row_setup<STAGE>(L, i, j, n, pb, dist, c, inv_m, idt, w, cc < kWave ? cc : -1);
        w.env = i / dp.D;
        w.rank = 0;   // the level pass below re-ranks when some env holds two contacts
        if (cc < kWave) {
          w0 = w;
          have0 = true;
          L.cij[ln] = pj;
        } else if (cc < kDcRegRows * kWave) {
          w1 = w;
          have1 = true;
          L.cij1[ln] = pj;
        } else {
          dc_row_store(rows + (long long)(cc / kWave - kDcRegRows) * kWave * kRowR, ln, w);
        }
        L.stouch[i] = 1;
        L.stouch[j] = 1;
        atomicAdd(&L.ecnt[w.env], 1);
        atomicMin(&L.ek0[w.env], cc);
        atomicMax(&L.ek1[w.env], cc + 1);
      }
    }
    ncon += total;
    wave_lds_sync();   // this pass's near slots and staging are rewritten by the next one
  }
  const int ncpass = (ncon + kWave - 1) / kWave;
  for (int x = ln; x < ncpass; x += kWave) {
    const int lo = x * kWave, n_in = ncon - lo;
    L.contw[x] = n_in >= kWave ? ~0ull : ((1ull << n_in) - 1ull);
  }
  // ---- the island: drones in a pair contact that touch the plane bring their plane rows
  bool isl = false;
  if (plane) {
    wave_lds_sync();
    // a drone in contact whose lowest plane candidate is above the breaking threshold has no plane
    // row (the plane solve's own gate, contact_low, with its margin): no island, rows not formed
    bool low = false;
    if (L.stouch[ln]) {
      const R r8 = L.dc[DC_AZ][ln], h67 = g_max1(g_abs(L.dc[DC_R6][ln]), g_abs(L.dc[DC_R7][ln]));
      const R zc = (-r8 < R(0) ? -c.cyl_hh : c.cyl_hh) + c.cyl_zoff;
      low = (L.dc[DC_PZ][ln] + r8 * zc) - c.cyl_r * h67 < c.brk + R(1e-6);
    }
    if (__ballot(low) != 0ull && low) isl = island_rows<STAGE>(L, ln, c, inv_m, idt);
    L.island[ln] = isl ? 1 : 0;
  }
  const bool any_isl = __ballot(isl) != 0ull;
  wave_lds_sync();
#ifdef GPD_CONTACT_STATS
  t1 = __builtin_readcyclecounter();
#endif
  // the largest contact count of an env
  int maxcnt = ln < nenv ? L.ecnt[ln] : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(maxcnt, o);
    maxcnt = x > maxcnt ? x : maxcnt;
  }
  // Gauss-Seidel levels (only when some env holds two contacts): a contact's level is one more
  // than the highest level among the earlier contacts (in (i, j) order) that share a drone with it.
  // Contacts of one level share no drone, so solving a level's contacts at once and the levels in
  // order IS the sequential sweep over the env's contacts (non-adjacent rows of disjoint drones
  // commute) - a pile of contacts through one drone still takes one round per contact, independent
  // pairs of one env take one; a pair's points (same two drones) take one round each.
  int rounds = maxcnt;
  if (maxcnt > 1) {
    L.dlev[ln] = 0;
    L.clev[ln] = 0;
    L.clev1[ln] = 0;
    wave_lds_sync();
    int lmax = ln < nenv && L.ecnt[ln] > 0 ? 1 : 0;
    if (ln < nenv && L.ecnt[ln] > 1) {
      for (int k = L.ek0[ln]; k < L.ek1[ln]; ++k) {
        int pij;
        int* ints = nullptr;
        if (k < kWave) {
          pij = L.cij[k];
        } else if (k < kDcRegRows * kWave) {
          pij = L.cij1[k - kWave];
        } else {
          ints = reinterpret_cast<int*>(rows + (long long)(k / kWave - kDcRegRows) * kWave * kRowR + kRowReal * kWave) +
                 (k & (kWave - 1));
          pij = ints[0] | (ints[kWave] << 8);
        }
        const int i = pij & 255, j = pij >> 8;
        const int li = L.dlev[i], lj = L.dlev[j];
        const int lev = (li > lj ? li : lj) + 1;
        L.dlev[i] = lev;
        L.dlev[j] = lev;
        if (k < kWave) L.clev[k] = lev - 1;
        else if (k < kDcRegRows * kWave) L.clev1[k - kWave] = lev - 1;
        else ints[3 * kWave] = lev - 1;
        lmax = lev > lmax ? lev : lmax;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int x = __shfl_xor(lmax, o);
      lmax = x > lmax ? x : lmax;
    }
    rounds = lmax;
    wave_lds_sync();
    if (have0) w0.rank = L.clev[ln];
    if (have1) w1.rank = L.clev1[ln];
  }
  const R mu = c.dd_mu, resid = c.resid, pmu = c.mu;
  const int iters = c.iters;
#ifdef GPD_CONTACT_STATS
  t2 = __builtin_readcyclecounter();
  int it_used = 0;
#endif
#if GPD_DC_DIAG == 8
  if (true) {   // diagnostic build: narrowphase and rows, no iterations
  } else
#endif
  if (maxcnt <= 1 && ncpass <= 1 && !any_isl) {
    // ---- every env has at most one contact and no island: its lane owns both drones' deltas
    R vi[6] = {R(0), R(0), R(0), R(0), R(0), R(0)}, vj[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    DcInv<R> I0;
    if (!STAGE) dc_inv(L, w0.i, w0.j, I0);
    bool done = !have0;
    for (int it = 0; it < iters; ++it) {
      if (__ballot(!done) == 0ull) break;
#ifdef GPD_CONTACT_STATS
      it_used = it + 1;
#endif
      if (!done) {
        R res;
        if (STAGE) {
          const DcJacLds<R> J0{dc_stage<R>(), ln};
          res = dc_normal(w0, inv_m, vi, vj, J0);
          res = g_fmax(res, dc_friction(w0, mu, inv_m, vi, vj, J0));
        } else {
          const DcJacRow<R> J0{w0, I0};
          res = dc_normal(w0, inv_m, vi, vj, J0);
          res = g_fmax(res, dc_friction(w0, mu, inv_m, vi, vj, J0));
        }
        done = res <= resid;
      }
    }
    if (have0) {
      L.dc[DC_DLX][w0.i] = vi[0]; L.dc[DC_DLY][w0.i] = vi[1]; L.dc[DC_DLZ][w0.i] = vi[2];
      L.dc[DC_DAX][w0.i] = vi[3]; L.dc[DC_DAY][w0.i] = vi[4]; L.dc[DC_DAZ][w0.i] = vi[5];
      L.dc[DC_DLX][w0.j] = vj[0]; L.dc[DC_DLY][w0.j] = vj[1]; L.dc[DC_DLZ][w0.j] = vj[2];
      L.dc[DC_DAX][w0.j] = vj[3]; L.dc[DC_DAY][w0.j] = vj[4]; L.dc[DC_DAZ][w0.j] = vj[5];
    }
  } else {
    // ---- general case: per phase (normal rows, then friction pairs) the island drones' plane rows
    // (one round: each drone's own rows), then round r solves the level-r contacts of every env;
    // deltas through LDS (bullet_mb.drone_contact's order: plane normal, pair normal, plane
    // friction, pair friction)
    if (ln < nenv) { L.edone[ln] = L.ecnt[ln] == 0; L.eres[ln] = R(0); }
    wave_lds_sync();
    R vi[6], vj[6];
    // one row: deltas from LDS, the row's step, deltas back; its squared residual
    auto visit = [&](DcRow<R>& w, bool friction, int slot) -> R {
#pragma unroll
      for (int x = 0; x < 6; ++x) { vi[x] = L.dc[DC_DLX + x][w.i]; vj[x] = L.dc[DC_DLX + x][w.j]; }
      R rr;
      if (STAGE && slot >= 0) {
        const DcJacLds<R> J{dc_stage<R>(), slot};
        rr = friction ? dc_friction(w, mu, inv_m, vi, vj, J) : dc_normal(w, inv_m, vi, vj, J);
      } else {
        DcInv<R> I;
        dc_inv(L, w.i, w.j, I);
        const DcJacRow<R> J{w, I};
        rr = friction ? dc_friction(w, mu, inv_m, vi, vj, J) : dc_normal(w, inv_m, vi, vj, J);
      }
#pragma unroll
      for (int x = 0; x < 6; ++x) { L.dc[DC_DLX + x][w.i] = vi[x]; L.dc[DC_DLX + x][w.j] = vj[x]; }
      return rr;
    };
    const int my_env = ln / dp.D;
#ifdef GPD_CONTACT_STATS
    unsigned long long tg_isl = 0, tg_nrm = 0, tg_fr = 0, tg_end = 0, tg0 = __builtin_readcyclecounter();
#endif
    for (int it = 0; it < iters; ++it) {
      // edone / eres of every env are settled here (the previous iteration's end)
      if (__ballot(ln < nenv && !L.edone[ln]) == 0ull) break;
#ifdef GPD_CONTACT_STATS
      it_used = it + 1;
#endif
      // the envs still iterating, read once per iteration; each lane's residuals per env in registers
      const bool live0 = have0 && !L.edone[w0.env], live1 = have1 && !L.edone[w1.env];
      const bool livei = isl && !L.edone[my_env];
      R res0 = R(0), res1 = R(0), resi = R(0);
      for (int ph = 0; ph < 2; ++ph) {              // normal rows, then friction pairs
#ifdef GPD_CONTACT_STATS
        const unsigned long long tga = __builtin_readcyclecounter();
        tg_end += tga - tg0;
#endif
        if (any_isl) {
          if (livei) resi = g_fmax(resi, island_sweep<STAGE>(L, ln, ph == 1, pmu, inv_m));
          wave_lds_sync();
        }
#ifdef GPD_CONTACT_STATS
        const unsigned long long tgb = __builtin_readcyclecounter();
        tg_isl += tgb - tga;
#endif
        for (int r = 0; r < rounds; ++r) {
          if (live0 && w0.rank == r) res0 = g_fmax(res0, visit(w0, ph == 1, ln));
          if (live1 && w1.rank == r) res1 = g_fmax(res1, visit(w1, ph == 1, -1));
          for (int ch = kDcRegRows; ch < ncpass; ++ch) {
            if (((L.contw[ch] >> ln) & 1ull) == 0) continue;
            R* chunk = rows + (long long)(ch - kDcRegRows) * kWave * kRowR;
            if (reinterpret_cast<const int*>(chunk + kRowReal * kWave)[3 * kWave + ln] != r) continue;   // its rank
            DcRow<R> w;
            dc_row_load(chunk, ln, w);
            if (L.edone[w.env]) continue;
            eres_max(L, w.env, visit(w, ph == 1, -1));
#pragma unroll
            for (int q = 0; q < 3; ++q) chunk[(kRowLam + q) * kWave + ln] = w.lam[q];
          }
          wave_lds_sync();
        }
#ifdef GPD_CONTACT_STATS
        tg0 = __builtin_readcyclecounter();
        if (ph == 0) tg_nrm += tg0 - tgb; else tg_fr += tg0 - tgb;
#endif
      }
      if (live0) eres_max(L, w0.env, res0);
      if (live1) eres_max(L, w1.env, res1);
      if (livei) eres_max(L, my_env, resi);
      wave_lds_sync();
      if (ln < nenv) {
        if (!L.edone[ln]) L.edone[ln] = L.eres[ln] <= resid;
        L.eres[ln] = R(0);
      }
      wave_lds_sync();
    }
#ifdef GPD_CONTACT_STATS
    tg_end += __builtin_readcyclecounter() - tg0;
    if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
      atomicAdd(&g_pc_hist[kPcNp + 7], tg_isl);    // general path: island sweeps
      atomicAdd(&g_pc_hist[kPcNp + 8], tg_nrm);    // normal rounds
      atomicAdd(&g_pc_hist[kPcNp + 9], tg_fr);     // friction rounds
      atomicAdd(&g_pc_hist[kPcNp + 10], tg_end);   // iteration ends (convergence checks)
      atomicAdd(&g_pc_hist[kPcNp + 11], (unsigned long long)it_used * rounds);   // rounds per phase run
      atomicAdd(&g_pc_hist[kPcNp + 12], (unsigned long long)it_used);            // general-path iterations
    }
#endif
  }
#ifdef GPD_CONTACT_STATS
  {
    const unsigned long long t3 = __builtin_readcyclecounter();
    int tot = n_near;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
      atomicAdd(&g_pc_hist[116], 1ull);
      atomicAdd(&g_pc_hist[117], t2 - t0);
      atomicAdd(&g_pc_hist[118], t3 - t2);
      atomicAdd(&g_pc_hist[119], (unsigned long long)it_used);
      atomicAdd(&g_pc_hist[123], t1 - t0);
      atomicAdd(&g_pc_hist[254], t_np - t0);   // to the end of pass 0's narrowphases
      atomicAdd(&g_pc_hist[126], (unsigned long long)ncon);
      atomicAdd(&g_pc_hist[127], (unsigned long long)tot);
      atomicAdd(&g_pc_hist[124], any_isl ? 1ull : 0ull);                                   // island solves
      atomicAdd(&g_pc_hist[125], (maxcnt <= 1 && ncpass <= 1 && !any_isl) ? 1ull : 0ull);  // register fast path
      atomicAdd(&g_pc_hist[243], (unsigned long long)rounds);                               // GS rounds per phase
      atomicMax(&g_pc_hist[255], (unsigned long long)ncon);                                 // most contacts of a solve
      atomicAdd(&g_pc_hist[kPcNp + 5], ncon > kDcRegRows * kWave ? 1ull : 0ull);           // solves using the row store
      atomicAdd(&g_pc_hist[kPcNp + 6], (unsigned long long)ncpass);
      const unsigned long long cyc = t3 - t0;
      atomicAdd(&g_pc_hist[128 + (63 - __clzll(cyc | 1ull))], 1ull);
      atomicAdd(&g_pc_hist[192 + it_used], 1ull);
      if (blockIdx.x < 4096) atomicAdd(&g_pc_hist[256 + blockIdx.x], cyc);
    }
  }
#endif
  wave_lds_sync();   // the caller reads the velocity deltas
}
// the solve as a call (its registers out of the caller's allocation; the run-time-flag kernels and
// the downwash flag sets)
template <typename R, bool STAGE>
__device__ GPD_DC_ATTR void dc_solve(const Consts<R>* cp, R inv_m, R dt, int ln, DcPairs dp, bool plane) {
  dc_solve_body<R, STAGE, false>(cp, inv_m, dt, ln, dp, plane);
}
// the hook bullet_substep calls (multi-drone envs of one-wave blocks): pk parks the caller's
// values in LDS around the solve (bullet_substep), so nothing of the substep loop is live across
// the call and the loop's own register allocation does not see the solve.  INL: the solve and its
// narrowphase inlined (no call, no callee-saved register spills): the compiled-in PYB flag sets
// without downwash - the 2-drone MultiHover PYB batch 127.1 -> 119.5 us, while the 8-drone
// PYB_GND_DRAG_DW batch, whose island sweeps then share the kernel's register allocation, went
// 3 103 -> 3 535 us (profiles/r6/contact/probe_inline_ab.log); inlined only here: 2-drone
// 126.7 -> 119.9 us, 8-drone PYB 16.3 -> 14.2 us, 8-drone PYB_GND_DRAG_DW unchanged (probe_selective_inline_ab.log)
template <bool INL>
struct DcHookT {
  int tid;
  DcPairs dp;
  // returns whether this lane's drone joined the island (its plane rows were solved here)
  template <typename R, class PK>
  __device__ __forceinline__ bool operator()(Drone<R>& s, R* Rm, const Consts<R>& c, const DynK<R>& k, const PK& pk,
                                             bool plane) const {
#if GPD_DC_DIAG == 3
    return false;   // diagnostic build: no drone contact at all (the hook compiled in, its body not)
#endif
    DcLds<R>& L = dc_lds<R>();
    const DcPairs& P = dp;
    const int ln = tid & (kWave - 1);
    const R zo = c.cyl_zoff;
    L.dc[DC_CX][ln] = s.px + Rm[2] * zo; L.dc[DC_CY][ln] = s.py + Rm[5] * zo; L.dc[DC_CZ][ln] = s.pz + Rm[8] * zo;
    L.dc[DC_AX][ln] = Rm[2]; L.dc[DC_AY][ln] = Rm[5]; L.dc[DC_AZ][ln] = Rm[8];
    wave_lds_sync();
    bool any = false, isl = false;
    for (int ch = 0; ch < P.nch; ++ch) {
      const int p = ln + kWave * ch;
      bool near = false;
      if (p < P.npairs) {
        const int pij = dc_pair_of(P, ch, p);
        near = dc_near(L, pij & 255, pij >> 8, c);
      }
      const unsigned long long w = __ballot(near);
      if (ln == 0) L.nearw[ch] = w;
      any = any || w != 0ull;
    }
#if GPD_DC_DIAG == 1
    any = false;   // diagnostic build: broadphase only, no solve
#elif GPD_DC_DIAG == 6
    any = any && (k.flags & (1 << 29)) != 0;   // diagnostic build: the solve compiled, never entered
#endif
    if (GPD_RARE(any)) {
#ifdef GPD_CONTACT_STATS
      const unsigned long long tr0 = __builtin_readcyclecounter();
#endif
      // this lane's columns for the solve: pose, velocities, world inverse inertia R diag(1/I) R^T
      const R q00 = k.ijx * Rm[0], q01 = k.ijy * Rm[1], q02 = k.ijz * Rm[2];
      const R q10 = k.ijx * Rm[3], q11 = k.ijy * Rm[4], q12 = k.ijz * Rm[5];
      const R q20 = k.ijx * Rm[6], q21 = k.ijy * Rm[7], q22 = k.ijz * Rm[8];
      L.dc[DC_I00][ln] = pc_dot(q00, q01, q02, Rm[0], Rm[1], Rm[2]);
      L.dc[DC_I01][ln] = pc_dot(q00, q01, q02, Rm[3], Rm[4], Rm[5]);
      L.dc[DC_I02][ln] = pc_dot(q00, q01, q02, Rm[6], Rm[7], Rm[8]);
      L.dc[DC_I11][ln] = pc_dot(q10, q11, q12, Rm[3], Rm[4], Rm[5]);
      L.dc[DC_I12][ln] = pc_dot(q10, q11, q12, Rm[6], Rm[7], Rm[8]);
      L.dc[DC_I22][ln] = pc_dot(q20, q21, q22, Rm[6], Rm[7], Rm[8]);
      L.dc[DC_PX][ln] = s.px; L.dc[DC_PY][ln] = s.py; L.dc[DC_PZ][ln] = s.pz;
      L.dc[DC_VX][ln] = s.vx; L.dc[DC_VY][ln] = s.vy; L.dc[DC_VZ][ln] = s.vz;
      L.dc[DC_WX][ln] = s.wx; L.dc[DC_WY][ln] = s.wy; L.dc[DC_WZ][ln] = s.wz;
      L.dc[DC_R0][ln] = Rm[0]; L.dc[DC_R1][ln] = Rm[1]; L.dc[DC_R3][ln] = Rm[3];
      L.dc[DC_R4][ln] = Rm[4]; L.dc[DC_R6][ln] = Rm[6]; L.dc[DC_R7][ln] = Rm[7];
      const R inv_m = k.inv_m, dt = k.dt;
      const DcPairs dpc = P;
      wave_lds_sync();
#ifdef GPD_CONTACT_STATS
      const unsigned long long tr1 = __builtin_readcyclecounter();
#endif
      pk.park();
#ifdef GPD_CONTACT_STATS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned long long tr2 = __builtin_readcyclecounter();
#endif
      if (INL) dc_solve_body<R, PK::kStage, true>(&c, inv_m, dt, ln, dpc, plane);
      else dc_solve<R, PK::kStage>(&c, inv_m, dt, ln, dpc, plane);
#ifdef GPD_CONTACT_STATS
      const unsigned long long tr3 = __builtin_readcyclecounter();
#endif
      pk.unpark();
      isl = L.island[ln] != 0;
      if (L.stouch[ln]) {
        s.vx = s.vx + L.dc[DC_DLX][ln]; s.vy = s.vy + L.dc[DC_DLY][ln]; s.vz = s.vz + L.dc[DC_DLZ][ln];
        s.wx = s.wx + L.dc[DC_DAX][ln]; s.wy = s.wy + L.dc[DC_DAY][ln]; s.wz = s.wz + L.dc[DC_DAZ][ln];
      }
#ifdef GPD_CONTACT_STATS
      {
        const unsigned long long tr4 = __builtin_readcyclecounter();
        if (ln == 0) {
          if (blockIdx.x < 4096) atomicAdd(&g_pc_hist[256 + 12288 + blockIdx.x], tr4 - tr0);
          atomicAdd(&g_pc_hist[244], tr1 - tr0);   // columns for the solve
          atomicAdd(&g_pc_hist[245], tr2 - tr1);   // park
          atomicAdd(&g_pc_hist[246], tr3 - tr2);   // the call (the solve included)
          atomicAdd(&g_pc_hist[247], tr4 - tr3);   // unpark + deltas
          atomicAdd(&g_pc_hist[248], 1ull);
        }
      }
#endif
    }
    wave_lds_sync();   // the centre columns are rewritten by the next substep
    return isl;
  }
};

// One physics substep of every drone of the block, including the readback that precedes it
// (BaseAviary.py:343-372 loop body).  MULTI: envs have D > 1 drones and may need downwash.
template <typename R, bool MULTI, int PF, bool ANGV = true>
__device__ __forceinline__ void substep_block(Drone<R>& s, R rpm[4], R W[4], R last[4],
                                              const Consts<R>& c, DynK<R>& k, R* sx, R* sy, R* sz, int tid,
                                              int base, int D, DwPairs pairs, R* spair, const DcPairs& dcp) {
  R dw = R(0);
  if (MULTI && pf_on<PF>(k.flags, F_DW)) {
    sx[tid] = s.px; sy[tid] = s.py; sz[tid] = s.pz;
    wave_lds_sync();
    if (pairs.n > 0) {
      for (int p = tid; p < pairs.n; p += kWave) {
        const int i = (p * pairs.dmagic) >> 20;          // drone of the block
        const int j = p - i * D;                          // neighbour within its env
        const int ib = ((i * pairs.dmagic) >> 20) * D;   // the env's first drone in the block
        spair[p] = dw_pair(sx[i], sy[i], sz[i], sx[ib + j], sy[ib + j], sz[ib + j], c);
      }
      wave_lds_sync();
      if (tid * D < pairs.n)
        for (int j = 0; j < D; ++j) dw = dw + spair[tid * D + j];
    } else {
      dw = downwash_sum(s.px, s.py, s.pz, sx, sy, sz, base, D, c);
    }
    wave_lds_sync();
  }
  // the drone contact inlined in the compiled-in flag sets without downwash (DcHookT)
  constexpr bool kDcInl = PF != kPfRuntime && (PF & F_DW) == 0;
  if (MULTI) dyn_substep<R, PF, ANGV, 1, DcHookT<kDcInl>>(s, rpm, W, last, dw, c, k, DcHookT<kDcInl>{tid, dcp});
  else dyn_substep<R, PF, ANGV>(s, rpm, W, last, dw, c, k);
}

// Bytes of dynamic LDS the step kernel needs for its observation tile: the row's columns
// (state, history, current action).  A == 4 keeps float4 columns (state 3, history+action L);
// A == 1 / 3 keep float columns (state 12, history+action L*A).
#ifndef GPD_TILE_MIN
#define GPD_TILE_MIN 0   // diagnostic builds only: minimum LDS per block (occupancy probe)
#endif
__host__ __device__ inline int step_tile_bytes(int A, int ring_len) {
  const int b = A == 4 ? (3 + ring_len) * kPad * 16 : (12 + ring_len * A) * kPad * 4;
  return b > GPD_TILE_MIN ? b : GPD_TILE_MIN;
}

// Copy-out of the observation tile: the block's nact rows of NC columns (float4 columns for
// A == 4, float otherwise), streamed by NL lanes with coalesced (write-through with wt & 1)
// stores; rows flagged in done_rows also go to terminal_obs (their non-state columns - the
// state part was stored from registers).  t / NC is (t * nc_magic) >> 16 for t <= NL.  U tile
// elements per lane per batch (LDS reads in flight); lanes past the end are masked off.
template <int A, int NL, int U = 6, int AUX = kAuxWt>
__device__ __forceinline__ void tile_copy_out(const float4* tile4, const float* tilef, int lane, int nact, int NC,
                                              int nc_magic, int wt, unsigned long long done_rows, float* obs,
                                              float* terminal_obs, long long n0) {
  // lane `lane` streams tile elements g = lane, lane+NL, ... (row-major over the block's rows).
  // A lane whose element index passes the end reads the last element and stores nothing (an
  // exec-masked store; re-storing the last element instead would send up to NL*U writes of one
  // 16-byte word through one L2 channel).  Rows of envs that finished this step are also
  // written to terminal_obs (state columns from the extra tile columns).
  const int total = nact * NC;
  const int drow = (NL * nc_magic) >> 16, dcol = NL - drow * NC;
  int row = (lane * nc_magic) >> 16;
  int col = lane - row * NC;
  const int last_row = nact - 1, last_col = NC - 1;
  const int ncs = A == 4 ? 3 : 12;  // state columns
  for (int g0 = lane; g0 - lane < total; g0 += U * NL) {
    if (A == 4) {
      float4 val[U];
      int idx[U];
      int rr[U], cc[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = g0 + u * NL < total;
        rr[u] = ok[u] ? row : last_row;
        cc[u] = ok[u] ? col : last_col;
        val[u] = tile4[__umul24(cc[u], kPad) + rr[u]];   // 24-bit multiply: full-rate VALU
        idx[u] = ok[u] ? g0 + u * NL : total - 1;
        col += dcol; row += drow;
        if (col >= NC) { col -= NC; ++row; }
      }
      GPD_STAMP(8);
      float4* dst = reinterpret_cast<float4*>(obs) + n0 * NC;
      if (wt & 1) {
        // masked-off elements get an offset past num_records: the buffer unit drops the store
        // (no exec-mask branch per element)
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, 0, total * 16, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) store_wt<AUX>(r, ok[u] ? idx[u] * 16 : total * 16, val[u]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (ok[u]) dst[idx[u]] = val[u];
      }
      GPD_STAMP(9);
      if (done_rows) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (ok[u] && ((done_rows >> rr[u]) & 1ull)) {
            if (cc[u] >= ncs) reinterpret_cast<float4*>(terminal_obs)[n0 * NC + idx[u]] = val[u];
          }
        }
      }
    } else {
      float val[U];
      int idx[U];
      int rr[U], cc[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = g0 + u * NL < total;
        rr[u] = ok[u] ? row : last_row;
        cc[u] = ok[u] ? col : last_col;
        val[u] = tilef[__umul24(cc[u], kPad) + rr[u]];
        idx[u] = ok[u] ? g0 + u * NL : total - 1;
        col += dcol; row += drow;
        if (col >= NC) { col -= NC; ++row; }
      }
      float* dst = obs + n0 * NC;
      if (wt & 1) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, 0, total * 4, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) store_wt<AUX>(r, ok[u] ? idx[u] * 4 : total * 4, val[u]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (ok[u]) dst[idx[u]] = val[u];
      }
      if (done_rows) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (ok[u] && ((done_rows >> rr[u]) & 1ull)) {
            if (cc[u] >= ncs) terminal_obs[n0 * NC + idx[u]] = val[u];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// gpd_step: one env.step() for every env (BaseAviary.py:259-383) in ONE launch.
// ACT: action type (GPD_ACT_*); PID types run DSLPIDControl before the substeps.
// PF: the physics flags compiled in (pf_on): 0 = plain DYN (the bench path, aero / PYB-wrench code
// compiled out), a flag set for the BASELINE configs' combinations, kPfRuntime for the rest.
template <typename R, int ACT, bool MULTI, int PF, bool STREAM = false>
// STREAM: the cache policies for batches far past the Infinity Cache (kAuxWtStream above).
// The leading scalar arguments duplicate the SimView / StepIO fields the first loads need: the
// library is built with kernarg preloading, so they arrive in SGPRs at wave launch instead of
// through an s_load round trip on the kernel-argument segment before the first state load.
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(GPD_STEP_WPE))) void step_kernel(R* __restrict__ state_p, const float* __restrict__ actions_p,
                                                     int2* __restrict__ ctr_p, const Consts<R>* __restrict__ cp,
                                                     long long npad_p, int n_p, int tpb_p, SimView<R> v, StepIO<R> io) {
  v.state = state_p; v.ctr = ctr_p; v.npad = npad_p; v.N = n_p; v.tpb = tpb_p;
  io.actions = actions_p;
  constexpr int A = act_width(ACT);
  extern __shared__ float4 tile4[];          // A == 4: [3+L][kPad] float4
  float* tilef = reinterpret_cast<float*>(tile4);  // A == 1, 3: [12+L*A][kPad] float
  __shared__ R sx[MULTI ? 2 * kWave : 1], sy[MULTI ? 2 * kWave : 1], sz[MULTI ? 2 * kWave : 1];
  // per-drone reward / distance in the compute precision: MultiHoverAviary sums both in fp64
  // (MultiHoverAviary.py:75-106) and tests the summed distance against 1e-4
  __shared__ R srew[MULTI ? 2 * kWave : 1], sdist[MULTI ? 2 * kWave : 1];
  __shared__ int sflag[MULTI ? 2 * kWave : 1];
  __shared__ R spair[MULTI ? kPairMax : 1];
  GPD_RSTAMP(11);
  GPD_STAMP(0);
#ifdef GPD_CONTACT_STATS
  const unsigned long long tk0 = __builtin_readcyclecounter();
#endif
  const Consts<R>& c = *cp;
  const int tid = threadIdx.x;
  const int D = MULTI ? v.D : 1;
  const int d = MULTI ? tid % D : 0;
  const int base = tid - d;
  const long long n0 = (long long)blockIdx.x * v.tpb;
  const long long n = n0 + tid;
  const int nact = (int)((v.N - n0) < v.tpb ? (v.N - n0) : v.tpb);  // drones owned by this block
  const bool active = tid < nact;
  // inactive lanes compute on the block's first drone and store nothing: a copy of a drone the
  // block integrates anyway, so a wave-uniform solve (the PYB contact) never waits for a drone
  // of another block (with drone 0's copies, every block paid drone 0's contact iterations)
  const long long nn = active ? n : n0;
  const long long e = MULTI ? nn / D : nn;
  const bool drag = pf_on<PF>(c.flags, F_DRAG);
  // drone <-> drone contact: the block's pair layout (the pair table loads go out with the state's)
  const DcPairs dcp = dc_enabled<MULTI, PF>(c.flags) ? dc_pairs_for(v, tid, nact) : dc_pairs_none();

  Drone<R> s;
  R last[4];
  load_drone<R, STREAM>(v, nn, s, last, drag);
  const int2 cv = v.ctr[e];
  const int sc = cv.x;        // step_counter
  const int head = cv.y;      // ring slot receiving this step's action
  float a[A];
  if (A == 4) {
    const float4 a4 = *reinterpret_cast<const float4*>(io.actions + nn * 4);
    a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
  } else {
#pragma unroll
    for (int j = 0; j < A; ++j) a[j] = io.actions[nn * A + j];
  }

  // the constants of the whole step, loaded in one batch while the state loads are in flight
  DynK<R> dk = dyn_consts(c);
  // warm the scalar cache with the kernel-argument lines the rest of the step reads (ring /
  // counters, task fields + obs pointers, done-flag pointers): one batch of misses now, in the
  // shadow of the state loads, instead of serialised misses behind later branches
  asm volatile("" ::"s"(v.ring), "s"(v.task), "s"(io.trunc));
#ifdef GPD_STAMPS
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // diagnostic: loads landed
  GPD_STAMP(10);
#endif
  R rpm[4];
  R cs[9];  // controller state (PID types)
  if (!act_is_pid(ACT)) {
    // _preprocessAction: rpm = HOVER_RPM*(1+0.05*a)  (BaseRLAviary.py:191-192, :224-225)
#pragma unroll
    for (int k = 0; k < 4; ++k) rpm[k] = (R)action_to_rpm(dk.hover_f32, a[A == 4 ? k : 0]);
  } else {
    // PID / VEL / ONE_D_PID (BaseRLAviary.py:193-235): DSLPIDControl on the state vector of
    // the last readback (_getDroneStateVector :559-561)
#pragma unroll
    for (int k = 0; k < 9; ++k) cs[k] = v.ctrl[tidx(nn, k, 9)];
    R qn[4], Rm[9], rpy[3];
    readback_fused(s.qx, s.qy, s.qz, s.qw, qn, Rm);
    quat_to_euler(qn, rpy[0], rpy[1], rpy[2]);
    const R pos[3] = {s.px, s.py, s.pz}, vel[3] = {s.vx, s.vy, s.vz};
    R tpos[3], tvel[3], tyaw;
    pid_targets<R, ACT>(c.pid, a, pos, rpy, tpos, tyaw, tvel);
    dsl_pid<R, ACT != ACT_VEL>(c.pid, pos, Rm, rpy, vel, tpos, tyaw, tvel, cs, rpm);
  }

  const int nh = v.ring_len - 1;
  // history ring -> obs tile: the L-1 oldest actions (LDS-DMA).  Issued after the first
  // substep: hipcc waits vmcnt(0) at the next use of an ordinary load while an LDS-DMA is in
  // flight, so issuing it before the state/action loads were consumed would put the DMA round
  // trip on the critical path.  Issued there it overlaps the remaining substeps.
  auto history_dma = [&]() {
    for (int k = 0; k < nh; ++k) {
      int slot = head + 1 + k;
      slot -= slot >= v.ring_len ? v.ring_len : 0;
      const float* src = v.ring + ridx(nn, slot, v.ring_len, A);
      if (A == 4) {
        __builtin_amdgcn_global_load_lds((gbl_void_ptr)src, (lds_void_ptr)(tile4 + (3 + k) * kPad), 16, 0,
                                         STREAM ? kAuxDmaStream : 0);
      } else {
#pragma unroll
        for (int j = 0; j < A; ++j)
          __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + j), (lds_void_ptr)(tilef + (12 + k * A + j) * kPad), 4,
                                           0, STREAM ? kAuxDmaStream : 0);
      }
    }
  };
  // propeller wrench: the same RPMs drive every substep of the control step (:349-367)
  R W[4];
  rpm_wrench<R, PF>(rpm, dk, c, W);
  // substeps 1..nsub-1 skip the (write-only) world ang_v; the last one produces it
  // (the first substep is peeled so the loop body stays one basic block)
#ifdef GPD_DMA_EARLY
  history_dma();   // diagnostic build: the DMA behind the state loads instead of the first substep
#endif
#ifndef GPD_DC_DMA_LATE
#define GPD_DC_DMA_LATE 1   // A/B builds: 1 = multi-drone Bullet kernels issue the history DMA after the
                            // substeps (a drone-contact call waits for every memory operation in flight)
#endif
#ifndef GPD_PEEL_BULLET
#define GPD_PEEL_BULLET 0   // A/B builds: 1 = the Bullet flag sets peel the first / last substep too
#endif
  if (!GPD_PEEL_BULLET && PF != kPfRuntime && (PF & F_BULLET) != 0) {
    // Bullet flag sets: ONE copy of the substep (its plane and pair solves are most of the kernel's
    // code; peeled first / last copies would triple it past the instruction cache the SQC shares
    // between two CUs).  The world ang_v is a three-register copy here, so every substep makes it.
    for (int it = 0; it < dk.nsub; ++it) {
      substep_block<R, MULTI, PF, true>(s, rpm, W, last, c, dk, sx, sy, sz, tid, base, D, v.dw_pairs, spair, dcp);
#pragma unroll
      for (int k = 0; k < 4; ++k) last[k] = rpm[k];   // self.last_clipped_action = clipped_action  :372
#ifndef GPD_DMA_EARLY
      if (it == 0 && !(MULTI && GPD_DC_DMA_LATE)) history_dma();
#endif
    }
#ifndef GPD_DMA_EARLY
    if (MULTI && GPD_DC_DMA_LATE) history_dma();
#endif
  } else {
    if (dk.nsub > 1) {
      substep_block<R, MULTI, PF, false>(s, rpm, W, last, c, dk, sx, sy, sz, tid, base, D, v.dw_pairs, spair, dcp);
#pragma unroll
      for (int k = 0; k < 4; ++k) last[k] = rpm[k];   // self.last_clipped_action = clipped_action  :372
      GPD_STAMP(1);
#ifndef GPD_DMA_EARLY
      history_dma();
#endif
      for (int it = 1; it < dk.nsub - 1; ++it)
        substep_block<R, MULTI, PF, false>(s, rpm, W, last, c, dk, sx, sy, sz, tid, base, D, v.dw_pairs, spair, dcp);
    }
    substep_block<R, MULTI, PF, true>(s, rpm, W, last, c, dk, sx, sy, sz, tid, base, D, v.dw_pairs, spair, dcp);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];
#ifndef GPD_DMA_EARLY
    if (dk.nsub == 1) history_dma();
#endif
  }
  GPD_STAMP(2);
  // final readback (:374) -> obs / reward / done
  R qn[4], Rm[9];
  readback_fused(s.qx, s.qy, s.qz, s.qw, qn, Rm);
  AttitudeArgs<R> att = attitude_args(qn);
  bool tilted, up_unused;   // |roll| or |pitch| > 0.4, decided exactly near the limit (attitude_decide)
  attitude_decide<R, true, false>(s.qx, s.qy, s.qz, s.qw, att, tilted, up_unused);
  float roll, pitch, yaw;
  obs_euler_f32(qn, att, roll, pitch, yaw);

  // ---- task hooks, evaluated before step_counter += PYB_STEPS_PER_CTRL (:376-382)
  float reward = -1.0f;
  bool term = false, trunc = false;
  if (v.task != TASK_NONE) {
    const R* tg = MULTI ? v.target + d * 3 : c.target0;
    const R tx = tg[0] - s.px, ty = tg[1] - s.py, tz = tg[2] - s.pz;
    // |e|^2 gives the reward max(0, 2 - |e|^4); the done test is made on |e| itself, as the
    // reference's np.linalg.norm(...) < .0001 (HoverAviary.py:92, MultiHoverAviary.py:101-104)
    const R d2 = tx * tx + ty * ty + tz * tz;
    const R dist = g_sqrt(d2);
    R r = R(2) - d2 * d2;
    r = r > R(0) ? r : R(0);
    const bool oob = g_abs(s.px) > v.bound_xy || g_abs(s.py) > v.bound_xy || s.pz > R(2) || tilted;
    if (MULTI) {
      srew[tid] = r;
      sdist[tid] = dist;
      sflag[tid] = oob ? 1 : 0;
      wave_lds_sync();   // one-wave block; no __syncthreads(): its fence would wait for the history DMA
      if (d == 0) {
        // MultiHoverAviary: summed reward, sum of distances < 1e-4, any drone out of bounds
        R rs = R(0), ds = R(0);
        int anyo = 0;
        for (int j = 0; j < D; ++j) { rs += srew[base + j]; ds += sdist[base + j]; anyo |= sflag[base + j]; }
        reward = (float)rs;
        term = ds < R(1e-4);
        trunc = anyo != 0 || sc >= v.trunc_sc;
        sflag[tid] = (term ? 1 : 0) | (trunc ? 2 : 0);
        srew[tid] = reward;
      }
      wave_lds_sync();
      const int fl = sflag[base];
      term = fl & 1;
      trunc = (fl >> 1) & 1;
      reward = (float)srew[base];
    } else {
      reward = (float)r;
      term = dist < R(1e-4);
      trunc = oob || sc >= v.trunc_sc;
    }
  }
  const bool done = term || trunc;
  const bool do_reset = done && v.autoreset;

  float row12[12] = {(float)s.px, (float)s.py, (float)s.pz, roll, pitch, yaw,
                     (float)s.vx, (float)s.vy, (float)s.vz, (float)s.ax, (float)s.ay, (float)s.az};
  GPD_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // history DMA has landed in the tile
  GPD_STAMP(4);
  // current action into the ring (deque.append); issued after the wait above so that the wait
  // does not also cover this store's write acknowledgement.  The DMA never reads slot `head`.
  if (active) {
    float* ring_cur = v.ring + ridx(n, head, v.ring_len, A);
    if (A == 4) *reinterpret_cast<float4*>(ring_cur) = make_float4(a[0], a[1], a[2], a[3]);
    else
#pragma unroll
      for (int j = 0; j < A; ++j) ring_cur[j] = a[j];
  }


  const int NC = A == 4 ? 3 + v.ring_len : 12 + v.ring_len * A;  // tile columns (float4 / float)
  if (do_reset) {
    // the terminal row's state part is stored straight from registers (finished envs are rare;
    // its history and action columns equal the reset row's and go out with the tile copy-out);
    // the env goes back to INIT_XYZS / INIT_RPYS (_housekeeping :458-477; SB3 DummyVecEnv keeps
    // the last obs as terminal_observation)
    if (active && io.terminal_obs != nullptr) {
      float* trow = io.terminal_obs + n * v.W;
      if (A == 4) {   // W = 72: 16-byte aligned rows
        float4* t4 = reinterpret_cast<float4*>(trow);
        t4[0] = make_float4(row12[0], row12[1], row12[2], row12[3]);
        t4[1] = make_float4(row12[4], row12[5], row12[6], row12[7]);
        t4[2] = make_float4(row12[8], row12[9], row12[10], row12[11]);
      } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) trow[k] = row12[k];
      }
    }
    const R* ini = MULTI ? v.init + d * 10 : c.init0;
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
  // bit r set <=> tile row r belongs to an env that finished this step (tile rows are lanes)
  const unsigned long long done_rows = __ballot(do_reset && active && io.terminal_obs != nullptr);

  GPD_STAMP(5);
  // ---- state columns + current action into the tile, then coalesced copy-out of the rows
  if (A == 4) {
    tile4[0 * kPad + tid] = make_float4(row12[0], row12[1], row12[2], row12[3]);
    tile4[1 * kPad + tid] = make_float4(row12[4], row12[5], row12[6], row12[7]);
    tile4[2 * kPad + tid] = make_float4(row12[8], row12[9], row12[10], row12[11]);
    tile4[(3 + nh) * kPad + tid] = make_float4(a[0], a[1], a[2], a[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 12; ++k) tilef[k * kPad + tid] = row12[k];
#pragma unroll
    for (int j = 0; j < A; ++j) tilef[(12 + nh * A + j) * kPad + tid] = a[j];
  }
  __syncthreads();
  GPD_STAMP(6);
  tile_copy_out<A, kWave, 6, STREAM ? kAuxWtStream : kAuxWt>(tile4, tilef, tid, nact, NC, v.nc_magic, v.wt, done_rows,
                                                             io.obs, io.terminal_obs, n0);
  GPD_STAMP(7);
  GPD_RSTAMP(12);
#ifdef GPD_CONTACT_STATS
  if (tid == 0 && blockIdx.x < 4096) atomicAdd(&g_pc_hist[256 + 4096 + blockIdx.x], __builtin_readcyclecounter() - tk0);
#endif
  if (!active) return;
  store_drone_step<R, STREAM ? kAuxWtStream : kAuxWt>(v, n, s, last);
  mark_last_in_ring(v, n);
  if (act_is_pid(ACT)) {
#pragma unroll
    for (int k = 0; k < 9; ++k) v.ctrl[tidx(n, k, 9)] = cs[k];
  }
  if (d == 0) {
    io.reward[e] = reward;
    io.term[e] = term ? 1 : 0;
    io.trunc[e] = trunc ? 1 : 0;
    v.ctr[e] = make_int2(do_reset ? 0 : sc + dk.nsub, head + 1 == v.ring_len ? 0 : head + 1);
  }
}


// ---------------------------------------------------------------------------------------
// step_kernel_duo: step_kernel<R, ACT, false, true> (single-drone envs, plain DYN, RPM action
// types: the bench path) with every drone's work split over TWO waves of one workgroup.
// With few envs per CU (4096 envs: one 16-drone wave per CU) a launch lasts as long as one
// wave's serial instruction stream, and a substep is ~115 issue-bound f64 instructions.
// Without aero terms it falls into two chains (rate_half / pose_half, gpd_device.h):
//   wave 1 (rates): ω' and the _integrateQ weights, handed over through LDS;
//   wave 0 (pose):  readback, v, p, and the quaternion update with those weights.
// One barrier per substep; the hand-off is double-buffered by substep parity, so wave 1
// computes substep k+1 while wave 0 finishes substep k.  Wave 1 also issues the history DMA
// behind its last substep (it lands while wave 0 finishes) and writes the current action (ring
// + tile); both waves stream the tile copy-out.  (Moving the final Euler angles to wave 1 as
// well measured slower: 5.56 -> 5.89 us at 4096 envs.)  Same operations as step_kernel<R, ACT, false, true>; results agree to
// rounding (tests/test_gpu_parity.py::test_duo_kernel_matches_single_wave).
// IO = true adds a third wave ("io wave") that writes the action-history columns of the
// observation rows (83 % of a row's bytes, independent of the physics: ring slots head+1.. and
// the current action) WHILE the pose / rate waves integrate, and appends the action to the
// ring.  The pose wave then stores only the 12 state columns of its rows straight from
// registers, so the LDS observation tile and its copy-out leave the critical path.
template <typename R, int ACT, bool IO>
__global__ __launch_bounds__(IO ? 3 * kWave : 2 * kWave) void step_kernel_duo(R* __restrict__ state_p,
                                                             const float* __restrict__ actions_p,
                                                             int2* __restrict__ ctr_p, const Consts<R>* __restrict__ cp,
                                                             long long npad_p, int n_p, int tpb_p, SimView<R> v,
                                                             StepIO<R> io) {
  static_assert(!act_is_pid(ACT), "the duo kernel serves the RPM action types");
  v.state = state_p; v.ctr = ctr_p; v.npad = npad_p; v.N = n_p; v.tpb = tpb_p;
  io.actions = actions_p;
  constexpr int A = act_width(ACT);
  extern __shared__ float4 tile4[];
  float* tilef = reinterpret_cast<float*>(tile4);
  __shared__ R shand[2][5][kWave];        // rate_half -> pose_half, by substep parity
  __shared__ R sw[3][kWave];              // rpy_rates after the last substep
  __shared__ unsigned long long sdone;    // done-row mask of the block (tile rows)
  GPD_RSTAMP(11);
  GPD_STAMP(0);
  const Consts<R>& c = *cp;
  const int tid = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x) / kWave;   // wave-uniform
  const bool rate_wave = wave == 1;
  const long long n0 = (long long)blockIdx.x * v.tpb;
  const long long n = n0 + tid;
  const int nact = (int)((v.N - n0) < v.tpb ? (v.N - n0) : v.tpb);
  const bool active = tid < nact;
  const long long nn = active ? n : n0;  // inactive lanes compute on the block's first drone, store nothing
#ifdef GPD_STAMPS
  {   // diagnostic: which SIMD / CU each wave of the block runs on (HW_ID: SIMD_ID bits 5:4)
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    if (tid == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + 14 + wave] = hw;
  }
#endif

  if (IO && wave == 2) {
    // ------------------------------------------------------------ wave 2: history columns
    // The history columns of a row are ring slots head+1 .. head+L-1 (oldest first,
    // BaseRLAviary.py:307-319) and the current action.  The wave appends the action to the
    // ring and the tile, follows the pose/rate waves' hand-off barriers, then DMAs the ring
    // slots into the tile and streams the tile, transposed (conflict-free thanks to the column
    // pad), into the rows' history columns with coalesced stores - beside the pose wave's last
    // substep and epilogue, which then stores only the 12 state columns.  The tile stays for
    // the terminal rows of envs that finish, known after the final barrier.
    const int L = v.ring_len;
    const int nsub = c.nsub;
    const int2 cv = v.ctr[nn];
    const int hd = cv.y;                          // ring slot receiving this step's action
    float a[A];
    if (A == 4) {
      const float4 a4 = *reinterpret_cast<const float4*>(io.actions + nn * 4);
      a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
    } else {
      a[0] = io.actions[nn];
    }
    // The current action goes into its tile column BEFORE the DMA is issued: a ds_write after
    // an LDS-DMA in flight makes the compiler wait for the whole DMA (vmcnt(0)) first.
    if (A == 4) tile4[(L - 1) * kPad + tid] = make_float4(a[0], a[1], a[2], a[3]);
    else tilef[(L - 1) * kPad + tid] = a[0];
    if (active) {      // deque.append of the current action; the DMA never reads slot `head`
      float* ring_cur = v.ring + ridx(n, hd, L, A);
      if (A == 4) *reinterpret_cast<float4*>(ring_cur) = make_float4(a[0], a[1], a[2], a[3]);
      else ring_cur[0] = a[0];
    }
    // This wave publishes nothing to the others, so its barriers skip lds_barrier's
    // lgkmcnt(0) wait: an LDS-DMA in flight holds that counter until it lands.
    GPD_IOSTAMP(0);
    // (an LDS-counter hand-off between the pose and rate waves, which would free this wave of
    // their barriers, measured 5.3 / 6.4 us against 4.9: profiles/r6/duo_flags/)
    asm volatile("s_barrier" ::: "memory");       // hand-off 0
    GPD_IOSTAMP(1);
    for (int k = 1; k < nsub; ++k) asm volatile("s_barrier" ::: "memory");   // hand-offs 1 .. nsub-1
    // history ring -> tile (LDS-DMA) behind the last hand-off: an LDS-DMA in flight while the
    // pose / rate waves still exchange hand-offs slowed their substeps by ~850 cycles per launch
    // (phase stamps, 4096 envs), issued here it lands beside the pose wave's last substep and
    // epilogue.  Slot head+1+m of every drone of the block -> tile column m (one coalesced
    // 64-drone run per slot, lane-contiguous in LDS).
    {
      const float* rb = v.ring + ridx(nn, 0, L, A);
      int slot = hd + 1 == L ? 0 : hd + 1;
      for (int m = 0; m < L - 1; ++m) {
        const float* src = rb + slot * (64 * A);
        if (A == 4) __builtin_amdgcn_global_load_lds((gbl_void_ptr)src, (lds_void_ptr)(tile4 + m * kPad), 16, 0, 0);
        else __builtin_amdgcn_global_load_lds((gbl_void_ptr)src, (lds_void_ptr)(tilef + m * kPad), 4, 0, 0);
        slot = slot + 1 == L ? 0 : slot + 1;
      }
    }
    GPD_IOSTAMP(2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA has landed in its tile
    GPD_IOSTAMP(3);
    const int total = nact * L;
    const int NC = A == 4 ? 3 + L : v.W;          // row stride in elements
    const int c0 = A == 4 ? 3 : 12;               // first history column
    const float rL = 1.0f / (float)L;             // (g + 0.5) / L: exact row index for g < 2^12
    float* const dst0 = io.obs + n0 * v.W;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(dst0, 0, nact * v.W * 4, 0x00020000);
    // four elements per lane in flight per pass (LDS reads, then stores); an element past the
    // end gets an offset past num_records, so the buffer unit drops its store
    constexpr int U = 4;
    for (int g0 = tid; g0 < total; g0 += U * kWave) {
      int off[U];
      float4 v4[U];
      float v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int g = g0 + u * kWave;
        const bool ok = g < total;
        const int gg = ok ? g : total - 1;
        const int i = (int)(((float)gg + 0.5f) * rL), k = gg - i * L;
        const int e = i * NC + c0 + k;
        off[u] = ok ? e * (A == 4 ? 16 : 4) : nact * v.W * 4;
        if (A == 4) v4[u] = tile4[__umul24(k, kPad) + i];
        else v1[u] = tilef[__umul24(k, kPad) + i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (v.wt & 1) {
          if (A == 4) store_wt(rsrc, off[u], v4[u]);
          else store_wt(rsrc, off[u], v1[u]);
        } else {
          if (A == 4) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gpd_v4i, v4[u]), rsrc, off[u], 0, 0);
          else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v1[u]), rsrc, off[u], 0, 0);
        }
      }
    }
    GPD_IOSTAMP(4);
    lds_barrier();     // final: sdone published by the pose wave
    GPD_IOSTAMP(5);
    const unsigned long long dr = sdone;
    if (dr) {
      float* const tdst = io.terminal_obs + n0 * v.W;
      for (int g = tid; g < total; g += kWave) {
        const int i = (int)(((float)g + 0.5f) * rL), k = g - i * L;
        if ((dr >> i) & 1ull) {
          const int e = i * NC + c0 + k;
          if (A == 4) reinterpret_cast<float4*>(tdst)[e] = tile4[__umul24(k, kPad) + i];
          else tdst[e] = tilef[__umul24(k, kPad) + i];
        }
      }
    }
#ifdef GPD_STAMPS
    {   // diagnostic: the io wave's end (realtime) into phase 13
      __builtin_amdgcn_sched_barrier(0);
      unsigned long long t_;
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
      if (tid == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + 13] = t_;
    }
#endif
    return;
  }

  float a[A];
  if (A == 4) {
    const float4 a4 = *reinterpret_cast<const float4*>(io.actions + nn * 4);
    a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
  } else {
#pragma unroll
    for (int j = 0; j < A; ++j) a[j] = io.actions[nn * A + j];
  }
  const R* st = v.state + tidx(nn, 0, kStateComps);
  // each wave issues its state loads first and only then pins the step's constants into VGPRs
  // (dyn_consts waits for the scalar loads): one exposed memory round trip, not two

  if (rate_wave) {
    // ------------------------------------------------------------ wave 1: body rates
    R wx = st[10 * 64], wy = st[11 * 64], wz = st[12 * 64];
    const int head = v.ctr[nn].y;
    DynK<R> dk = dyn_consts(c);   // the ring fields are first needed after the substeps
    const int nsub = dk.nsub, nh = v.ring_len - 1;
    const int NC = A == 4 ? 3 + v.ring_len : 12 + v.ring_len * A;
    R rpm[4], W[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rpm[k] = (R)action_to_rpm(dk.hover_f32, a[A == 4 ? k : 0]);
    rpm_wrench<R, 0>(rpm, dk, c, W);
    for (int k = 0; k < nsub; ++k) {
      R h[5];
      rate_half(wx, wy, wz, W, dk, h);
#pragma unroll
      for (int j = 0; j < 5; ++j) shand[k & 1][j][tid] = h[j];
      if (k == nsub - 1) { sw[0][tid] = wx; sw[1][tid] = wy; sw[2][tid] = wz; }
      lds_barrier();   // hand-off k published
    }
    if (IO) {          // the io wave owns the history columns and the ring append
      lds_barrier();   // final
      return;
    }
    // history ring -> obs tile (LDS-DMA): issued once the last hand-off is out, it lands while
    // the pose wave finishes its last substep, the final readback and the task hooks.  The
    // env's ring slots are 64*A floats apart in its 64-drone tile.
    {
      const float* rb = v.ring + ridx(nn, 0, v.ring_len, A);
      int slot = head + 1 == v.ring_len ? 0 : head + 1;
      for (int m = 0; m < nh; ++m) {
        const float* src = rb + slot * (64 * A);
        if (A == 4) {
          __builtin_amdgcn_global_load_lds((gbl_void_ptr)src, (lds_void_ptr)(tile4 + (3 + m) * kPad), 16, 0, 0);
        } else {
#pragma unroll
          for (int j = 0; j < A; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + j), (lds_void_ptr)(tilef + (12 + m * A + j) * kPad), 4,
                                             0, 0);
        }
        slot = slot + 1 == v.ring_len ? 0 : slot + 1;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // history DMA has landed in the tile
    if (active) {      // current action into the ring (deque.append); the DMA never reads `head`
      float* ring_cur = v.ring + ridx(n, head, v.ring_len, A);
      if (A == 4) *reinterpret_cast<float4*>(ring_cur) = make_float4(a[0], a[1], a[2], a[3]);
      else
#pragma unroll
        for (int j = 0; j < A; ++j) ring_cur[j] = a[j];
    }
    if (A == 4) {
      tile4[(3 + nh) * kPad + tid] = make_float4(a[0], a[1], a[2], a[3]);
    } else {
#pragma unroll
      for (int j = 0; j < A; ++j) tilef[(12 + nh * A + j) * kPad + tid] = a[j];
    }
    lds_barrier();     // tile complete, sdone published
    tile_copy_out<A, 2 * kWave, 3>(tile4, tilef, threadIdx.x, nact, NC, v.nc_magic, v.wt, sdone, io.obs,
                                io.terminal_obs, n0);
#ifdef GPD_STAMPS
    {   // diagnostic: the rate wave's end (realtime) into phase 13
      __builtin_amdgcn_sched_barrier(0);
      unsigned long long t_;
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
      if (tid == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * kStampPhases + 13] = t_;
    }
#endif
    return;
  }

  // -------------------------------------------------------------- wave 0: pose
  Drone<R> s;
  R last[4];
  load_drone(v, nn, s, last, false);
  const int2 cv = v.ctr[nn];
  const int sc = cv.x;          // step_counter
  const int head = cv.y;        // ring slot receiving this step's action
  DynK<R> dk = dyn_consts(c, v.task, io.trunc);
  const int nsub = dk.nsub;
  const int NC = A == 4 ? 3 + v.ring_len : 12 + v.ring_len * A;
#ifdef GPD_STAMPS
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // diagnostic: loads landed
  GPD_STAMP(10);
#endif
  R fz;
  {
    R rpm[4], W[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rpm[k] = (R)action_to_rpm(dk.hover_f32, a[A == 4 ? k : 0]);
    rpm_wrench<R, 0>(rpm, dk, c, W);
    fz = W[0];
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];   // self.last_clipped_action = clipped_action  :372
  }
  const R wnone[3] = {R(0), R(0), R(0)};
  auto hand_off = [&](int k, R h[5]) {
#pragma unroll
    for (int j = 0; j < 5; ++j) h[j] = shand[k & 1][j][tid];
  };
  if (nsub > 1) {
    lds_barrier();   // hand-off 0
    R h[5];
    hand_off(0, h);
    pose_half<R, false, true>(s, fz, h, wnone, dk);
    GPD_STAMP(1);
    for (int k = 1; k < nsub - 1; ++k) {
      lds_barrier();   // hand-off k
      hand_off(k, h);
      pose_half<R, false, false>(s, fz, h, wnone, dk);
    }
  }
  {
    lds_barrier();   // last hand-off + final rates
    R h[5];
    hand_off(nsub - 1, h);
    s.wx = sw[0][tid]; s.wy = sw[1][tid]; s.wz = sw[2][tid];
    const R w[3] = {s.wx, s.wy, s.wz};
    if (nsub > 1) pose_half<R, true, false>(s, fz, h, w, dk);
    else pose_half<R, true, true>(s, fz, h, w, dk);
  }
  GPD_STAMP(2);
  // final readback (:374) -> obs / reward / done
  R qn[4], Rm[9];
  readback_fused(s.qx, s.qy, s.qz, s.qw, qn, Rm);
  AttitudeArgs<R> att = attitude_args(qn);
  bool tilted, up_unused;   // |roll| or |pitch| > 0.4, decided exactly near the limit (attitude_decide)
  attitude_decide<R, true, false>(s.qx, s.qy, s.qz, s.qw, att, tilted, up_unused);
  float roll, pitch, yaw;
  obs_euler_f32(qn, att, roll, pitch, yaw);
  float reward = -1.0f;
  bool term = false, trunc = false;
  if (v.task != TASK_NONE) {
    const R* tg = c.target0;
    const R tx = tg[0] - s.px, ty = tg[1] - s.py, tz = tg[2] - s.pz;
    const R d2 = tx * tx + ty * ty + tz * tz;
    R r = R(2) - d2 * d2;
    r = r > R(0) ? r : R(0);
    const bool oob = g_abs(s.px) > v.bound_xy || g_abs(s.py) > v.bound_xy || s.pz > R(2) || tilted;
    reward = (float)r;
    term = g_sqrt(d2) < R(1e-4);   // np.linalg.norm(...) < .0001 (HoverAviary.py:92)
    trunc = oob || sc >= v.trunc_sc;
  }
  const bool done = term || trunc;
  const bool do_reset = done && v.autoreset;
  GPD_STAMP(3);
  GPD_STAMP(4);
  float row12[12] = {(float)s.px, (float)s.py, (float)s.pz, roll, pitch, yaw,
                     (float)s.vx, (float)s.vy, (float)s.vz, (float)s.ax, (float)s.ay, (float)s.az};
  if (do_reset) {
    if (active && io.terminal_obs != nullptr) {
      float* trow = io.terminal_obs + n * v.W;
      if (A == 4) {
        float4* t4 = reinterpret_cast<float4*>(trow);
        t4[0] = make_float4(row12[0], row12[1], row12[2], row12[3]);
        t4[1] = make_float4(row12[4], row12[5], row12[6], row12[7]);
        t4[2] = make_float4(row12[8], row12[9], row12[10], row12[11]);
      } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) trow[k] = row12[k];
      }
    }
    const R* ini = c.init0;
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
  const unsigned long long done_rows = __ballot(do_reset && active && io.terminal_obs != nullptr);
  if (IO) {
    // the row's 12 state columns straight from registers; the io wave writes the rest
    GPD_STAMP(5);
    if (active) {
      if (A == 4) {
        const float4 r0 = make_float4(row12[0], row12[1], row12[2], row12[3]);
        const float4 r1 = make_float4(row12[4], row12[5], row12[6], row12[7]);
        const float4 r2 = make_float4(row12[8], row12[9], row12[10], row12[11]);
        if (v.wt & 1) {
          const __amdgpu_buffer_rsrc_t r =
              __builtin_amdgcn_make_buffer_rsrc(io.obs + n0 * v.W, 0, nact * v.W * 4, 0x00020000);
          const int o = tid * v.W * 4;
          store_wt(r, o, r0); store_wt(r, o + 16, r1); store_wt(r, o + 32, r2);
        } else {
          float4* o4 = reinterpret_cast<float4*>(io.obs + n * v.W);
          o4[0] = r0; o4[1] = r1; o4[2] = r2;
        }
      } else {
        float* orow = io.obs + n * v.W;
#pragma unroll
        for (int k = 0; k < 12; ++k) orow[k] = row12[k];
      }
    }
    if (tid == 0) sdone = done_rows;
    lds_barrier();   // final: sdone published (the io wave writes the terminal rows' history)
    GPD_STAMP(6);
    GPD_STAMP(8);
    GPD_STAMP(9);
  } else {
    if (A == 4) {
      tile4[0 * kPad + tid] = make_float4(row12[0], row12[1], row12[2], row12[3]);
      tile4[1 * kPad + tid] = make_float4(row12[4], row12[5], row12[6], row12[7]);
      tile4[2 * kPad + tid] = make_float4(row12[8], row12[9], row12[10], row12[11]);
    } else {
#pragma unroll
      for (int k = 0; k < 12; ++k) tilef[k * kPad + tid] = row12[k];
    }
    if (tid == 0) sdone = done_rows;
    GPD_STAMP(5);
    lds_barrier();     // tile complete, sdone published
    GPD_STAMP(6);
    tile_copy_out<A, 2 * kWave, 3>(tile4, tilef, threadIdx.x, nact, NC, v.nc_magic, v.wt, done_rows, io.obs,
                                io.terminal_obs, n0);
  }
  GPD_STAMP(7);
  GPD_RSTAMP(12);
  if (!active) return;
  store_drone_step(v, n, s, last);
  mark_last_in_ring(v, n);
  io.reward[n] = reward;
  io.term[n] = term ? 1 : 0;
  io.trunc[n] = trunc ? 1 : 0;
  v.ctr[n] = make_int2(do_reset ? 0 : sc + nsub, head + 1 == v.ring_len ? 0 : head + 1);
}

// ---------------------------------------------------------------------------------------
// Envs of more than 64 drones (MultiHoverAviary(num_drones=D), D <= kWideMax): one env per
// workgroup of ceil(D/64) waves.  (Also envs of any D whose observation rows overflow the one-wave
// kernels' LDS tile, gpd_create: up to 64 / D of them packed into one wave when D <= 32.)  The per-substep position exchange of _downwash
// (BaseAviary.py:785-811, O(D^2)) and the env's reward / done reductions go through LDS with
// workgroup barriers; lanes d >= D compute on drone 0 of the env and store nothing.  Physics
// flags are tested at run time; observation rows are stored straight from registers (history
// columns read from the ring), without the LDS tile of the one-wave kernels.  Same operations
// and order as step_kernel / integrate_kernel (tests/test_gpu_wide.py).
constexpr int kWideMax = 1024;

// t: the thread (its LDS slot), active: it owns a drone, base: its env's first slot
template <typename R>
__device__ __forceinline__ R wide_downwash(const Drone<R>& s, R* sx, R* sy, R* sz, int t, bool active, int base,
                                           int D, const Consts<R>& c, int flags) {
  R dw = R(0);
  if (flags & F_DW) {
    __syncthreads();                       // previous readers of sx/sy/sz are done
    if (active) { sx[t] = s.px; sy[t] = s.py; sz[t] = s.pz; }
    __syncthreads();
    dw = downwash_sum(s.px, s.py, s.pz, sx, sy, sz, base, D, c);
  }
  return dw;
}

// The history columns of the workgroup's observation rows (and terminal rows): ring slots
// head+1 .. head+L-1 of each drone, copied by every thread of the workgroup (ACT's A floats per
// slot, float4 items for A = 4), kWideU loads in flight per thread before their stores.  n0: the
// workgroup's first drone, nd: its drones; shead[env slot] = ring head | 1 << 30 when the env's
// terminal row is written.
constexpr int kWideU = 8;
constexpr int kWideTrow = 1 << 30;
template <typename R, int A>
__device__ __forceinline__ void wide_history(const SimView<R>& v, const StepIO<R>& io, long long n0, int nd, int D,
                                             const int* shead) {
  const int L = v.ring_len, Wd = v.W, H = L - 1, nth = blockDim.x;
  constexpr int G = A == 4 ? 4 : 1;              // floats per item
  const int per = H * (A / G);                   // items per drone
  const int total = nd * per;
  for (int i0 = 0; i0 < total; i0 += nth * kWideU) {
    float x[kWideU][G];
    long long dst[kWideU];
    bool tr[kWideU];
#pragma unroll
    for (int u = 0; u < kWideU; ++u) {
      const int i = i0 + u * nth + (int)threadIdx.x;
      dst[u] = -1;
      if (i < total) {
        const int dq = i / per, r = i - dq * per;
        const int k = G == 4 ? r : r / A, j = G == 4 ? 0 : r - k * A;
        const int hv = shead[dq / D], head = hv & (kWideTrow - 1);
        tr[u] = (hv & kWideTrow) != 0;
        int slot = head + 1 + k;
        slot -= slot >= L ? L : 0;
        const float* src = v.ring + ridx(n0 + dq, slot, L, A) + j;
        if (G == 4) {
          const float4 q = *reinterpret_cast<const float4*>(src);
          x[u][0] = q.x; x[u][G > 1 ? 1 : 0] = q.y; x[u][G > 2 ? 2 : 0] = q.z; x[u][G > 3 ? 3 : 0] = q.w;
        } else {
          x[u][0] = *src;
        }
        dst[u] = (n0 + dq) * Wd + 12 + k * A + j;
      }
    }
#pragma unroll
    for (int u = 0; u < kWideU; ++u) {
      if (dst[u] < 0) continue;
      if (G == 4) {
        const float4 q = make_float4(x[u][0], x[u][G > 1 ? 1 : 0], x[u][G > 2 ? 2 : 0], x[u][G > 3 ? 3 : 0]);
        *reinterpret_cast<float4*>(io.obs + dst[u]) = q;
        if (tr[u]) *reinterpret_cast<float4*>(io.terminal_obs + dst[u]) = q;
      } else {
        io.obs[dst[u]] = x[u][0];
        if (tr[u]) io.terminal_obs[dst[u]] = x[u][0];
      }
    }
  }
}

// MAXT: the workgroup size bound the instantiation is compiled for (256 / 512 / 1024 threads:
// the register budget per lane halves with each doubling, 1024 spills to scratch).
// DC: the drone <-> drone contact (DcHookT, the one-wave kernels' solve): one-wave workgroups
// (D <= 64, MAXT = 64) of a long-history PYB* env; its DcLds is static LDS, so only these
// instantiations carry it.
template <typename R, int ACT, int MAXT, bool DC = false>
__global__ __launch_bounds__(MAXT) void step_kernel_wide(SimView<R> v, StepIO<R> io, const Consts<R>* __restrict__ cp) {
  constexpr int A = act_width(ACT);
  __shared__ R sx[MAXT], sy[MAXT], sz[MAXT];
  __shared__ int sflag[MAXT];
  __shared__ int shead[kWave];
  const Consts<R>& c = *cp;
  const int D = v.D;
  // GE = v.tpb / D envs per workgroup: one for D > 32; up to 64 / D packed into one wave for the
  // small envs that run here because their observation rows overflow the one-wave kernels' LDS tile
  const int GE = v.tpb / D;
  const int t = threadIdx.x;
  const int g = t / D, d = t - g * D;           // env slot, drone in the env
  const long long e0 = (long long)blockIdx.x * GE, e = e0 + g;
  const long long nenv = v.N / D;
  const bool active = g < GE && e < nenv;
  const int slot0 = (g < GE ? g : 0) * D;       // the env's first LDS slot
  // lanes without a drone compute on the first drone of their own wave (a drone this wave
  // integrates anyway: the waves take turns in the contact solve) and store nothing
  const long long n = active ? e * D + d : e0 * D + (t & ~(kWave - 1));
  const long long es = active ? e : e0;
  const int nact = (int)(nenv - e0 < GE ? nenv - e0 : GE) * D;   // drones owned by this workgroup
  const DcPairs dcp = DC ? dc_pairs_for(v, t, nact) : dc_pairs_none();
  const bool drag = (c.flags & F_DRAG) != 0;
  Drone<R> s;
  R last[4];
  load_drone(v, n, s, last, drag);
  const int2 cv = v.ctr[es];
  const int sc = cv.x, head = cv.y;
  float a[A];
#pragma unroll
  for (int j = 0; j < A; ++j) a[j] = io.actions[n * A + j];
  DynK<R> dk = dyn_consts(c);
  R rpm[4];
  R cs[9];
  if (!act_is_pid(ACT)) {
#pragma unroll
    for (int k = 0; k < 4; ++k) rpm[k] = (R)action_to_rpm(dk.hover_f32, a[A == 4 ? k : 0]);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) cs[k] = v.ctrl[tidx(n, k, 9)];
    R qn[4], Rm[9], rpy[3];
    readback_fused(s.qx, s.qy, s.qz, s.qw, qn, Rm);
    quat_to_euler(qn, rpy[0], rpy[1], rpy[2]);
    const R pos[3] = {s.px, s.py, s.pz}, vel[3] = {s.vx, s.vy, s.vz};
    R tpos[3], tvel[3], tyaw;
    pid_targets<R, ACT>(c.pid, a, pos, rpy, tpos, tyaw, tvel);
    dsl_pid<R, ACT != ACT_VEL>(c.pid, pos, Rm, rpy, vel, tpos, tyaw, tvel, cs, rpm);
  }
  R W[4];
  rpm_wrench<R, kPfRuntime>(rpm, dk, c, W);
  const int nw = (int)(blockDim.x / kWave);
  for (int it = 0; it < dk.nsub; ++it) {
    const R dw = wide_downwash(s, sx, sy, sz, t, active, slot0, D, c, dk.flags);
    if (DC) dyn_substep<R, kPfRuntime, true, 1, DcHookT<false>>(s, rpm, W, last, dw, c, dk, DcHookT<false>{t, dcp});
    else if (nw > 1) dyn_substep<R, kPfRuntime, true, 16>(s, rpm, W, last, dw, c, dk);
    else dyn_substep<R, kPfRuntime, true, 1>(s, rpm, W, last, dw, c, dk);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];   // self.last_clipped_action = clipped_action  :372
  }
  // final readback (:374) -> obs / reward / done
  R qn[4], Rm[9];
  readback_fused(s.qx, s.qy, s.qz, s.qw, qn, Rm);
  AttitudeArgs<R> att = attitude_args(qn);
  bool tilted, up_unused;   // |roll| or |pitch| > 0.4, decided exactly near the limit (attitude_decide)
  attitude_decide<R, true, false>(s.qx, s.qy, s.qz, s.qw, att, tilted, up_unused);
  float roll, pitch, yaw;
  obs_euler_f32(qn, att, roll, pitch, yaw);
  float reward = -1.0f;
  bool term = false, trunc = false;
  if (v.task != TASK_NONE) {
    const R* tg = v.target + (active ? d : 0) * 3;
    const R tx = tg[0] - s.px, ty = tg[1] - s.py, tz = tg[2] - s.pz;
    const R d2 = tx * tx + ty * ty + tz * tz;
    const R dist = g_sqrt(d2);
    R r = R(2) - d2 * d2;
    r = r > R(0) ? r : R(0);
    const bool oob = g_abs(s.px) > v.bound_xy || g_abs(s.py) > v.bound_xy || s.pz > R(2) || tilted;
    __syncthreads();
    if (active) { sx[t] = r; sy[t] = dist; sflag[t] = oob ? 1 : 0; }
    __syncthreads();
    if (active && d == 0) {   // MultiHoverAviary: the summed reward / distance in the reference's order
      R rs = R(0), ds = R(0);
      int anyo = 0;
      for (int j = slot0; j < slot0 + D; ++j) { rs += sx[j]; ds += sy[j]; anyo |= sflag[j]; }
      sflag[slot0] = (ds < R(1e-4) ? 1 : 0) | ((anyo != 0 || sc >= v.trunc_sc) ? 2 : 0);
      sx[slot0] = rs;
    }
    __syncthreads();
    const int fl = sflag[slot0];
    term = fl & 1;
    trunc = (fl >> 1) & 1;
    reward = (float)sx[slot0];
  }
  const bool done = term || trunc;
  const bool do_reset = done && v.autoreset;
  float row12[12] = {(float)s.px, (float)s.py, (float)s.pz, roll, pitch, yaw,
                     (float)s.vx, (float)s.vy, (float)s.vz, (float)s.ax, (float)s.ay, (float)s.az};
  const int L = v.ring_len, Wd = v.W;
  // history columns: ring slots head+1 .. head+L-1 (oldest first), then the current action
  // (BaseRLAviary.py:307-319); the same for the terminal row and the (reset) observation.  The
  // history columns are copied by the whole workgroup, kWideU independent loads per thread
  // before their stores: a lane copying its own row element by element waited out one memory
  // round trip per element (680 us per step for 4096 single-drone envs with a 240-step history)
  if (active && d == 0) shead[g] = head | ((do_reset && io.terminal_obs) ? kWideTrow : 0);
  // (also: every wave has read ctr[e] (kernel entry) before lane d == 0 overwrites it below;
  // without a task, downwash or contact no other workgroup barrier orders the two)
  __syncthreads();
  wide_history<R, A>(v, io, e0 * D, nact, D, shead);
  if (!active) return;
  float* orow = io.obs + n * Wd;
  float* trow = (do_reset && io.terminal_obs) ? io.terminal_obs + n * Wd : nullptr;
  for (int j = 0; j < A; ++j) {
    orow[12 + (L - 1) * A + j] = a[j];
    if (trow) trow[12 + (L - 1) * A + j] = a[j];
  }
  float* ring_cur = v.ring + ridx(n, head, L, A);     // deque.append (slot head is not read above)
  for (int j = 0; j < A; ++j) ring_cur[j] = a[j];
  if (do_reset) {
    if (trow)
      for (int k = 0; k < 12; ++k) trow[k] = row12[k];
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
    for (int k = 6; k < 12; ++k) row12[k] = 0.0f;
  }
  for (int k = 0; k < 12; ++k) orow[k] = row12[k];
  store_drone_step(v, n, s, last);
  mark_last_in_ring(v, n);
  if (act_is_pid(ACT)) {
#pragma unroll
    for (int k = 0; k < 9; ++k) v.ctrl[tidx(n, k, 9)] = cs[k];
  }
  if (d == 0) {
    io.reward[e] = reward;
    io.term[e] = term ? 1 : 0;
    io.trunc[e] = trunc ? 1 : 0;
    v.ctr[e] = make_int2(do_reset ? 0 : sc + dk.nsub, head + 1 == L ? 0 : head + 1);
  }
}

// gpd_integrate for envs of more than 64 drones (see step_kernel_wide).
template <typename R, bool TRAJ, int MAXT>
__global__ __launch_bounds__(MAXT) void integrate_kernel_wide(SimView<R> v, const Consts<R>* __restrict__ cp,
                                                              const R* __restrict__ rpm_in, int n_sub,
                                                              R* __restrict__ traj) {
  __shared__ R sx[MAXT], sy[MAXT], sz[MAXT];
  const Consts<R>& c = *cp;
  const int D = v.D;
  const int d = threadIdx.x;
  const bool active = d < D;
  const long long n = (long long)blockIdx.x * D + (active ? d : (d & ~(kWave - 1)));   // (step_kernel_wide)
  Drone<R> s;
  R last[4];
  load_drone(v, n, s, last, true);
  DynK<R> dk = dyn_consts(c);
  const int nw = (D + kWave - 1) / kWave;
  const long long N = v.N;
  for (int t = 0; t < n_sub; ++t) {
    const R* src = rpm_in + ((long long)t * N + n) * 4;
    R rpm[4] = {src[0], src[1], src[2], src[3]};
    R W[4];
    rpm_wrench<R, kPfRuntime>(rpm, dk, c, W);
    const R dw = wide_downwash(s, sx, sy, sz, d, active, 0, D, c, dk.flags);
    if (nw > 1) dyn_substep<R, kPfRuntime, true, 16>(s, rpm, W, last, dw, c, dk);
    else dyn_substep<R, kPfRuntime, true, 1>(s, rpm, W, last, dw, c, dk);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];
    if (TRAJ && active) {
      R qn[4], roll, pitch, yaw;   // the literal Bullet readback (as state20): exact gimbal branches
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
  if (active && n_sub > 0) store_drone(v, n, s, last);
}

// ---------------------------------------------------------------------------------------
// gpd_integrate: n_sub raw substeps with explicit per-substep RPMs, each followed by a readback.
// PF as in step_kernel: 0 (plain DYN, the raw-integrator bench) or kPfRuntime; TRAJ: record the
// [n_sub][N][20] trajectory.
// STREAM (plain DYN batches past the Infinity Cache): nt loads of the once-read RPM stream and the
// state, nt stores of the state (as step_kernel's STREAM).
template <typename R, bool MULTI, int PF, bool TRAJ, bool STREAM = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(GPD_INTEGRATE_WPE))) void integrate_kernel(SimView<R> v, const Consts<R>* __restrict__ cp,
                                                          const R* __restrict__ rpm_in, int n_sub, R* __restrict__ traj) {
  __shared__ R sx[MULTI ? 2 * kWave : 1], sy[MULTI ? 2 * kWave : 1], sz[MULTI ? 2 * kWave : 1];
  const Consts<R>& c = *cp;
  const int tid = threadIdx.x;
  const int D = MULTI ? v.D : 1;
  const int d = MULTI ? tid % D : 0;
  const int base = tid - d;
  const long long n = (long long)blockIdx.x * v.tpb + tid;
  const bool active = tid < v.tpb && n < v.N;
  const long long nn = active ? n : (long long)blockIdx.x * v.tpb;   // the block's first drone (step_kernel)
  (void)d;
  const long long nleft = v.N - (long long)blockIdx.x * v.tpb;
  const int nact = (int)(nleft < v.tpb ? nleft : v.tpb);
  Drone<R> s;
  R last[4];
  load_drone<R, STREAM>(v, nn, s, last, true);
  const long long N = v.N;
  DynK<R> dk = dyn_consts(c);
  const DcPairs dcp = dc_enabled<MULTI, PF>(c.flags) ? dc_pairs_for(v, tid, nact) : dc_pairs_none();
  // RPMs are loaded two substeps ahead of their use (substeps t+1 and t+2 in flight while t
  // integrates): more bytes in flight per wave for the HBM stream.  A drone's 4 RPMs are one
  // aligned 4*sizeof(R)-byte vector (rows of the [T][N][4] tensor).
  using V = typename std::conditional<sizeof(R) == 8, double2, float4>::type;
  auto load4 = [&](int t, R out[4]) {
    const R* src = rpm_in + ((long long)t * N + nn) * 4;
    typedef double gpd_d2 __attribute__((ext_vector_type(2)));
    typedef float gpd_f4 __attribute__((ext_vector_type(4)));
    if (sizeof(R) == 8) {
      gpd_d2 a, b;
      if (STREAM) {
        a = __builtin_nontemporal_load(reinterpret_cast<const gpd_d2*>(src));
        b = __builtin_nontemporal_load(reinterpret_cast<const gpd_d2*>(src) + 1);
      } else {
        a = reinterpret_cast<const gpd_d2*>(src)[0];
        b = reinterpret_cast<const gpd_d2*>(src)[1];
      }
      out[0] = (R)a.x; out[1] = (R)a.y; out[2] = (R)b.x; out[3] = (R)b.y;
    } else {
      const gpd_f4 a = STREAM ? __builtin_nontemporal_load(reinterpret_cast<const gpd_f4*>(src))
                              : *reinterpret_cast<const gpd_f4*>(src);
      out[0] = (R)a.x; out[1] = (R)a.y; out[2] = (R)a.z; out[3] = (R)a.w;
    }
  };
  (void)sizeof(V);
  R nxt[4], nxt2[4];
  if (n_sub > 0) load4(0, nxt);
  if (n_sub > 1) load4(1, nxt2);
  for (int t = 0; t < n_sub; ++t) {
    R rpm[4] = {nxt[0], nxt[1], nxt[2], nxt[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) nxt[k] = nxt2[k];
    if (t + 2 < n_sub) load4(t + 2, nxt2);
    R W[4];
    rpm_wrench<R, PF>(rpm, dk, c, W);
    substep_block<R, MULTI, PF>(s, rpm, W, last, c, dk, sx, sy, sz, tid, base, D, DwPairs{0, 0}, nullptr, dcp);
#pragma unroll
    for (int k = 0; k < 4; ++k) last[k] = rpm[k];
    if (TRAJ && active) {   // TRAJ: the trajectory variant (its readback / Euler registers stay out of the other)
      R qn[4], roll, pitch, yaw;   // the literal Bullet readback (as state20): exact gimbal branches
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
  if (!active) return;
  if (n_sub == 0) return;
  store_drone<R, STREAM>(v, n, s, last);
}

// ---------------------------------------------------------------------------------------
// gpd_reset: masked re-initialisation (+ reset observation rows).
template <typename R>
__global__ __launch_bounds__(256) void reset_kernel(SimView<R> v, const uint8_t* __restrict__ mask, float* obs) {
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
  const int head = v.ctr[e].y;
  if (d == 0) v.ctr[e].x = 0;
  if (obs) {
    float* orow = obs + n * v.W;
    orow[0] = (float)ini[0]; orow[1] = (float)ini[1]; orow[2] = (float)ini[2];
    orow[3] = (float)ini[7]; orow[4] = (float)ini[8]; orow[5] = (float)ini[9];
    for (int k = 6; k < 12; ++k) orow[k] = 0.0f;
    const int A = v.A;
    for (int k = 0; k < v.ring_len; ++k) {   // oldest first: the slot about to be overwritten
      int slot = head + k;
      slot -= slot >= v.ring_len ? v.ring_len : 0;
      const float* src = v.ring + ridx(n, slot, v.ring_len, A);
      for (int j = 0; j < A; ++j) orow[12 + k * A + j] = src[j];
    }
  }
}

// last_clipped_action back into the state (store_drone_step): when ctr[E].x is set, drone n's
// state[16..19] = action_to_rpm of its ring's newest slot (head - 1 after the step; the same
// float32 mapping as the step, _preprocessAction BaseRLAviary.py:191-192), or 0 when its env's
// step_counter is 0 (_housekeeping zeroes last_clipped_action, BaseAviary.py:466).  The caller
// clears the mark afterwards (stream order).
template <typename R>
__global__ __launch_bounds__(256) void last_from_ring_kernel(SimView<R> v, const Consts<R>* __restrict__ c) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  if (v.ctr[v.N / v.D].x == 0) return;
  const int2 cv = v.ctr[n / v.D];
  R last[4] = {R(0), R(0), R(0), R(0)};
  if (cv.x != 0) {
    const int slot = cv.y == 0 ? v.ring_len - 1 : cv.y - 1;
    const float* a = v.ring + ridx(n, slot, v.ring_len, v.A);
    const float hover = c->hover_f32;
    for (int k = 0; k < 4; ++k) last[k] = (R)action_to_rpm(hover, a[v.A == 4 ? k : 0]);
  }
  for (int k = 0; k < 4; ++k) v.state[tidx(n, 16 + k, kStateComps)] = last[k];
}

// state20 (BaseAviary._getDroneStateVector :541-561, literal Bullet readback) / raw transposes
template <typename R>
__global__ __launch_bounds__(256) void state20_kernel(SimView<R> v, R* __restrict__ out, int raw) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  R* o = out + n * 20;
  if (raw) {
    for (int k = 0; k < 20; ++k) o[k] = v.state[tidx(n, k, kStateComps)];
    return;
  }
  Drone<R> s;
  R last[4];
  load_drone_full(v, n, s, last);
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

// Per-env non-finite guard: flag[e] = 1 when any drone of env e holds a
// non-finite integrated state component (pos, stored quat, vel, rates, ang_v), e.g. after the
// downwash quotient's beta = 0 edge (BaseAviary.py:802-804).  flag is zeroed by the caller;
// several drones of one env may store the same 1.
template <typename R>
__global__ __launch_bounds__(256) void nonfinite_kernel(SimView<R> v, uint8_t* __restrict__ flag) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 16; ++k) bad = bad || !isfinite(v.state[tidx(n, k, kStateComps)]);
  if (bad) flag[n / v.D] = 1;
}

template <typename R>
__global__ __launch_bounds__(256) void set_raw_kernel(SimView<R> v, const R* __restrict__ in) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= v.N) return;
  for (int k = 0; k < 20; ++k) v.state[tidx(n, k, kStateComps)] = in[n * 20 + k];
}

// tiled SoA <-> [N][comps] rows (controller state access)
template <typename R>
__global__ __launch_bounds__(256) void soa_to_rows_kernel(const R* __restrict__ soa, long long npad, int comps, int N,
                                                          R* __restrict__ out) {
  (void)npad;
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int k = 0; k < comps; ++k) out[n * comps + k] = soa[tidx(n, k, comps)];
}
template <typename R>
__global__ __launch_bounds__(256) void rows_to_soa_kernel(const R* __restrict__ in, long long npad, int comps, int N,
                                                          R* __restrict__ soa) {
  (void)npad;
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int k = 0; k < comps; ++k) soa[tidx(n, k, comps)] = in[n * comps + k];
}

}  // namespace gpd
