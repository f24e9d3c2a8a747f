// gpd_policy.hip — fused rollout policy (include/gpd_policy.h) for gfx950.
//
// The reference's caller of the hot path is stable-baselines3 PPO (examples/learn.py:52-94):
// per env.step its rollout runs the actor + critic MLPs ([64, 64] tanh, separate networks:
// SB3 MlpPolicy), samples Normal(mu, exp(log_std)), clips to the Box and writes the rollout
// buffer; after env.step it bootstraps time-limit truncations with V(terminal_observation).
// Eager, that is ~25 library launches per step (bench.py rollout leg: 62.9 us of policy beside a
// 5.9 us env step).  Here it is ONE kernel per step.
//
// A block of four waves takes groups of 16 rows (the M of v_mfma_f32_16x16x4_f32, f32 in / f32
// accumulate: the f32 rounding the torch forward has, at the f32 VALU's rate but with one
// 40-cycle dependent step per 4 x 16 x 16 products instead of 16 dependent FMAs).  Wave w owns
// hidden neurons 16w .. 16w+15 of both layers and both networks:
//   * its B operands - the slices of W1 and W2 it needs - are loaded ONCE into VGPRs at the start
//     (no LDS staging: every load in flight at once, one L2 round trip per launch);
//   * layer 1: the group's input rows, k-major in LDS, are the A operand; tanh(acc + b1) goes to
//     LDS (the next layer sums over neurons of all four waves);
//   * layer 2 likewise; its tanh stays in the accumulator registers;
//   * the output layer (n_act + 1 dot products of 64): per lane the products of its neuron, a
//     16-lane DPP butterfly per wave (row_mirror, row_half_mirror, two quad_perms: VALU, no LDS)
//     and the four waves' partial sums added through LDS in wave order;
//   * then one lane per (row, action): the Philox4x32-10 / Box-Muller sample, the clip, the Normal
//     log-density written as torch.distributions.Normal.log_prob computes it; one lane per row:
//     the log-probability sum, the value and the stores.
// The previous step's time-limit bootstrap, V(terminal row), runs in groups that hold a truncated
// env: a third MFMA chain (critic weights, terminal rows) beside the actor's and the critic's, in
// the same layer passes - its instruction sequence is the critic's, so the same bits as a forward
// of its own, at no extra dependent step.
// Built with -ffp-contract=off: everything written "as torch computes it" (the sample, the
// log-density, the bootstrap, GAE) rounds every operation as torch's elementwise kernels do.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/gpd_policy.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

constexpr int kOk = 0, kEinval = -1, kEhip = -2, kEunsupported = -4;   // gpd.h GPD_OK / GPD_E*

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(kEhip, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int H = GPD_POLICY_HIDDEN;
constexpr int kWaves = 4;                      // waves per block: neurons 16w .. 16w+15 each
constexpr int kBlock = kWaves * 64;
constexpr int kM = 16;                         // rows per group (MFMA M)
constexpr int kXs = kM + 1;                    // LDS row stride of the k-major tiles (odd: no bank conflicts)
constexpr int kRes = 16;                       // LDS stride of a row's outputs (n_act + 1 <= 9)
constexpr int kMaxKq = GPD_POLICY_MAX_OBS / 4;
typedef float f4 __attribute__((ext_vector_type(4)));

struct Net {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
};

struct Args {
  Net pi, vf;
  const float* log_std;
  int n_obs, kq, n_rows;               // kq = n_obs rounded up to 4, / 4
  const float* obs;
  float *act_env, *buf_obs, *buf_act, *buf_logp, *buf_val;
  int deterministic, sample, forward, actor;
  uint64_t* rng;
  const float* reward;
  const uint8_t *term, *trunc;
  const float* tobs;
  float gamma;
  float *buf_rew, *buf_done;
};

// ---- Philox4x32-10 (Salmon et al., SC'11): counter (row, sub, call lo, call hi), key = seed
__device__ inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int i = 0; i < 10; ++i) {
    const uint32_t h0 = __umulhi(0xD2511F53u, c[0]), l0 = 0xD2511F53u * c[0];
    const uint32_t h1 = __umulhi(0xCD9E8D57u, c[2]), l1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
__device__ inline float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }   // (0, 1)

// standard normal number `a` (< 8) of `row` for call `call`
__device__ inline float std_normal(uint64_t seed, uint64_t call, int row, int a) {
  uint32_t c[4] = {(uint32_t)row, (uint32_t)(a >> 2), (uint32_t)call, (uint32_t)(call >> 32)};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const int p = (a & 3) >> 1;                       // Box-Muller pair (c0, c1) or (c2, c3)
  const float u0 = u01(p ? c[2] : c[0]), u1 = u01(p ? c[3] : c[1]);
  const float rad = sqrtf(-2.0f * logf(u0));
  float s, co;
  sincosf(6.283185307179586f * u1, &s, &co);
  return (a & 1) ? rad * s : rad * co;
}

template <int CTRL>
__device__ inline float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// the sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15), in every lane of the row
__device__ inline float row16_sum(float v) {
  v += dpp<0x140>(v);   // row_mirror: i <-> 15 - i
  v += dpp<0x141>(v);   // row_half_mirror: i <-> 7 - i within each half
  v += dpp<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += dpp<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  return v;
}

struct Lds {
  float xt[kMaxKq * 4 * kXs];      // the group's input rows, k-major: xt[k * kXs + row]
  float xb[kMaxKq * 4 * kXs];      // its terminal rows (bootstrap), the same layout
  float h1v[H * kXs], h1p[H * kXs], h1b[H * kXs];   // layer-1 activations, neuron-major
  float part[kWaves][kM][kRes];    // per wave: its 16 neurons' share of the output sums
  float res[kM][kRes];             // per row: mu[0..n_act), value at n_act, V(terminal row) at n_act + 1
  float lp[kM][GPD_POLICY_MAX_ACT];
  float b3[GPD_POLICY_MAX_ACT + 1];   // output biases: mu_0 .. mu_{n_act-1}, value
};

// This lane's slice of the weights: B operands W1[j][g KQ + s] (s < KQ), W2[j][16 g + s], output
// weights W3[o][j], biases of neuron j (j = 16 w + (l & 15), g = l >> 4).  The K index of MFMA
// step s and operand slot g is g KQ + s (not 4 s + g): a lane's weights of one layer are then
// contiguous in the row-major nn.Linear weight, so they arrive as float4 loads (a quarter of the
// load instructions; one scalar load per element took ~2 us of address processing per launch).
template <int NA, int KQ>
struct Regs {
  float w1v[KQ], w1p[KQ], w2v[16], w2p[16], w3p[NA], w3v, b1v, b1p, b2v, b2p;
  float sc;           // exp(log_std[a]) of this lane's action a = threadIdx.x % NA (sampling lanes)
};

template <int N>
__device__ inline void load_slice(float (&dst)[N], const float* __restrict__ row, int k0, int n, bool on) {
  // dst[s] = row[k0 + s] (0 past n or when !on); float4 / float2 loads when the slice is 16- / 8-B aligned
  if (N % 4 == 0 && on && (n & 3) == 0 && (k0 & 3) == 0 && ((uintptr_t)row & 15) == 0 && k0 + N <= n) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(row + k0)[q];
      dst[4 * q] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
    }
  } else if (N % 2 == 0 && on && (n & 1) == 0 && (k0 & 1) == 0 && ((uintptr_t)row & 7) == 0 && k0 + N <= n) {
#pragma unroll
    for (int q = 0; q < N / 2; ++q) {   // float2 (KQ = 18: the slices start 72 B apart)
      const float2 v = reinterpret_cast<const float2*>(row + k0)[q];
      dst[2 * q] = v.x; dst[2 * q + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int s = 0; s < N; ++s) dst[s] = on && k0 + s < n ? row[k0 + s] : 0.0f;
  }
}
template <int NA, int KQ>
__device__ inline void load_regs(const Args& A, Regs<NA, KQ>& R, int j, int g) {
  load_slice<KQ>(R.w1v, A.vf.w1 + (size_t)j * A.n_obs, g * KQ, A.n_obs, true);
  load_slice<KQ>(R.w1p, A.actor ? A.pi.w1 + (size_t)j * A.n_obs : A.vf.w1, g * KQ, A.n_obs, A.actor);
  load_slice<16>(R.w2v, A.vf.w2 + (size_t)j * H, 16 * g, H, true);
  load_slice<16>(R.w2p, A.actor ? A.pi.w2 + (size_t)j * H : A.vf.w2, 16 * g, H, A.actor);
#pragma unroll
  for (int a = 0; a < NA; ++a) R.w3p[a] = A.actor ? A.pi.w3[a * H + j] : 0.0f;
  R.w3v = A.vf.w3[j];
  R.b1v = A.vf.b1[j]; R.b2v = A.vf.b2[j];
  R.b1p = A.actor ? A.pi.b1[j] : 0.0f;
  R.b2p = A.actor ? A.pi.b2[j] : 0.0f;
  R.sc = A.actor ? expf(A.log_std[threadIdx.x % NA]) : 1.0f;
}

// A group's rows [row0, row0 + 16) of `src` (n_obs wide) in registers (element idx = threadIdx.x +
// u * kBlock of the row-major 16 x kq*4 tile; zero past n_rows / n_obs): issued together with
// everything else the group needs, so a group costs one memory round trip.
template <int KQ>
struct RowRegs {
  static constexpr int U = (kM * KQ * 4 + kBlock - 1) / kBlock;
  float v[U];
};
template <int KQ>
__device__ inline void load_rows(RowRegs<KQ>& X, const Args& A, const float* __restrict__ src, int row0) {
  constexpr int w4 = KQ * 4;   // every k an MFMA step reads (zero past n_obs)
#pragma unroll
  for (int u = 0; u < RowRegs<KQ>::U; ++u) {
    const int idx = threadIdx.x + u * kBlock;
    const int i = idx / w4, k = idx - i * w4;
    const int row = row0 + i;
    X.v[u] = (idx < kM * w4 && row < A.n_rows && k < A.n_obs) ? src[(size_t)row * A.n_obs + k] : 0.0f;
  }
}
// ... -> L.xt (k-major, conflict-free writes: odd row stride); `copy` (nullable) receives the rows (buf_obs)
template <int KQ>
__device__ inline void stage_rows(float* xt, const Args& A, const RowRegs<KQ>& X, int row0, float* copy) {
  constexpr int w4 = KQ * 4;
#pragma unroll
  for (int u = 0; u < RowRegs<KQ>::U; ++u) {
    const int idx = threadIdx.x + u * kBlock;
    if (idx < kM * w4) {
      const int i = idx / w4, k = idx - i * w4;
      const int row = row0 + i;
      xt[k * kXs + i] = X.v[u];
      if (copy && row < A.n_rows && k < A.n_obs) copy[(size_t)row * A.n_obs + k] = X.v[u];
    }
  }
}

// The group's forward pass (rows staged in L.xt / L.xb and synchronised by the caller):
//   ACT:  the actor on L.xt  -> L.res[row][a] = mu_a
//   CRIT: the critic on L.xt -> L.res[row][NA] = V(obs)
//   BOOT: the critic on L.xb -> L.res[row][NA + 1] = V(terminal row)
// Ends synchronised.
template <int NA, int KQ, bool ACT, bool CRIT, bool BOOT>
__device__ inline void forward(Lds& L, const Args& A, const Regs<NA, KQ>& R, int w, int l) {
  const int g = l >> 4, i = l & 15, j = 16 * w + i;
  f4 av = {0.f, 0.f, 0.f, 0.f}, ap = {0.f, 0.f, 0.f, 0.f}, ab = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KQ; ++s) {
    const int o = (g * KQ + s) * kXs + i;              // A[row i][k = g KQ + s]
    if (CRIT || ACT) {
      const float x = L.xt[o];
      if (CRIT) av = __builtin_amdgcn_mfma_f32_16x16x4f32(x, R.w1v[s], av, 0, 0, 0);
      if (ACT) ap = __builtin_amdgcn_mfma_f32_16x16x4f32(x, R.w1p[s], ap, 0, 0, 0);
    }
    if (BOOT) ab = __builtin_amdgcn_mfma_f32_16x16x4f32(L.xb[o], R.w1v[s], ab, 0, 0, 0);
  }
  // D[row 4g + r][col i] = neuron j of row 4g + r
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (CRIT) L.h1v[j * kXs + 4 * g + r] = tanhf(av[r] + R.b1v);
    if (ACT) L.h1p[j * kXs + 4 * g + r] = tanhf(ap[r] + R.b1p);
    if (BOOT) L.h1b[j * kXs + 4 * g + r] = tanhf(ab[r] + R.b1v);
  }
  __syncthreads();
  av = f4{0.f, 0.f, 0.f, 0.f};
  ap = f4{0.f, 0.f, 0.f, 0.f};
  ab = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int o = (16 * g + s) * kXs + i;
    if (CRIT) av = __builtin_amdgcn_mfma_f32_16x16x4f32(L.h1v[o], R.w2v[s], av, 0, 0, 0);
    if (ACT) ap = __builtin_amdgcn_mfma_f32_16x16x4f32(L.h1p[o], R.w2p[s], ap, 0, 0, 0);
    if (BOOT) ab = __builtin_amdgcn_mfma_f32_16x16x4f32(L.h1b[o], R.w2v[s], ab, 0, 0, 0);
  }
  // output layer: this wave's 16 neurons' products, summed over the DPP row (the 16 lanes of one g)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float sv = 0.0f, sb = 0.0f, sp[NA];
    if (CRIT) sv = row16_sum(R.w3v * tanhf(av[r] + R.b2v));
    if (BOOT) sb = row16_sum(R.w3v * tanhf(ab[r] + R.b2v));
    if (ACT) {
      const float hp = tanhf(ap[r] + R.b2p);
#pragma unroll
      for (int a = 0; a < NA; ++a) sp[a] = row16_sum(R.w3p[a] * hp);
    }
    if (i == 0) {
      if (CRIT) L.part[w][4 * g + r][NA] = sv;
      if (BOOT) L.part[w][4 * g + r][NA + 1] = sb;
      if (ACT) {
#pragma unroll
        for (int a = 0; a < NA; ++a) L.part[w][4 * g + r][a] = sp[a];
      }
    }
  }
  __syncthreads();
  // the four waves' shares, in wave order, plus the output biases (the bootstrap's: the critic's)
  const int t = threadIdx.x;
  if (t < kM * (NA + 2)) {
    const int row = t / (NA + 2), o = t - row * (NA + 2);
    if ((ACT && o < NA) || (CRIT && o == NA) || (BOOT && o == NA + 1)) {
      float acc = L.part[0][row][o];
#pragma unroll
      for (int ww = 1; ww < kWaves; ++ww) acc += L.part[ww][row][o];
      L.res[row][o] = acc + L.b3[o < NA + 1 ? o : NA];   // (an index into R, even a select chain, puts R in scratch)
    }
  }
  __syncthreads();
}

// a group's loads: its terminal rows, flags and rewards (bootstrap) and its observation rows
template <int KQ>
__device__ inline void issue_group(const Args& A, RowRegs<KQ>& X, RowRegs<KQ>& TX, float& rw, bool& te, bool& tr,
                                   uint64_t& call, int row0, int t) {
  if (A.sample) call = A.rng[2 + row0 / kM];
  if (A.reward) {
    load_rows(TX, A, A.tobs, row0);
    const bool mine = t < kM && row0 + t < A.n_rows;
    rw = mine ? A.reward[row0 + t] : 0.0f;
    te = mine && A.term[row0 + t];
    tr = mine && A.trunc[row0 + t];
  }
  if (A.forward) load_rows(X, A, A.obs, row0);
}

template <int NA, int KQ>
__global__ void __launch_bounds__(kBlock) rollout_kernel(Args A) {
  __shared__ Lds L;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, t = threadIdx.x;
  // the Philox call counter of a row group is rng[2 + group]: read with the group's loads, moved on
  // by the block that samples the group (one reader-writer per counter and call: a plain load and
  // store; a single counter took one atomic per block, ~3.8 us of a sampled launch as 256 blocks
  // queued on one address: scripts/policy_probe.py graph, profiles/r6/policy/)
  const uint64_t seed = A.sample ? A.rng[0] : 0;
  // everything a group reads from memory is issued before anything waits for it; the block's
  // weight slices go out behind the first group's rows, the next group's loads behind this one's
  // stores (one memory round trip per group)
  RowRegs<KQ> X, TX;
  float rw = 0.0f;
  bool te = false, tr = false;
  uint64_t call = 0;
  int row0 = blockIdx.x * kM;
  const int stride = gridDim.x * kM;
  issue_group(A, X, TX, rw, te, tr, call, row0, t);
  Regs<NA, KQ> R;
  load_regs(A, R, 16 * w + (l & 15), l >> 4);
  if (t <= NA) L.b3[t] = t == NA ? A.vf.b3[0] : (A.actor ? A.pi.b3[t] : 0.0f);   // read after a barrier
  for (; row0 < A.n_rows; row0 += stride) {
    // the previous step's time-limit bootstrap (groups holding a truncated env) rides in this
    // step's forward as a third chain
    const bool boot = A.reward && __syncthreads_or(t < kM && tr && !te);
    if (A.forward) stage_rows(L.xt, A, X, row0, A.buf_obs);
    if (boot) stage_rows(L.xb, A, TX, row0, nullptr);
    if (A.forward || boot) {
      __syncthreads();
      if (!A.forward) forward<NA, KQ, false, false, true>(L, A, R, w, l);
      else if (A.actor && boot) forward<NA, KQ, true, true, true>(L, A, R, w, l);
      else if (A.actor) forward<NA, KQ, true, true, false>(L, A, R, w, l);
      else if (boot) forward<NA, KQ, false, true, true>(L, A, R, w, l);
      else forward<NA, KQ, false, true, false>(L, A, R, w, l);
    }
    // ---- the previous step's reward / done rows
    if (A.reward && t < kM && row0 + t < A.n_rows) {
      // learn.py: r + gamma * V(terminal_obs) (two roundings; this file has no contraction)
      A.buf_rew[row0 + t] = (tr && !te) ? rw + A.gamma * L.res[t][NA + 1] : rw;
      A.buf_done[row0 + t] = (te || tr) ? 1.0f : 0.0f;
    }
    if (!A.forward) {   // (the next group's first barrier orders these reads before its forward)
      if (row0 + stride < A.n_rows) issue_group(A, X, TX, rw, te, tr, call, row0 + stride, t);
      continue;
    }
    // ---- this step: the sample and the rows
    if (A.actor && t < kM * NA) {   // one lane per (row, action)
      const int i = t / NA, a = t - i * NA;
      const int row = row0 + i;
      const float m = L.res[i][a];
      const float sc = R.sc;
      float act = m;
      // torch Normal.rsample: loc + eps * scale (two roundings: no contraction in this file)
      if (!A.deterministic) act = m + std_normal(seed, call, row, a) * sc;
      // torch.distributions.Normal.log_prob:
      //   -((value - loc) ** 2) / (2 * var) - log(scale) - log(sqrt(2 * pi)),  var = scale ** 2
      const float d = act - m;
      L.lp[i][a] = -(d * d) / (2.0f * (sc * sc)) - logf(sc) - 0.91893853320467274f;
      if (row < A.n_rows) {
        if (A.buf_act) A.buf_act[(size_t)row * NA + a] = act;
        if (A.act_env) A.act_env[(size_t)row * NA + a] = fminf(fmaxf(act, -1.0f), 1.0f);
      }
    }
    if (A.sample && t == 0) A.rng[2 + row0 / kM] = call + 1;   // this group's counter moves on
    __syncthreads();
    if (t < kM) {
      const int row = row0 + t;
      if (row < A.n_rows) {
        if (A.buf_val) A.buf_val[row] = L.res[t][NA];
        if (A.actor && A.buf_logp) {
          float logp = 0.0f;
#pragma unroll
          for (int a = 0; a < NA; ++a) logp += L.lp[t][a];
          A.buf_logp[row] = logp;
        }
      }
    }
    if (row0 + stride < A.n_rows) issue_group(A, X, TX, rw, te, tr, call, row0 + stride, t);
    __syncthreads();   // res / lp are rewritten by the next group
  }
}

// GAE(gamma, lambda) per env, written as examples/learn.py's torch loop evaluates it (every
// operation rounded to f32: this file is compiled with -ffp-contract=off), so the result is
// bit-identical to it
__global__ void __launch_bounds__(256) gae_kernel(int T, int n, const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ done, const float* __restrict__ last_val,
                                                  float gamma, float gl, float* __restrict__ adv, float* __restrict__ ret) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = 0.0f;
  float nv = last_val[i];
  for (int t = T - 1; t >= 0; --t) {
    const size_t o = (size_t)t * n + i;
    const float v = val[o];
    const float nonterm = 1.0f - done[o];
    const float delta = (rew[o] + (gamma * nv) * nonterm) - v;
    g = delta + (gl * nonterm) * g;
    adv[o] = g;
    ret[o] = g + v;
    nv = v;
  }
}

template <int NA, int KQ>
int launch(const Args& A, int grid, hipStream_t st) {
  hipLaunchKernelGGL((rollout_kernel<NA, KQ>), dim3(grid), dim3(kBlock), 0, st, A);
  HIP_TRY(hipGetLastError());
  return kOk;
}
// the weight slices live in VGPRs: the layer-1 slice sized by the obs width's bucket (18 / 36:
// the KIN observation of one / two RPM drones, 72 / 144 wide, without padding MFMA steps)
template <int NA>
int launch_kq(const Args& A, int grid, hipStream_t st) {
  if (A.kq <= 8) return launch<NA, 8>(A, grid, st);
  if (A.kq <= 16) return launch<NA, 16>(A, grid, st);
  if (A.kq <= 18) return launch<NA, 18>(A, grid, st);
  if (A.kq <= 24) return launch<NA, 24>(A, grid, st);
  if (A.kq <= 36) return launch<NA, 36>(A, grid, st);
  return launch<NA, kMaxKq>(A, grid, st);
}

}  // namespace

extern "C" {

int gpd_policy_abi_version(void) { return GPD_POLICY_ABI_VERSION; }
const char* gpd_policy_last_error(void) { return g_err.c_str(); }

int gpd_policy_rollout_step(const gpd_mlp_policy* p, int n_rows, const float* obs, float* act_env, float* buf_obs,
                            float* buf_act, float* buf_logp, float* buf_val, int deterministic, uint64_t* rng,
                            int rng_groups, const float* reward, const uint8_t* terminated, const uint8_t* truncated,
                            const float* terminal_obs, float gamma, float* buf_rew, float* buf_done, void* stream) {
  if (!p) return fail(kEinval, "gpd_policy_rollout_step: NULL policy");
  if (n_rows < 1) return fail(kEinval, "gpd_policy_rollout_step: n_rows < 1");
  if (p->n_obs < 1 || p->n_obs > GPD_POLICY_MAX_OBS)
    return fail(kEunsupported, "gpd_policy_rollout_step: n_obs must be in [1, " +
                                   std::to_string(GPD_POLICY_MAX_OBS) + "]");
  if (p->n_act < 1 || p->n_act > GPD_POLICY_MAX_ACT)
    return fail(kEunsupported, "gpd_policy_rollout_step: n_act must be in [1, 8]");
  if (!p->vf_w1 || !p->vf_b1 || !p->vf_w2 || !p->vf_b2 || !p->vf_w3 || !p->vf_b3)
    return fail(kEinval, "gpd_policy_rollout_step: NULL critic weight");
  Args A = {};
  A.pi = {p->pi_w1, p->pi_b1, p->pi_w2, p->pi_b2, p->pi_w3, p->pi_b3};
  A.vf = {p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->vf_w3, p->vf_b3};
  A.log_std = p->log_std;
  A.n_obs = p->n_obs;
  A.kq = (p->n_obs + 3) / 4;
  A.n_rows = n_rows;
  A.obs = obs; A.act_env = act_env; A.buf_obs = buf_obs; A.buf_act = buf_act; A.buf_logp = buf_logp;
  A.buf_val = buf_val;
  A.deterministic = deterministic ? 1 : 0;
  A.actor = obs && (act_env || buf_act || buf_logp);
  A.forward = obs != nullptr;
  A.sample = A.actor && !A.deterministic;
  A.rng = rng;
  A.reward = reward; A.term = terminated; A.trunc = truncated; A.tobs = terminal_obs; A.gamma = gamma;
  A.buf_rew = buf_rew; A.buf_done = buf_done;
  if (A.actor && (!p->pi_w1 || !p->pi_b1 || !p->pi_w2 || !p->pi_b2 || !p->pi_w3 || !p->pi_b3 || !p->log_std))
    return fail(kEinval, "gpd_policy_rollout_step: NULL actor weight");
  if (A.sample && !rng) return fail(kEinval, "gpd_policy_rollout_step: sampling needs the rng state");
  if (A.sample && (long long)rng_groups * kM < n_rows)
    return fail(kEinval, "gpd_policy_rollout_step: rng holds " + std::to_string(rng_groups) +
                             " row-group counters, sampling " + std::to_string(n_rows) + " rows needs " +
                             std::to_string((n_rows + kM - 1) / kM));
  if (reward && (!terminated || !truncated || !terminal_obs || !buf_rew || !buf_done))
    return fail(kEinval, "gpd_policy_rollout_step: the bootstrap needs terminated, truncated, terminal_obs, "
                         "buf_rew and buf_done");
  if (!A.forward && !reward) return fail(kEinval, "gpd_policy_rollout_step: nothing to do (obs and reward NULL)");
  const int groups = (n_rows + kM - 1) / kM;
  const int grid = groups < 2048 ? groups : 2048;
  hipStream_t st = (hipStream_t)stream;
  switch (p->n_act) {
    case 1: return launch_kq<1>(A, grid, st);
    case 2: return launch_kq<2>(A, grid, st);
    case 3: return launch_kq<3>(A, grid, st);
    case 4: return launch_kq<4>(A, grid, st);
    case 5: return launch_kq<5>(A, grid, st);
    case 6: return launch_kq<6>(A, grid, st);
    case 7: return launch_kq<7>(A, grid, st);
    default: return launch_kq<8>(A, grid, st);
  }
}

int gpd_policy_gae(int n_steps, int n_rows, const float* rew, const float* val, const float* done,
                   const float* last_val, double gamma, double lam, float* adv, float* ret, void* stream) {
  if (n_steps < 1 || n_rows < 1 || !rew || !val || !done || !last_val || !adv || !ret)
    return fail(kEinval, "gpd_policy_gae: invalid argument");
  // examples/learn.py: gamma * gae_lambda is a Python (double) product; torch rounds a Python
  // scalar to the tensor's f32 once per operation
  const float gf = (float)gamma, gl = (float)(gamma * lam);
  hipLaunchKernelGGL(gae_kernel, dim3((n_rows + 255) / 256), dim3(256), 0, (hipStream_t)stream, n_steps, n_rows,
                     rew, val, done, last_val, gf, gl, adv, ret);
  HIP_TRY(hipGetLastError());
  return kOk;
}

}  // extern "C"
