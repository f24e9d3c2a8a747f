// gpd_policy.hip — fused rollout policy (include/gpd_policy.h) for gfx950.
//
// The reference's caller of the hot path is stable-baselines3 PPO (examples/learn.py:52-94):
// per env.step its rollout runs the actor + critic MLPs ([64, 64] tanh, separate networks:
// SB3 MlpPolicy), samples Normal(mu, exp(log_std)), clips to the Box and writes the rollout
// buffer; after env.step it bootstraps time-limit truncations with V(terminal_observation).
// Eager, that is ~25 library launches per step (bench.py rollout leg: 62.9 us of policy beside a
// 5.9 us env step).  Here it is ONE kernel per step:
//
//   * a block stages both networks' first two layers in LDS (float4-interleaved so that lane j
//     reads neuron j's four weights of k..k+3 in one conflict-free ds_read_b128), then loops over
//     groups of kWaves x kRows rows;
//   * lane j of a wave is hidden neuron j, for kRows rows at once (register blocking: every
//     weight read from LDS feeds kRows FMAs); the rows' inputs are broadcast LDS reads;
//   * the output layers (n_act + 1 dot products of 64) are wave butterfly reductions;
//   * lane r < kRows then finishes row r: the Philox4x32-10 / Box-Muller sample, the clip, the
//     Normal log-density written as torch.distributions.Normal.log_prob computes it, the stores.
//
// The MLP is VALU f32 FMA work (~12-18 K MACs per row): at 4096 rows a few microseconds, the
// weight staging (40-75 KB per block from L2) and the layer-to-layer dependency chain dominate.
// No MFMA: f32 MFMA runs at the VALU's rate on CDNA4 and bf16 would not reproduce the torch
// forward to f32 rounding.  Built with -ffp-contract=off: the MLP's FMAs are explicit fmaf, and
// everything written "as torch computes it" (the sample, the log-density, the bootstrap, GAE)
// rounds every operation as torch's elementwise kernels do.
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
constexpr int kRows = 4;                // rows per wave pass
constexpr int kWaves = 4;               // waves per block
constexpr int kBlock = kWaves * 64;
constexpr int kGroup = kWaves * kRows;  // rows per block pass

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
  const float u0 = u01(c[2 * p]), u1 = u01(c[2 * p + 1]);
  const float rad = sqrtf(-2.0f * logf(u0));
  float s, co;
  sincosf(6.283185307179586f * u1, &s, &co);
  return (a & 1) ? rad * s : rad * co;
}

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// LDS layout (floats): w1 pi | w1 vf  [kq][64][4] each,  w2 pi | w2 vf  [16][64][4] each,
// then per wave: x [kRows][kq*4], h pi [kRows][64], h vf [kRows][64], res [kRows][kRes]
struct Lds {
  float4 *w1p, *w1v, *w2p, *w2v;
  float *x, *hp, *hv, *res;   // res: [kRows][kRes] per wave, the output sums handed to lane r
};
constexpr int kRes = 16;

// Weight staging: row-major nn.Linear weights [64][n] -> LDS [n/4][64][4] (float4 q of neuron j
// at q * 64 + j).  Element idx -> (q = idx / 64, j = idx % 64): consecutive lanes write consecutive
// LDS float4s; every lane issues all its loads before its first store, so a block's ~70 KB arrive
// in one L2 round trip instead of one per loop iteration (the first build's scalar loop of
// dependent load -> store pairs took ~20 us of a 24 us launch).
template <int U>
__device__ inline void stage_rows4(float4* __restrict__ dst, const float* __restrict__ w, int n, int kq) {
  const int total = kq * H;
  const bool vec = (n & 3) == 0 && ((uintptr_t)w & 15) == 0;
  for (int base = threadIdx.x; base < total; base += U * kBlock) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * kBlock;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < total) {
        const int q = idx >> 6, j = idx & 63, k = 4 * q;
        const float* src = w + (size_t)j * n + k;
        if (vec) {
          v[u] = *reinterpret_cast<const float4*>(src);
        } else {
          v[u].x = src[0];
          v[u].y = k + 1 < n ? src[1] : 0.0f;
          v[u].z = k + 2 < n ? src[2] : 0.0f;
          v[u].w = k + 3 < n ? src[3] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * kBlock;
      if (idx < total) dst[idx] = v[u];
    }
  }
}

// hidden layers of one network for the wave's kRows rows: x (LDS rows) -> h2 in `h` (lane = neuron)
struct Bias {
  float p1, v1, p2, v2;   // neuron `lane`'s first / second layer biases (actor, critic)
};
template <bool BOTH>
__device__ inline void hidden(const Lds& s, const Args& A, const Bias& B, float (&hp)[kRows], float (&hv)[kRows],
                              int lane) {
  float ap[kRows], av[kRows];
  const float bp = B.p1, bv = B.v1;
#pragma unroll
  for (int r = 0; r < kRows; ++r) { ap[r] = bp; av[r] = bv; }
  const float4* x4 = (const float4*)s.x;
  for (int q = 0; q < A.kq; ++q) {
    const float4 wv = s.w1v[q * H + lane];
    float4 wp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (BOTH) wp = s.w1p[q * H + lane];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const float4 x = x4[r * A.kq + q];
      av[r] = fmaf(wv.x, x.x, av[r]); av[r] = fmaf(wv.y, x.y, av[r]);
      av[r] = fmaf(wv.z, x.z, av[r]); av[r] = fmaf(wv.w, x.w, av[r]);
      if (BOTH) {
        ap[r] = fmaf(wp.x, x.x, ap[r]); ap[r] = fmaf(wp.y, x.y, ap[r]);
        ap[r] = fmaf(wp.z, x.z, ap[r]); ap[r] = fmaf(wp.w, x.w, ap[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    s.hv[r * H + lane] = tanhf(av[r]);
    if (BOTH) s.hp[r * H + lane] = tanhf(ap[r]);
  }
  __syncthreads();
  const float b2p = B.p2, b2v = B.v2;
#pragma unroll
  for (int r = 0; r < kRows; ++r) { ap[r] = b2p; av[r] = b2v; }
  const float4* hv4 = (const float4*)s.hv;
  const float4* hp4 = (const float4*)s.hp;
#pragma unroll 4
  for (int q = 0; q < H / 4; ++q) {
    const float4 wv = s.w2v[q * H + lane];
    float4 wp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (BOTH) wp = s.w2p[q * H + lane];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const float4 y = hv4[r * (H / 4) + q];
      av[r] = fmaf(wv.x, y.x, av[r]); av[r] = fmaf(wv.y, y.y, av[r]);
      av[r] = fmaf(wv.z, y.z, av[r]); av[r] = fmaf(wv.w, y.w, av[r]);
      if (BOTH) {
        const float4 z = hp4[r * (H / 4) + q];
        ap[r] = fmaf(wp.x, z.x, ap[r]); ap[r] = fmaf(wp.y, z.y, ap[r]);
        ap[r] = fmaf(wp.z, z.z, ap[r]); ap[r] = fmaf(wp.w, z.w, ap[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    hv[r] = tanhf(av[r]);
    hp[r] = BOTH ? tanhf(ap[r]) : 0.0f;
  }
  __syncthreads();   // the next pass rewrites x / h of this wave
}

// rows [row0, row0 + kRows) of `src` (n_obs wide) -> the wave's x tile (zero past n_rows / n_obs);
// `copy` (nullable) receives the same rows (buf_obs)
__device__ inline void load_rows(const Lds& s, const Args& A, const float* __restrict__ src, int row0, int lane,
                                 float* copy) {
  const int w = A.kq * 4;
  for (int i = lane; i < kRows * w; i += 64) {
    const int r = i / w, k = i - r * w;
    const int row = row0 + r;
    float v = 0.0f;
    if (row < A.n_rows && k < A.n_obs) {
      v = src[(size_t)row * A.n_obs + k];
      if (copy) copy[(size_t)row * A.n_obs + k] = v;
    }
    s.x[i] = v;
  }
}

template <int NA>
__global__ void __launch_bounds__(kBlock) rollout_kernel(Args A) {
  extern __shared__ float4 lds4[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Lds s;
  s.w1p = lds4;
  s.w1v = s.w1p + A.kq * H;
  s.w2p = s.w1v + A.kq * H;
  s.w2v = s.w2p + (H / 4) * H;
  float* scratch = (float*)(s.w2v + (H / 4) * H);
  const int per_wave = kRows * A.kq * 4 + 2 * kRows * H + kRows * kRes;
  s.x = scratch + wave * per_wave;
  s.hp = s.x + kRows * A.kq * 4;
  s.hv = s.hp + kRows * H;
  s.res = s.hv + kRows * H;

  stage_rows4<8>(s.w1v, A.vf.w1, A.n_obs, A.kq);
  stage_rows4<4>(s.w2v, A.vf.w2, H, H / 4);
  if (A.actor) {
    stage_rows4<8>(s.w1p, A.pi.w1, A.n_obs, A.kq);
    stage_rows4<4>(s.w2p, A.pi.w2, H, H / 4);
  }
  uint64_t seed = 0, call = 0;
  if (A.sample) { seed = A.rng[0]; call = A.rng[1]; }
  Bias B;
  B.v1 = A.vf.b1[lane]; B.v2 = A.vf.b2[lane];
  B.p1 = A.actor ? A.pi.b1[lane] : 0.0f;
  B.p2 = A.actor ? A.pi.b2[lane] : 0.0f;
  // output-layer weights of neuron `lane`
  float w3p[NA], b3p[NA], scale[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    w3p[a] = A.actor ? A.pi.w3[a * H + lane] : 0.0f;
    b3p[a] = A.actor ? A.pi.b3[a] : 0.0f;
    scale[a] = A.actor ? expf(A.log_std[a]) : 1.0f;
  }
  const float w3v = A.vf.w3[lane], b3v = A.vf.b3[0];
  __syncthreads();

  for (int g0 = blockIdx.x * kGroup; g0 < A.n_rows; g0 += gridDim.x * kGroup) {
    const int row0 = g0 + wave * kRows;
    float hp[kRows], hv[kRows];
    // ---- the previous step: time-limit bootstrap + reward / done rows
    if (A.reward) {
      bool any = false;
      if (lane < kRows) {
        const int row = row0 + lane;
        any = row < A.n_rows && A.trunc[row] && !A.term[row];
      }
      if (__syncthreads_or(any)) {
        load_rows(s, A, A.tobs, row0, lane, nullptr);
        __syncthreads();
        hidden<false>(s, A, B, hp, hv, lane);
      } else {
#pragma unroll
        for (int r = 0; r < kRows; ++r) hv[r] = 0.0f;
      }
      float vb[kRows];
#pragma unroll
      for (int r = 0; r < kRows; ++r) vb[r] = wave_sum(w3v * hv[r]) + b3v;
      // every lane holds the sums; lane 0 hands them to lane r through LDS (a lane-indexed pick
      // from registers would go through scratch)
      if (lane == 0) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) s.res[r * kRes] = vb[r];
      }
      __syncthreads();
      if (lane < kRows) {
        const int row = row0 + lane;
        if (row < A.n_rows) {
          const float rw = A.reward[row];
          const bool te = A.term[row], tr = A.trunc[row];
          // learn.py: r + gamma * V(terminal_obs) (two roundings; this file has no contraction)
          A.buf_rew[row] = (tr && !te) ? rw + A.gamma * s.res[lane * kRes] : rw;
          A.buf_done[row] = (te || tr) ? 1.0f : 0.0f;
        }
      }
      __syncthreads();
    }
    if (!A.forward) continue;
    // ---- this step: actor + critic on obs
    load_rows(s, A, A.obs, row0, lane, A.buf_obs);
    __syncthreads();
    if (A.actor) hidden<true>(s, A, B, hp, hv, lane);
    else hidden<false>(s, A, B, hp, hv, lane);
    float val[kRows], mu[NA][kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      val[r] = wave_sum(w3v * hv[r]) + b3v;
#pragma unroll
      for (int a = 0; a < NA; ++a) mu[a][r] = A.actor ? wave_sum(w3p[a] * hp[r]) + b3p[a] : 0.0f;
    }
    // lane r < kRows finishes row r; lane 0 hands it the row's sums through LDS
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        s.res[r * kRes + NA] = val[r];
#pragma unroll
        for (int a = 0; a < NA; ++a) s.res[r * kRes + a] = mu[a][r];
      }
    }
    __syncthreads();
    if (lane < kRows) {
      const int row = row0 + lane;
      const float* my = s.res + lane * kRes;
      if (row < A.n_rows) {
        if (A.buf_val) A.buf_val[row] = my[NA];
        if (A.actor) {
          float logp = 0.0f;
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            const float m = my[a];
            float act = m;
            // torch Normal.rsample: loc + eps * scale (two roundings: no contraction in this file)
            if (!A.deterministic) act = m + std_normal(seed, call, row, a) * scale[a];
            // torch.distributions.Normal.log_prob:
            //   -((value - loc) ** 2) / (2 * var) - log(scale) - log(sqrt(2 * pi)),  var = scale ** 2
            const float d = act - m;
            const float lp = -(d * d) / (2.0f * (scale[a] * scale[a])) - logf(scale[a]) - 0.91893853320467274f;
            logp += lp;
            if (A.buf_act) A.buf_act[(size_t)row * NA + a] = act;
            if (A.act_env) A.act_env[(size_t)row * NA + a] = fminf(fmaxf(act, -1.0f), 1.0f);
          }
          if (A.buf_logp) A.buf_logp[row] = logp;
        }
      }
    }
    __syncthreads();   // res is rewritten by the next pass
  }
  // the last block to finish advances the call counter (every block has read it above)
  if (A.sample) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned long long t = atomicAdd((unsigned long long*)&A.rng[2], 1ull);
      if (t == gridDim.x - 1) {
        A.rng[1] = call + 1;
        A.rng[2] = 0;
        __threadfence();
      }
    }
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

template <int NA>
int launch(const Args& A, int grid, size_t lds, hipStream_t st) {
  // dynamic LDS past 64 KB must be allowed per kernel, up to what this launch needs
  static size_t allowed = 64 * 1024;
  if (lds > allowed) {
    const hipError_t e = hipFuncSetAttribute((const void*)rollout_kernel<NA>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) {
      (void)hipGetLastError();   // do not leave the error for the next caller's hipGetLastError
      return fail(kEhip, std::string("hipFuncSetAttribute(rollout_kernel, ") + std::to_string(lds) +
                             " B of dynamic LDS): " + hipGetErrorString(e));
    }
    allowed = lds;
  }
  hipLaunchKernelGGL(rollout_kernel<NA>, dim3(grid), dim3(kBlock), lds, st, A);
  HIP_TRY(hipGetLastError());
  return kOk;
}

}  // namespace

extern "C" {

int gpd_policy_abi_version(void) { return GPD_POLICY_ABI_VERSION; }
const char* gpd_policy_last_error(void) { return g_err.c_str(); }

int gpd_policy_rollout_step(const gpd_mlp_policy* p, int n_rows, const float* obs, float* act_env, float* buf_obs,
                            float* buf_act, float* buf_logp, float* buf_val, int deterministic, uint64_t* rng,
                            const float* reward, const uint8_t* terminated, const uint8_t* truncated,
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
  if (reward && (!terminated || !truncated || !terminal_obs || !buf_rew || !buf_done))
    return fail(kEinval, "gpd_policy_rollout_step: the bootstrap needs terminated, truncated, terminal_obs, "
                         "buf_rew and buf_done");
  if (!A.forward && !reward) return fail(kEinval, "gpd_policy_rollout_step: nothing to do (obs and reward NULL)");
  const size_t lds = sizeof(float) * ((size_t)2 * A.kq * 4 * H + (size_t)2 * H * H +
                                      (size_t)kWaves * (kRows * A.kq * 4 + 2 * kRows * H + kRows * kRes));
  static_assert(kRows * 4 <= 64, "rows per pass");
  const int groups = (n_rows + kGroup - 1) / kGroup;
  const int grid = groups < 1024 ? groups : 1024;
  hipStream_t st = (hipStream_t)stream;
  switch (p->n_act) {
    case 1: return launch<1>(A, grid, lds, st);
    case 2: return launch<2>(A, grid, lds, st);
    case 3: return launch<3>(A, grid, lds, st);
    case 4: return launch<4>(A, grid, lds, st);
    case 5: return launch<5>(A, grid, lds, st);
    case 6: return launch<6>(A, grid, lds, st);
    case 7: return launch<7>(A, grid, lds, st);
    default: return launch<8>(A, grid, lds, st);
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
