// Achievable HBM rate on this box (the ceiling the large-N step rows are quoted against, DESIGN.md
// §7.1): coalesced float4 streams far past the 256 MB Infinity Cache, with U independent 16-B
// loads in flight per lane (U = 1 is scripts/ubench/rw_mix.hip's shape), plain or nontemporal,
// at 1..8 blocks of 256 threads per CU.  Shapes: copy 1:1, read-only, fill, and the step
// kernel's 22 read : 29 written float4 per element (352 B read + 465 B written per drone, PMC).
// Reports GB/s of bytes moved (reads + writes), best of the sweep per shape at the end.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_ceiling hbm_ceiling.hip && ./hbm_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return -1.0;                                                                    \
    }                                                                                 \
  } while (0)
// (also built as libhbm_ceiling.so with -DHBM_CEILING_LIB -shared -fPIC: hbm_ceiling_gbps below)

template <bool NT>
__device__ __forceinline__ float4 ld(const float4* p) {
  if (NT) {
    float4 v;
    v.x = __builtin_nontemporal_load(&p->x); v.y = __builtin_nontemporal_load(&p->y);
    v.z = __builtin_nontemporal_load(&p->z); v.w = __builtin_nontemporal_load(&p->w);
    return v;
  }
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(float4* p, float4 v) {
  if (NT) {
    __builtin_nontemporal_store(v.x, &p->x); __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z); __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}

// R read streams and W write streams of n float4 each (stream k at offset k*n); every lane handles
// U elements per pass, 256 apart (coalesced), all U*R loads issued before the first store.
template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                     long long n) {
  const long long step = (long long)gridDim.x * 256 * U;
  for (long long b = (long long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += step) {
    float4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      float4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = b + u * 256;
        x[u] = i < n ? ld<NT>(src + k * n + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u].x += x[u].x; acc[u].y += x[u].y; acc[u].z += x[u].z; acc[u].w += x[u].w;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = b + u * 256;
      if (i >= n) continue;
      if (W == 0) {
        if (acc[u].x == -1.0f) dst[i] = acc[u];   // keeps a read-only pass's loads alive
      }
#pragma unroll
      for (int k = 0; k < W; ++k) st<NT>(dst + k * n + i, make_float4(acc[u].x + k, acc[u].y, acc[u].z, acc[u].w));
    }
  }
}

template <int R, int W, int U, bool NT>
double run(float4* src, float4* dst, long long n, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  stream_kernel<R, W, U, NT><<<blocks, 256>>>(src, dst, n);
  CHECK(hipDeviceSynchronize());
  const int reps = 8;
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) stream_kernel<R, W, U, NT><<<blocks, 256>>>(src, dst, n);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return (double)(R + W) * n * 16 / (ms / reps * 1e-3) / 1e9;
}

template <int R, int W>
double shape(const char* name, float4* src, float4* dst, long long n, bool print) {
  double best = 0;
  int bu = 0, bb = 0, bnt = 0;
  for (int bpc : {1, 2, 4, 8}) {
    const int blocks = 256 * bpc;
    double g[8];
    g[0] = run<R, W, 1, false>(src, dst, n, blocks);
    g[1] = run<R, W, 2, false>(src, dst, n, blocks);
    g[2] = run<R, W, 4, false>(src, dst, n, blocks);
    g[3] = run<R, W, 8, false>(src, dst, n, blocks);
    g[4] = run<R, W, 1, true>(src, dst, n, blocks);
    g[5] = run<R, W, 2, true>(src, dst, n, blocks);
    g[6] = run<R, W, 4, true>(src, dst, n, blocks);
    g[7] = run<R, W, 8, true>(src, dst, n, blocks);
    if (print)
      std::printf("%-14s %d blocks/CU  plain U=1,2,4,8: %6.0f %6.0f %6.0f %6.0f   nt: %6.0f %6.0f %6.0f %6.0f GB/s\n",
                  name, bpc, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]);
    for (int k = 0; k < 8; ++k)
      if (g[k] > best) { best = g[k]; bu = 1 << (k & 3); bb = bpc; bnt = k >= 4; }
  }
  if (print) std::printf("BEST %-14s %6.0f GB/s  (U=%d, %d blocks/CU, %s)\n", name, best, bu, bb, bnt ? "nt" : "plain");
  return best;
}

// shape 0: copy 1:1, 1: read 1:0, 2: fill 0:1, 3: the step's 22:29; returns the best GB/s of the
// sweep (bench.py loads this as libhbm_ceiling.so: the large-N rows' achievable ceiling)
extern "C" double hbm_ceiling_gbps(int which, int print) {
  const long long n = 1 << 20;
  float4 *src = nullptr, *dst = nullptr;
  if (hipMalloc(&src, 22 * n * sizeof(float4)) != hipSuccess) return -1;
  if (hipMalloc(&dst, 29 * n * sizeof(float4)) != hipSuccess) { (void)hipFree(src); return -1; }
  (void)hipMemset(src, 0, 22 * n * sizeof(float4));
  (void)hipMemset(dst, 0, 29 * n * sizeof(float4));
  double r = -1;
  if (which == 0) r = shape<1, 1>("copy 1:1", src, dst, 22 * n, print);
  if (which == 1) r = shape<1, 0>("read 1:0", src, dst, 22 * n, print);
  if (which == 2) r = shape<0, 1>("fill 0:1", src, dst, 29 * n, print);
  if (which == 3) r = shape<22, 29>("step 22:29", src, dst, n, print);
  (void)hipDeviceSynchronize();
  (void)hipFree(src);
  (void)hipFree(dst);
  return r;
}

#ifndef HBM_CEILING_LIB
int main() {
  for (int k = 0; k < 4; ++k)
    if (hbm_ceiling_gbps(k, 1) < 0) return 1;
  return 0;
}
#endif
