// Achievable HBM rate on this box for the step kernel's traffic shape at large N:
// per element, read R float4 and write W float4 from / to arrays far larger than the 256 MB
// Infinity Cache, coalesced (16 B per lane, consecutive lanes), grid-stride, plain or
// write-through (sc1) stores like the step kernel's.  The step kernel moves 352 B read +
// 465 B written per drone (PMC), i.e. R:W = 22:29 float4.  Reports GB/s of bytes moved.
//   hipcc --offload-arch=gfx950 -O3 -o rw_mix rw_mix.hip && ./rw_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

// src: R streams of n float4, dst: W streams of n float4 (stream k at offset k * n)
template <int R, int W, bool WT>
__global__ __launch_bounds__(256) void rw_kernel(const float4* __restrict__ src, float4* __restrict__ dst, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const float4 x = src[k * n + i];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    if (W == 0 && acc.x == -1.0f) dst[i] = acc;   // keeps a read-only pass's loads alive
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const float4 y = make_float4(acc.x + k, acc.y, acc.z, acc.w);
      if (WT && (k * n + i) * 16 < 0x7fffffffLL) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, y), rs, (int)((k * n + i) * 16), 0, 16);
      } else {
        dst[k * n + i] = y;
      }
    }
  }
}

template <int R, int W, bool WT>
int run(const char* name, float4* src, float4* dst, long long n, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  rw_kernel<R, W, WT><<<blocks, 256>>>(src, dst, n);
  CHECK(hipDeviceSynchronize());
  const int reps = 10;
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) rw_kernel<R, W, WT><<<blocks, 256>>>(src, dst, n);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)(R + W) * n * 16;
  std::printf("%-28s %8.0f GB/s  (%.1f MB per launch, %.1f us)\n", name, bytes / (ms / reps * 1e-3) / 1e9,
              bytes / 1e6, ms / reps * 1e3);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

int main() {
  // 22 read streams + 29 write streams of n float4: n = 1M -> 352 MB + 464 MB, like 1M drones
  const long long n = 1 << 20;
  float4 *src = nullptr, *dst = nullptr;
  CHECK(hipMalloc(&src, 22 * n * sizeof(float4)));
  CHECK(hipMalloc(&dst, 29 * n * sizeof(float4)));
  CHECK(hipMemset(src, 0, 22 * n * sizeof(float4)));
  CHECK(hipMemset(dst, 0, 29 * n * sizeof(float4)));
  const int blocks = 256 * 8;
  int rc = 0;
  rc |= run<1, 1, false>("copy 1:1", src, dst, 22 * n, blocks);
  rc |= run<0, 1, false>("fill 0:1", src, dst, 29 * n, blocks);
  rc |= run<1, 0, false>("read 1:0", src, dst, 22 * n, blocks);
  rc |= run<22, 29, false>("step shape 22:29", src, dst, n, blocks);
  rc |= run<22, 29, true>("step shape 22:29 wt stores", src, dst, n, blocks);
  rc |= run<22, 29, false>("step shape 22:29 4x grid", src, dst, n, blocks * 4);
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  return rc;
}
