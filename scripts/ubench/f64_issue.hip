// Micro-benchmark: issue cost and dependent latency of f64 VALU ops on one wave (gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -o f64_issue f64_issue.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void fma_chains(double* out, long long* cyc, int iters, double a, double b) {
  double x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) x[c] = __fma_rn(x[c], a, b);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void mul_chain32(float* out, long long* cyc, int iters, float a, float b) {
  float x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = __fmaf_rn(x[c], a, b);
  }
  const long long t1 = clock64();
  float s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


// FMA with three VGPR operands (per-lane a, b), 8 independent chains
__global__ void fma_vvv(double* out, long long* cyc, int iters, double a0, double b0) {
  double x[8], a[8], b[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    x[c] = threadIdx.x * 1e-3 + c;
    a[c] = a0 + threadIdx.x * 1e-9 * c;
    b[c] = b0 + threadIdx.x * 1e-12 * c;
  }
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = __fma_rn(x[c], a[c], b[c]);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// v_mul_f64 with two VGPR operands, 8 independent chains
__global__ void mul_vv(double* out, long long* cyc, int iters, double a0) {
  double x[8], a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    x[c] = threadIdx.x * 1e-3 + c;
    a[c] = a0 + threadIdx.x * 1e-12 * c;
  }
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = __dmul_rn(x[c], a[c]);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 32-bit integer VALU ops, 8 independent chains (v_xad/v_add_u32 class)
__global__ void int_vv(int* out, long long* cyc, int iters) {
  unsigned x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 7 + c;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = (x[c] ^ (x[(c + 1) & 7] + 0x9e3779b9u));
  }
  const long long t1 = clock64();
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  out[threadIdx.x] = (int)s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int CHAINS>
void run(double* d_out, long long* d_cyc, int iters) {
  long long cyc = 0;
  for (int rep = 0; rep < 3; ++rep) {
    fma_chains<CHAINS><<<1, 64>>>(d_out, d_cyc, iters, 0.999999, 1e-7);
    hipDeviceSynchronize();
  }
  hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
  const double n = (double)iters * 16 * CHAINS;
  printf("f64 fma, %d independent chain(s): %.2f cycles per instruction\n", CHAINS, cyc / n);
}

int main() {
  double* d_out;
  long long* d_cyc;
  hipMalloc(&d_out, 64 * 8);
  hipMalloc(&d_cyc, 8);
  const int iters = 4096;
  run<1>(d_out, d_cyc, iters);
  run<2>(d_out, d_cyc, iters);
  run<4>(d_out, d_cyc, iters);
  run<8>(d_out, d_cyc, iters);
  {  // the same 8 chains on a 16-lane wave (thin blocks): does the issue cost follow EXEC?
    long long c16 = 0;
    for (int rep = 0; rep < 3; ++rep) {
      fma_chains<8><<<1, 16>>>(d_out, d_cyc, iters, 0.999999, 1e-7);
      hipDeviceSynchronize();
    }
    hipMemcpy(&c16, d_cyc, 8, hipMemcpyDeviceToHost);
    printf("f64 fma, 8 chains, 16-lane wave: %.2f cycles per instruction\n", c16 / ((double)iters * 16 * 8));
    for (int rep = 0; rep < 3; ++rep) {
      fma_chains<1><<<1, 16>>>(d_out, d_cyc, iters, 0.999999, 1e-7);
      hipDeviceSynchronize();
    }
    hipMemcpy(&c16, d_cyc, 8, hipMemcpyDeviceToHost);
    printf("f64 fma, 1 chain, 16-lane wave: %.2f cycles per instruction\n", c16 / ((double)iters * 16));
  }
  long long cyc = 0;
  for (int rep = 0; rep < 3; ++rep) {
    mul_chain32<<<1, 64>>>((float*)d_out, d_cyc, iters, 0.999999f, 1e-7f);
    hipDeviceSynchronize();
  }
  hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("f32 fma, 8 independent chains: %.2f cycles per instruction\n", cyc / ((double)iters * 16 * 8));
  for (int rep = 0; rep < 3; ++rep) {
    fma_vvv<<<1, 64>>>(d_out, d_cyc, iters, 0.999999, 1e-7);
    hipDeviceSynchronize();
  }
  hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("f64 fma, 3 VGPR operands, 8 chains: %.2f cycles per instruction\n", cyc / ((double)iters * 16 * 8));
  for (int rep = 0; rep < 3; ++rep) {
    mul_vv<<<1, 64>>>(d_out, d_cyc, iters, 0.999999);
    hipDeviceSynchronize();
  }
  hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("f64 mul, 2 VGPR operands, 8 chains: %.2f cycles per instruction\n", cyc / ((double)iters * 16 * 8));
  for (int rep = 0; rep < 3; ++rep) {
    int_vv<<<1, 64>>>((int*)d_out, d_cyc, iters);
    hipDeviceSynchronize();
  }
  hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("u32 add+xor pairs, 8 chains: %.2f cycles per (add+xor)\n", cyc / ((double)iters * 16 * 8));
  return 0;
}
