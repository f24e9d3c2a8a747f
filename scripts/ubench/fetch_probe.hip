// FETCH_SIZE / WRITE_SIZE calibration (MI355X, gfx950): known bytes read from HBM by coalesced
// loads, and written by coalesced stores, of 4, 8 and 16 bytes per lane (the widths the step
// kernels use: f32 / f64 state components, float4 actions, ring slots and obs rows).  Each read
// kernel reads a 512 MiB buffer once (far beyond L2 and the 256 MiB MALL) and writes one float
// per thread; each write kernel fills the 512 MiB buffer once.  rocprofv3 --pmc FETCH_SIZE (and,
// in its own pass, WRITE_SIZE) over this binary gives the counters per kernel beside the exact
// byte counts printed here.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void read_kernel(const T* __restrict__ src, long long n, float* __restrict__ out) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (long long i = tid; i < n; i += stride) {
    const T v = src[i];
    const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc += f[k];
  }
  out[tid] = acc;
}

template <typename T>
__global__ void write_kernel(T* __restrict__ dst, long long n) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  T v;
  float* f = reinterpret_cast<float*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); ++k) f[k] = (float)(tid + k);
  for (long long i = tid; i < n; i += stride) dst[i] = v;
}

int main() {
  const size_t bytes = 512ull << 20;
  void* buf = nullptr;
  float* out = nullptr;
  const int blocks = 256 * 8, threads = 256;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, (size_t)blocks * threads * 4) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_kernel<float>, dim3(blocks), dim3(threads), 0, 0, (const float*)buf, (long long)(bytes / 4), out);
    hipLaunchKernelGGL(read_kernel<double>, dim3(blocks), dim3(threads), 0, 0, (const double*)buf, (long long)(bytes / 8), out);
    hipLaunchKernelGGL(read_kernel<float4>, dim3(blocks), dim3(threads), 0, 0, (const float4*)buf, (long long)(bytes / 16), out);
    hipLaunchKernelGGL(write_kernel<float>, dim3(blocks), dim3(threads), 0, 0, (float*)buf, (long long)(bytes / 4));
    hipLaunchKernelGGL(write_kernel<double>, dim3(blocks), dim3(threads), 0, 0, (double*)buf, (long long)(bytes / 8));
    hipLaunchKernelGGL(write_kernel<float4>, dim3(blocks), dim3(threads), 0, 0, (float4*)buf, (long long)(bytes / 16));
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("bytes read per kernel: %zu (%.1f KB); written: %d B\n", bytes, bytes / 1024.0, blocks * threads * 4);
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
