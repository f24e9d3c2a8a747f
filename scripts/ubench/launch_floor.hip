// Launch-boundary cost on one MI355X: back-to-back DEPENDENT launches of (a) an empty kernel,
// (b) an empty kernel with a 512-byte kernarg block, (c) a kernel whose 256 one-wave blocks
// store 3 MB of plain (write-back) data, (d) the same stores write-through (sc1).  Each case is
// timed with HIP events over N launches issued eagerly and as one hipGraph.  Prints us/launch.
//   hipcc --offload-arch=gfx950 -O3 -o launch_floor launch_floor.hip && ./launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Big { long long v[64]; };

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }
__global__ void k_bigarg(Big b, int* p) { if (p && threadIdx.x == 1000) p[0] = (int)b.v[63]; }
__global__ void k_store(float4* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = i; j < n; j += gridDim.x * blockDim.x) dst[j] = make_float4(1.f, 2.f, 3.f, (float)j);
}
__global__ void k_store_wt(float4* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, 0, n * 16, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  for (int j = i; j < n; j += gridDim.x * blockDim.x) {
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)j);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, j * 16, 0, 16);
  }
}

template <typename F>
int timeit(const char* name, F launch, hipStream_t st, int N) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 50; ++i) launch();
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  for (int i = 0; i < N; ++i) launch();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  // the same N launches as one graph
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < N; ++i) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float msg; CK(hipEventElapsedTime(&msg, a, b));
  printf("%-44s eager %6.2f us/launch   graph %6.2f us/launch\n", name, 1000 * ms / N, 1000 * msg / N);
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t st; CK(hipStreamCreate(&st));
  const int n = 3 << 20 >> 4;   // 3 MiB of float4
  float4* buf; CK(hipMalloc(&buf, (size_t)n * 16));
  int* flag; CK(hipMalloc(&flag, 4));
  Big big{}; big.v[63] = 7;
  const int N = 2000;
  if (timeit("empty, 1 block", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, flag); }, st, N)) return 1;
  if (timeit("empty, 256 blocks", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(64), 0, st, flag); }, st, N)) return 1;
  if (timeit("empty, 256 blocks, 512-B kernarg", [&] { hipLaunchKernelGGL(k_bigarg, dim3(256), dim3(64), 0, st, big, flag); }, st, N)) return 1;
  if (timeit("3 MiB plain stores, 256 blocks", [&] { hipLaunchKernelGGL(k_store, dim3(256), dim3(64), 0, st, buf, n); }, st, N)) return 1;
  if (timeit("3 MiB write-through stores, 256 blocks", [&] { hipLaunchKernelGGL(k_store_wt, dim3(256), dim3(64), 0, st, buf, n); }, st, N)) return 1;
  if (timeit("3 MiB plain stores, 1024 blocks", [&] { hipLaunchKernelGGL(k_store, dim3(1024), dim3(256), 0, st, buf, n); }, st, N)) return 1;
  CK(hipFree(buf)); CK(hipFree(flag));
  printf("ALLDONE\n");
  return 0;
}
