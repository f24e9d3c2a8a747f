// Does instruction fetch show up in FETCH_SIZE?  Three kernels that touch no
// data memory, launched with 256 one-wave blocks (one per CU, as the 4096-env step): an empty one,
// one with ~4 KB and one with ~24 KB of straight-line VALU code.  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./ifetch_probe
// and compare FETCH_SIZE per dispatch: a code-size-proportional difference (x the XCDs) is
// instruction fetch from beyond the L2.
//   hipcc --offload-arch=gfx950 -O3 -o ifetch_probe ifetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k_empty(float* out) {
  if (threadIdx.x == 1000) out[0] = 1.0f;
}

template <int N>
__global__ __launch_bounds__(64) void k_code(float* out) {
  float a = threadIdx.x * 1.0001f, b = 0.5f;
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b));   // 8-byte VOP3
  if (a == -1.0f) out[0] = a;
}

int main() {
  float* out = nullptr;
  if (hipMalloc(&out, 64) != hipSuccess) return 1;
  for (int r = 0; r < 20; ++r) {
    k_empty<<<256, 64>>>(out);
    k_code<512><<<256, 64>>>(out);    // ~4 KB of code
    k_code<3072><<<256, 64>>>(out);   // ~24 KB of code
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("done\n");
  (void)hipFree(out);
  return 0;
}
