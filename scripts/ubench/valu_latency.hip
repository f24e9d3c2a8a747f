// Dependent-issue latency of the f64 VALU ops on the contact solve's chain:
// one wave per CU runs N back-to-back dependent ops (chain) or the same count spread over 4
// independent chains (ilp4); shader cycles per op from s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 -o valu_latency valu_latency.hip && ./valu_latency
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int KIND>
__global__ __launch_bounds__(64) void k_chain(double* out, unsigned long long* cyc, double seed) {
  double a = seed + threadIdx.x, b = 1.0000001, c = 1e-9, d = a + 1, e = a + 2, f = a + 3;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < 16; ++i) {
    if (KIND == 0) { REP64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));) }
    if (KIND == 1) { REP64(asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(c));) }
    if (KIND == 2) { REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));) }
    if (KIND == 3) {   // 4 independent fma chains, same op count
      REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\tv_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5"
                              : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b), "v"(c));))
      i += 3;
    }
    if (KIND == 4) { REP64(asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(a) : "v"(c));) }
    if (KIND == 5) {   // compare + 64-bit select chain (the clamp of a normal row): 3 instructions
      REP64(a = a < c ? c : a; asm volatile("" : "+v"(a));)
    }
    if (KIND == 6) { REP64(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(*(float*)&a) : "v"(1.0001f), "v"(1e-9f));) }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + threadIdx.x] = a + d + e + f;
}

template <int KIND>
void run(const char* name, int ops_per_iter, double* out, unsigned long long* cyc) {
  unsigned long long h[256];
  for (int r = 0; r < 3; ++r) k_chain<KIND><<<256, 64>>>(out, cyc, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  std::printf("%-12s %6.2f cycles/op\n", name, (double)m / 256 / (16.0 * ops_per_iter));
}

int main() {
  double* out; unsigned long long* cyc;
  if (hipMalloc(&out, 256 * 64 * 8) != hipSuccess || hipMalloc(&cyc, 256 * 8) != hipSuccess) return 1;
  run<0>("fma_chain", 64, out, cyc);
  run<1>("add_chain", 64, out, cyc);
  run<2>("mul_chain", 64, out, cyc);
  run<3>("fma_ilp4", 64, out, cyc);   // 16 outer iterations of 4*64 ops counted as 4 x (16/4)
  run<4>("max_chain", 64, out, cyc);
  run<5>("cmp_sel", 64 * 3, out, cyc);
  run<6>("fma32_chain", 64, out, cyc);
  (void)hipFree(out); (void)hipFree(cyc);
  return 0;
}
