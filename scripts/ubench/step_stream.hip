// The large-N step kernel's memory traffic without its physics:
// per 64-drone tile (f64, RPM, the Gym observation layout) read 13 state components (tiled SoA),
// the action, the {step_counter, head} pair and 14 action-history ring slots (LDS-DMA into the
// observation tile), write 16 state components, the ring append, the 64 observation rows of 288 B
// (coalesced copy-out of the LDS tile), reward and done flags and the counters: 817 B per drone,
// as counted by PMC for the real kernel.  Launch forms:
//   tile : one 64-lane block per tile (the shipped step_kernel's geometry), LDS padded to B blocks/CU;
//   pers : persistent blocks (B per CU), each walking tiles t, t+G, ...; the next tile's state,
//          action, counters and ring DMA (second LDS buffer) are issued before this tile's stores.
// Reports GB/s of the 817 B/drone moved and the time per 1M-drone launch.
//   hipcc --offload-arch=gfx950 -O3 -o step_stream step_stream.hip && ./step_stream
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) void* gbl_ptr;
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int L = 15, NC = 3 + L, PAD = 65, TILE_F4 = NC * PAD;   // obs tile: 18 float4 columns
constexpr int SC = 20;                                           // state components per drone

struct Bufs {
  double* state;        // [T][20][64]
  float* ring;          // [T][15][64*4]
  const float* act;     // [N][4]
  int2* ctr;            // [N]
  float* obs;           // [N][72]
  float* rew;           // [N]
  unsigned char* te;    // [N]
  unsigned char* tr;    // [N]
  int T;
};

template <bool NT>
__device__ __forceinline__ void st16(float4* p, float4 v) {
  if (NT) {
    __builtin_nontemporal_store(v.x, &p->x); __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z); __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}

struct TileIn {
  double s[13];
  float4 a;
  int2 c;
};

__device__ __forceinline__ void load_tile(const Bufs& b, int t, int lane, TileIn& in, float4* tile) {
  const double* st = b.state + (long long)t * SC * 64 + lane;
#pragma unroll
  for (int k = 0; k < 13; ++k) in.s[k] = st[k * 64];
  const long long n = (long long)t * 64 + lane;
  in.a = reinterpret_cast<const float4*>(b.act)[n];
  in.c = b.ctr[n];
  // ring slots head+1 .. head+14 -> tile columns 3.. (head is uniform in lockstep runs)
  const int head = __builtin_amdgcn_readfirstlane(in.c.y);
  const float* rb = b.ring + (long long)t * L * 256 + lane * 4;
  int slot = head + 1 == L ? 0 : head + 1;
  for (int m = 0; m < L - 1; ++m) {
    __builtin_amdgcn_global_load_lds((gbl_ptr)(rb + slot * 256), (lds_ptr)(tile + (3 + m) * PAD), 16, 0, 0);
    slot = slot + 1 == L ? 0 : slot + 1;
  }
}

template <bool NT>
__device__ __forceinline__ void store_tile(const Bufs& b, int t, int lane, const TileIn& in, float4* tile) {
  const long long n = (long long)t * 64 + lane;
  double* st = b.state + (long long)t * SC * 64 + lane;
  double v[16];
#pragma unroll
  for (int k = 0; k < 13; ++k) v[k] = in.s[k] * 1.0000001;                 // stand-in for the physics
  v[13] = v[10]; v[14] = v[11]; v[15] = v[12];
#pragma unroll
  for (int k = 0; k < 16; ++k) st[k * 64] = v[k];
  const int head = in.c.y;
  reinterpret_cast<float4*>(b.ring + (long long)t * L * 256 + head * 256)[lane] = in.a;
  tile[0 * PAD + lane] = make_float4((float)v[0], (float)v[1], (float)v[2], 0.f);
  tile[1 * PAD + lane] = make_float4(0.f, 0.f, (float)v[7], (float)v[8]);
  tile[2 * PAD + lane] = make_float4((float)v[9], (float)v[13], (float)v[14], (float)v[15]);
  tile[(NC - 1) * PAD + lane] = in.a;
  // one-wave block: the wave's LDS operations are in order; only the compiler is fenced (a
  // __syncthreads() release would wait for every vector-memory op, the prefetch included)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  float4* dst = reinterpret_cast<float4*>(b.obs) + (long long)t * 64 * NC;
#pragma unroll 6
  for (int u = 0; u < NC; ++u) {                     // 64 rows x 18 float4, row-major, coalesced
    const int g = u * 64 + lane, row = g / NC, col = g - row * NC;
    st16<NT>(dst + g, tile[col * PAD + row]);
  }
  b.rew[n] = (float)v[2];
  b.te[n] = 0;
  b.tr[n] = 0;
  b.ctr[n] = make_int2(in.c.x + 8, head + 1 == L ? 0 : head + 1);
}

template <bool NT, int PADB>
__global__ __launch_bounds__(64) void k_tile(Bufs b) {
  __shared__ float4 tile[TILE_F4 + PADB];
  const int lane = threadIdx.x, t = blockIdx.x;
  TileIn in;
  load_tile(b, t, lane, in, tile);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring DMA has landed
  store_tile<NT>(b, t, lane, in, tile);
}

// two register sets and two LDS tiles: tile t's stores go out while tile t+G's loads and ring
// DMA (29 vector-memory ops) are in flight; vmcnt(29) = everything older than the prefetch landed
template <bool NT>
__global__ __launch_bounds__(64) void k_pers(Bufs b) {
  __shared__ float4 tile0[TILE_F4], tile1[TILE_F4];
  const int lane = threadIdx.x, G = gridDim.x;
  int t = blockIdx.x;
  if (t >= b.T) return;
  TileIn A, B;
  load_tile(b, t, lane, A, tile0);
  for (; t < b.T; t += 2 * G) {
    const int t1 = t + G, t2 = t + 2 * G;
    if (t1 < b.T) {
      load_tile(b, t1, lane, B, tile1);
      asm volatile("s_waitcnt vmcnt(29)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    store_tile<NT>(b, t, lane, A, tile0);
    if (t1 >= b.T) break;
    if (t2 < b.T) {
      load_tile(b, t2, lane, A, tile0);
      asm volatile("s_waitcnt vmcnt(29)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    store_tile<NT>(b, t1, lane, B, tile1);
  }
}

#define CHECK(x) do { if ((x) != hipSuccess) { std::printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

template <typename F>
double time_it(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps * 1e3;   // us
}

int main() {
  const long long N = 1 << 22;          // 4M drones: far past the 256 MB Infinity Cache
  const int T = (int)(N / 64);
  Bufs b;
  CHECK(hipMalloc(&b.state, N * SC * 8));
  CHECK(hipMalloc(&b.ring, N * L * 16));
  float* act;
  CHECK(hipMalloc(&act, N * 16));
  b.act = act;
  CHECK(hipMalloc(&b.ctr, N * 8));
  CHECK(hipMalloc(&b.obs, N * 288));
  CHECK(hipMalloc(&b.rew, N * 4));
  CHECK(hipMalloc(&b.te, N));
  CHECK(hipMalloc(&b.tr, N));
  CHECK(hipMemset(b.state, 0, N * SC * 8));
  CHECK(hipMemset(b.ring, 0, N * L * 16));
  CHECK(hipMemset(act, 0, N * 16));
  CHECK(hipMemset(b.ctr, 0, N * 8));
  b.T = T;
  const double bytes = 817.0 * N;
  auto rep = [&](const char* name, double us) {
    std::printf("%-34s %8.1f us  %6.0f GB/s  (%.1f us per 1M drones)\n", name, us, bytes / (us * 1e-6) / 1e9,
                us * (1 << 20) / N);
  };
  // LDS per block: 18.7 KB tile (8 blocks/CU, the shipped kernel); padded to 6 / 4 / 2 blocks/CU
  rep("tile  8/CU plain", time_it([&] { k_tile<false, 0><<<T, 64>>>(b); }, 10));
  rep("tile  8/CU nt", time_it([&] { k_tile<true, 0><<<T, 64>>>(b); }, 10));
  rep("tile  6/CU plain", time_it([&] { k_tile<false, 500><<<T, 64>>>(b); }, 10));
  rep("tile  4/CU plain", time_it([&] { k_tile<false, 1400><<<T, 64>>>(b); }, 10));
  rep("tile  4/CU nt", time_it([&] { k_tile<true, 1400><<<T, 64>>>(b); }, 10));
  rep("tile  2/CU plain", time_it([&] { k_tile<false, 3700><<<T, 64>>>(b); }, 10));
  for (int bpc : {1, 2, 3, 4}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "pers  %d/CU plain", bpc);
    rep(nm, time_it([&] { k_pers<false><<<256 * bpc, 64>>>(b); }, 10));
    std::snprintf(nm, sizeof nm, "pers  %d/CU nt", bpc);
    rep(nm, time_it([&] { k_pers<true><<<256 * bpc, 64>>>(b); }, 10));
  }
  return 0;
}
