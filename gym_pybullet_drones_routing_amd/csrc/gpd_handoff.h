// gpd_handoff.h — device side of the config-5 learner hand-off.
//
// The caller being replaced is the reference's SB3 stepping loop (examples/learn.py:52-94):
// one process steps its vectorised envs and hands obs / reward / done / terminal_observation to
// PPO.  Here every rank steps its env shard into ONE output pack (include/gpd.h
// gpd_pack_layout) and a single collective moves each rank's RECORD (obs | reward | terminated |
// truncated | terminal_state) to the learner.  Two kernels bracket that collective:
//
//   handoff_pack_kernel    before it, on every rank: the 12 state columns of the terminal rows of
//                          the envs that finished this step -> the record's terminal_state block.
//                          The reference never clears the action buffer on reset (BaseRLAviary
//                          has no reset override), so a finished env's terminal row
//                          and its auto-reset row share the 15 history columns: only the state
//                          columns need to travel.
//   handoff_unpack_kernel  after it, on the receiving ranks: the G gathered records -> the global
//                          batch obs [G*E][D][W], reward [G*E], terminated / truncated [G*E] and
//                          terminal rows [G*E][D][W] (state columns + the reset row's history for
//                          finished envs, zero elsewhere), in rank order.
//
// Both are byte movers: HBM-bound, coalesced, float4 wherever the row width allows.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gpd {

constexpr int kHandoffStateCols = 12;   // KIN obs: pos, rpy, vel, ang_v (BaseRLAviary.py:313-316)

struct HandoffView {
  long long obs, reward, term, trunc, tstate, tobs;   // byte offsets inside one rank's pack
  long long stride;                                   // bytes between consecutive ranks' records
  int E, D, W, G;
};

// one thread per terminal-state float: E*D*12 threads
__global__ void __launch_bounds__(256) handoff_pack_kernel(uint8_t* __restrict__ pack, HandoffView L) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned n = (unsigned)L.E * (unsigned)L.D * kHandoffStateCols;
  if (t >= n) return;
  const unsigned row = t / kHandoffStateCols, c = t - row * kHandoffStateCols;
  const unsigned e = row / (unsigned)L.D;
  if (!(pack[L.term + e] | pack[L.trunc + e])) return;   // rows of running envs are never read
  const float* tobs = (const float*)(pack + L.tobs);
  float* ts = (float*)(pack + L.tstate);
  ts[t] = tobs[(size_t)row * L.W + c];
}

template <int VEC>
struct HVec;
template <>
struct HVec<1> {
  typedef float T;
  __device__ static T zero() { return 0.0f; }
};
template <>
struct HVec<4> {
  typedef float4 T;
  __device__ static T zero() { return make_float4(0.0f, 0.0f, 0.0f, 0.0f); }
};

// Threads [0, G*E*D*W/VEC) move one obs vector each (and its terminal-row vector); threads
// [0, G*E) also move one env's reward and flags.  VEC = 4 needs W % 4 == 0 (then a vector never
// straddles two rows or the state / history boundary at column 12) and 16-B aligned records.
template <int VEC, bool TOBS>
__global__ void __launch_bounds__(256) handoff_unpack_kernel(const uint8_t* __restrict__ in, HandoffView L,
                                                             float* __restrict__ obs, float* __restrict__ reward,
                                                             uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                             float* __restrict__ tobs) {
  typedef typename HVec<VEC>::T V;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned wv = (unsigned)L.W / VEC;                       // vectors per row
  const unsigned nv = (unsigned)L.E * (unsigned)L.D * wv;        // vectors per rank
  if (t < nv * (unsigned)L.G) {
    const unsigned g = t / nv, v = t - g * nv;
    const uint8_t* rec = in + (size_t)g * (size_t)L.stride;
    const V x = ((const V*)(rec + L.obs))[v];
    ((V*)obs)[t] = x;
    if (TOBS) {
      const unsigned row = v / wv, col = (v - row * wv) * VEC;
      const unsigned e = row / (unsigned)L.D;
      V y = HVec<VEC>::zero();
      if (rec[L.term + e] | rec[L.trunc + e]) {
        y = col < (unsigned)kHandoffStateCols
                ? ((const V*)(rec + L.tstate))[(row * kHandoffStateCols + col) / VEC]
                : x;
      }
      ((V*)tobs)[t] = y;
    }
  }
  if (t < (unsigned)L.E * (unsigned)L.G) {
    const unsigned g = t / (unsigned)L.E, e = t - g * (unsigned)L.E;
    const uint8_t* rec = in + (size_t)g * (size_t)L.stride;
    reward[t] = ((const float*)(rec + L.reward))[e];
    term[t] = rec[L.term + e];
    trunc[t] = rec[L.trunc + e];
  }
}

}  // namespace gpd
