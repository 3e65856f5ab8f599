// Wave64 helpers shared by the kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

namespace mgpu {

// Broadcast lane k's value to the whole wave (v_readlane -> SGPR).  The
// source VGPR must have been written by lane k: load broadcast sources with
// the full wave active.
__device__ __forceinline__ int rl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ double rld(double v, int k) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), k);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ uint64_t rlu64(uint64_t v, int k) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(v & 0xffffffffu), k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(v >> 32), k);
  return ((uint64_t)hi << 32) | lo;
}

// Orders this wave's LDS writes before its later LDS reads by other lanes.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Deterministic arg-max: larger value wins, equal values -> lower index.
__device__ __forceinline__ void wave_argmax(double &v, int &idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(idx, o, 64);
    if (v2 > v || (v2 == v && i2 < idx)) {
      v = v2;
      idx = i2;
    }
  }
}

// ---- DPP reductions --------------------------------------------------------
// Cross-lane moves on the VALU (DPP) instead of ds_bpermute (LDS round trip):
// quad_perm xor 1 / xor 2, then row_ror 4 / 8 inside each 16-lane row, then
// the four row results are combined through v_readlane.  The result is wave
// uniform (in SGPRs).  Exchange patterns only, so any associative,
// commutative combine gives the same answer in every lane.
constexpr int kDppXor1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kDppRor4 = 0x124;  // row_ror:4
constexpr int kDppRor8 = 0x128;  // row_ror:8

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i32<CTRL>((int)(b & 0xffffffffLL));
  const int hi = dpp_i32<CTRL>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ void amax_combine(double &v, int &i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

// Arg-max over the wave (larger value wins, equal values -> lower index).
__device__ __forceinline__ void wave_argmax_dpp(double &v, int &idx) {
  amax_combine(v, idx, dpp_f64<kDppXor1>(v), dpp_i32<kDppXor1>(idx));
  amax_combine(v, idx, dpp_f64<kDppXor2>(v), dpp_i32<kDppXor2>(idx));
  amax_combine(v, idx, dpp_f64<kDppRor4>(v), dpp_i32<kDppRor4>(idx));
  amax_combine(v, idx, dpp_f64<kDppRor8>(v), dpp_i32<kDppRor8>(idx));
  double r = rld(v, 0);
  int ri = rl(idx, 0);
  amax_combine(r, ri, rld(v, 16), rl(idx, 16));
  amax_combine(r, ri, rld(v, 32), rl(idx, 32));
  amax_combine(r, ri, rld(v, 48), rl(idx, 48));
  v = r;
  idx = ri;
}

__device__ __forceinline__ double wave_max_dpp(double v) {
  v = fmax(v, dpp_f64<kDppXor1>(v));
  v = fmax(v, dpp_f64<kDppXor2>(v));
  v = fmax(v, dpp_f64<kDppRor4>(v));
  v = fmax(v, dpp_f64<kDppRor8>(v));
  return fmax(fmax(rld(v, 0), rld(v, 16)), fmax(rld(v, 32), rld(v, 48)));
}

// Arg-max where the index is the lane itself: larger value wins, equal
// values -> lowest lane (wave_argmax_dpp(v, lane) for non-NaN v, with a
// plain DPP max and one ballot instead of carrying the index through every
// step).  v becomes the wave maximum.
__device__ __forceinline__ int wave_argmax_lane(double &v) {
  const double mx = wave_max_dpp(v);
  const uint64_t hit = __ballot(v == mx);
  v = mx;
  return (int)__builtin_ctzll(hit);
}

__device__ __forceinline__ int wave_min_i32_dpp(int v) {
  v = min(v, dpp_i32<kDppXor1>(v));
  v = min(v, dpp_i32<kDppXor2>(v));
  v = min(v, dpp_i32<kDppRor4>(v));
  v = min(v, dpp_i32<kDppRor8>(v));
  return min(min(rl(v, 0), rl(v, 16)), min(rl(v, 32), rl(v, 48)));
}

// wave_argmax_dpp for a general index (e.g. a column slot*64 + lane): a DPP
// max, then the holder's index (one ballot; an int min only on ties).
__device__ __forceinline__ void wave_argmax_idx(double &v, int &idx) {
  const double mx = wave_max_dpp(v);
  const uint64_t hit = __ballot(v == mx);
  idx = __popcll(hit) == 1 ? rl(idx, __builtin_ctzll(hit))
                           : wave_min_i32_dpp(v == mx ? idx : INT_MAX);
  v = mx;
}

constexpr int kDppHalfMirror = 0x141;  // row_half_mirror: lane i <-> i ^ 7 in 8 lanes
constexpr int kDppMirror = 0x140;      // row_mirror: lane i <-> i ^ 15 in 16 lanes

// Deterministic wave sum with symmetric exchanges only: pairs (i, i^1),
// (i, i^2), the half-row mirror, the row mirror, then the four rows as
// (r0 + r1) + (r2 + r3).  Each step adds a lane and its partner (the same
// two values in both), so the association is fixed: oracle/lp_dual.c
// eta_dot restates it.  Wave uniform result.
__device__ __forceinline__ double wave_sum_sym(double v) {
  v = v + dpp_f64<kDppXor1>(v);
  v = v + dpp_f64<kDppXor2>(v);
  v = v + dpp_f64<kDppHalfMirror>(v);
  v = v + dpp_f64<kDppMirror>(v);
  return (rld(v, 0) + rld(v, 16)) + (rld(v, 32) + rld(v, 48));
}

__device__ __forceinline__ double wave_min_dpp(double v) {
  v = fmin(v, dpp_f64<kDppXor1>(v));
  v = fmin(v, dpp_f64<kDppXor2>(v));
  v = fmin(v, dpp_f64<kDppRor4>(v));
  v = fmin(v, dpp_f64<kDppRor8>(v));
  return fmin(fmin(rld(v, 0), rld(v, 16)), fmin(rld(v, 32), rld(v, 48)));
}

}  // namespace mgpu
