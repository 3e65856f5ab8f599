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

}  // namespace mgpu
