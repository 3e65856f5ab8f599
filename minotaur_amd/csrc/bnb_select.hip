// Best-first node selection of the batched tree, gfx950.
//
// The reference's bfs search keeps the open nodes in a heap ordered by their
// lower bound (NodeHeap.cpp:24-47) and, when it takes the next candidate,
// prunes those whose bound cannot beat the incumbent (TreeManager::
// getCandidate / shouldPrune_, TreeManager.cpp:162-186, :403-413).  Batched:
// one round takes the B open nodes with the lowest (bound, pool slot) at
// once:
//   bnb_keys   : one thread per pool slot [0, hw): prunes live nodes by the
//                incumbent (TreeManager::shouldPrune_'s rule), writes the
//                order-preserving 64-bit key of the node bound (dead slots:
//                UINT64_MAX) and the slot id, counts live / pruned nodes;
//   radix sort : rocPRIM's stable LSD radix sort of (key, slot) pairs, so
//                equal bounds keep ascending slot order (deterministic);
//   bnb_gather : one wave per selected node copies its box (and, with
//                parent warm starts, its basis) into the round's contiguous
//                batch and marks the slot free.
// Pool layout is the same [cap][n] boxes as the depth-first stack.
#include <rocprim/device/device_radix_sort.hpp>

#include "bnb_internal.h"

namespace mgpu {
namespace {

__device__ __forceinline__ uint64_t order_key(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

__global__ __launch_bounds__(256) void bnb_keys(const double *pnlb, uint8_t *plive, int hw,
                                                double cutoff, double ub, uint64_t *keys,
                                                uint32_t *vals, int32_t *counts) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int live = 0, pruned = 0;
  if (i < hw) {
    uint64_t key = ~0ull;
    if (plive[i]) {
      const double lb = pnlb[i];
      // TreeManager::shouldPrune_ (TreeManager.cpp:403-413), etol_ = 1e-6
      if (lb > cutoff - 1e-6 || fabs(ub - lb) / (fabs(ub) + 1e-6) * 100.0 < 1e-6) {
        plive[i] = 0;
        pruned = 1;
      } else {
        key = order_key(lb);
        live = 1;
      }
    }
    keys[i] = key;
    vals[i] = (uint32_t)i;
  }
  // wave totals, one atomic per wave
  const uint64_t lm = __ballot(live), pm = __ballot(pruned);
  if ((threadIdx.x & 63) == 0) {
    if (lm) atomicAdd(&counts[0], (int)__popcll(lm));
    if (pm) atomicAdd(&counts[1], (int)__popcll(pm));
  }
}

// One wave per selected node: its box and depth (and basis) into the batch.
__global__ __launch_bounds__(256) void bnb_gather(BnbSelIO io) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= io.nb) return;
  const size_t s = io.slots[k];
  const int n = io.n;
  for (int j = lane; j < n; j += 64) {
    io.wlb[(size_t)k * n + j] = io.plb[s * n + j];
    io.wub[(size_t)k * n + j] = io.pub[s * n + j];
  }
  if (io.ws_head != nullptr) {
    const int m = io.m, N = io.N;
    for (int j = lane; j < m; j += 64) io.bws_head[(size_t)k * m + j] = io.ws_head[s * m + j];
    for (int j = lane; j < N; j += 64) {
      io.bws_st[(size_t)k * N + j] = io.ws_st[s * N + j];
      io.bws_d[(size_t)k * N + j] = io.ws_d[s * N + j];
    }
    const size_t mm = (size_t)m * m;
    for (size_t j = lane; j < mm; j += 64) io.bws_binv[k * mm + j] = io.ws_binv[s * mm + j];
  }
  if (io.pk != nullptr) {
    const int kp = io.pk[s];
    if (lane == 0) io.bpk[k] = kp;
    if (lane < kp) io.bppath[(size_t)k * kPathMax + lane] = io.ppath[s * kPathMax + lane];
    if (kp > 0)
      for (int j = lane; j < io.N; j += 64) io.bpst[(size_t)k * io.N + j] = io.pst[s * io.N + j];
  }
  if (lane == 0) {
    io.depth_in[k] = io.pdepth[s];
    io.plive[s] = 0;
  }
}

}  // namespace

hipError_t launch_bnb_keys(const double *pnlb, uint8_t *plive, int hw, double cutoff, double ub,
                           uint64_t *keys, uint32_t *vals, int32_t *counts, hipStream_t stream) {
  if (hw <= 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_keys, dim3((hw + 255) / 256), dim3(256), 0, stream, pnlb, plive, hw,
                     cutoff, ub, keys, vals, counts);
  return hipGetLastError();
}

hipError_t bnb_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *keys_in,
                          uint64_t *keys_out, const uint32_t *vals_in, uint32_t *vals_out,
                          int count, hipStream_t stream) {
  return rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out,
                                   (unsigned int)count, 0, 64, stream);
}

hipError_t launch_bnb_gather(const BnbSelIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_gather, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

}  // namespace mgpu
