// Node migration between ranks of the node-sharded tree (SURVEY §8 e),
// gfx950.  MpiBranchAndBound::LoadBalance_ (src/base/MpiBranchAndBound.cpp:
// 78-195) serialises each node it hands to another rank (Serializer.cpp:
// 26-112: bound changes, lower bound, depth) and sends it with one MPI_Send
// per node.  Here the nodes a rank gives away are packed on the device into
// one f64 row each,
//     row t = [ lb (n) | ub (n) | node bound | depth ]      (2n + 2 doubles)
// and, in the tree's warm mode 2, the node's warm start behind it
//     [ k | path (kPathMax) | statuses packed 16 per double (2 bits each) ]
// (k 0 = the root basis; path entries past k and the statuses of k = 0
// are 0), so a migrated node keeps its parent's basis: every rank solved
// the same root LP, whose basis the path is relative to.  The exchange is
// one collective over device buffers (RCCL over xGMI) and no box crosses
// PCIe.  Three kernels, one wave per node:
//   bnb_pack   : pool slot slots[t] -> row t (a best-first slot is freed);
//   bnb_unpack : row t -> pool slot slots[t], with the slot's per-node state
//                reset as a migrated node needs it (live flag, no parent
//                branching data, root warm start);
//   bnb_move   : generic per-slot row move src[t] -> dst[t] through a scratch
//                copy (the depth-first stack closes the gaps the exported
//                nodes leave in its top region).
#include "bnb_internal.h"

namespace mgpu {
namespace {

__global__ __launch_bounds__(256) void bnb_pack(MigratePack io) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= io.k) return;
  const int n = io.n;
  const size_t s = (size_t)io.slots[t];
  double *row = io.buf + (size_t)t * io.W;
  for (int j = lane; j < n; j += 64) {
    row[j] = io.plb[s * n + j];
    row[n + j] = io.pub[s * n + j];
  }
  if (io.ppk != nullptr) {   // warm mode 2: the node's basis travels with it
    const int kp = io.ppk[s], N = io.N;
    double *w = row + 2 * n + 2;
    if (lane == 0) w[0] = (double)kp;
    if (lane < kPathMax) w[1 + lane] = lane < kp ? (double)io.ppath[s * kPathMax + lane] : 0.0;
    const int nq = (N + 15) / 16;
    for (int q = lane; q < nq; q += 64) {
      double v = 0.0;
      if (kp > 0) {
        uint32_t bits = 0;
        for (int i = 0; i < 16 && q * 16 + i < N; ++i)
          bits |= (uint32_t)(io.ppst[s * N + q * 16 + i] & 3) << (2 * i);
        v = (double)bits;
      }
      w[1 + kPathMax + q] = v;
    }
  }
  if (lane == 0) {
    row[2 * n] = io.pnlb[s];
    row[2 * n + 1] = (double)io.pdepth[s];
    if (io.plive) io.plive[s] = 0;   // best-first pool: the slot becomes free
  }
}

__global__ __launch_bounds__(256) void bnb_unpack(MigrateIO io) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= io.k) return;
  const int n = io.n;
  const size_t s = (size_t)io.slots[t];
  const double *row = io.buf + (size_t)t * io.W;
  for (int j = lane; j < n; j += 64) {
    io.plb[s * n + j] = row[j];
    io.pub[s * n + j] = row[n + j];
  }
  if (io.ws_head != nullptr) {  // parent warm starts: the root basis
    const int m = io.m, N = io.N;
    for (int j = lane; j < m; j += 64) io.ws_head[s * m + j] = io.r_head[j];
    for (int j = lane; j < N; j += 64) {
      io.ws_st[s * N + j] = io.r_st[j];
      io.ws_d[s * N + j] = io.r_d[j];
    }
    const size_t mm = (size_t)m * m;
    for (size_t j = lane; j < mm; j += 64) io.ws_binv[s * mm + j] = io.r_binv[j];
  }
  if (lane == 0) {
    io.pnlb[s] = row[2 * n];
    io.pdepth[s] = (int32_t)row[2 * n + 1];
    if (io.plive) io.plive[s] = 1;
    if (io.ppvar) io.ppvar[s] = -1;   // no parent branching data
  }
  if (io.ppk) {   // warm mode 2: the basis the row carries (k 0: the root's)
    const int N = io.N;
    const double *w = row + 2 * n + 2;
    const int kp = (int)w[0];
    if (lane == 0) io.ppk[s] = kp;
    if (lane < kPathMax) io.ppath[s * kPathMax + lane] = (uint32_t)w[1 + lane];
    if (kp > 0) {
      for (int j = lane; j < N; j += 64) {
        const uint32_t bits = (uint32_t)w[1 + kPathMax + j / 16];
        io.ppst[s * N + j] = (int8_t)((bits >> (2 * (j % 16))) & 3u);
      }
    }
  }
}

__global__ __launch_bounds__(256) void bnb_move(const unsigned char *src, unsigned char *dst,
                                                size_t row_bytes, const int32_t *from,
                                                const int32_t *to, int k) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= k) return;
  const size_t a = from ? (size_t)from[t] : (size_t)t;
  const size_t b = to ? (size_t)to[t] : (size_t)t;
  const unsigned char *p = src + a * row_bytes;
  unsigned char *q = dst + b * row_bytes;
  if ((row_bytes & 3) == 0) {
    const uint32_t *p4 = reinterpret_cast<const uint32_t *>(p);
    uint32_t *q4 = reinterpret_cast<uint32_t *>(q);
    for (size_t j = lane; j < row_bytes / 4; j += 64) q4[j] = p4[j];
  } else {
    for (size_t j = lane; j < row_bytes; j += 64) q[j] = p[j];
  }
}

}  // namespace

hipError_t launch_bnb_pack(const MigratePack &io, hipStream_t stream) {
  if (io.k <= 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_pack, dim3((io.k + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_bnb_unpack(const MigrateIO &io, hipStream_t stream) {
  if (io.k <= 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_unpack, dim3((io.k + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_bnb_move_rows(unsigned char *rows, unsigned char *tmp, size_t row_bytes,
                                const int32_t *from, const int32_t *to, int k,
                                hipStream_t stream) {
  if (k <= 0 || row_bytes == 0) return hipSuccess;
  const dim3 grid((k + 3) / 4), blk(256);
  hipLaunchKernelGGL(bnb_move, grid, blk, 0, stream, rows, tmp, row_bytes, from, nullptr, k);
  hipLaunchKernelGGL(bnb_move, grid, blk, 0, stream, tmp, rows, row_bytes, nullptr, to, k);
  return hipGetLastError();
}

hipError_t launch_bnb_gather_rows(const unsigned char *src, unsigned char *dst, size_t row_bytes,
                                  const int32_t *from, int k, hipStream_t stream) {
  if (k <= 0 || row_bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_move, dim3((k + 3) / 4), dim3(256), 0, stream, src, dst, row_bytes,
                     from, nullptr, k);
  return hipGetLastError();
}

}  // namespace mgpu
