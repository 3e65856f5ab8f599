// Batched branch-and-bound tree step, gfx950.
//
// The node pool lives in HBM as a stack of boxes ([cap][n] lb / ub, the
// parent's relaxation value as the node's lower bound).  One round pops the
// top B boxes (a contiguous slice: no gather), runs K1 FBBT -> K3 LP ->
// decide on them (mgpu_bnb_round, bnb.cpp) and then, here:
//   bnb_scan_block  : per 256-node block, the exclusive prefix of "branched"
//                     flags, the block's incumbent candidate (min cand_obj,
//                     lowest index on ties) and decision counts;
//   bnb_scan_top    : one workgroup scans the block totals;
//   bnb_children    : one wave per branched node writes its two children
//                     (IntVarHandler::getBranches, IntVarHandler.cpp:125-175:
//                     down ub = floor(x_j), up lb = ceil(x_j)) at
//                     base + prefix (prefix counts 2 children per branched
//                     node, 1 per node reliability branching modified), the
//                     preferred direction on top of the stack so it is
//                     popped first.
// Children inherit the node's FBBT-tightened box, as the reference keeps a
// node's presolve mods (PCBProcessor::presolveNode_, :134-175).
#include "bnb_internal.h"
#include "wave.h"

#include <climits>

namespace mgpu {
namespace {

constexpr int kScanBlock = 256;

__global__ __launch_bounds__(kScanBlock) void bnb_scan_block(BnbIO io) {
  __shared__ int s_pos[kScanBlock];
  __shared__ double s_min[kScanBlock];
  __shared__ int s_idx[kScanBlock];
  __shared__ int s_cnt[kScanBlock][8];   // decisions 0..4, LPs, pivots, K3P pivots
  const int t = threadIdx.x;
  const int i = blockIdx.x * kScanBlock + t;
  const bool live = i < io.nb;
  const int dec = live ? io.decision[i] : -1;
  // stack mode: depth before children overwrite the slots (best-first: gathered)
  if (live && io.slots == nullptr) io.depth_in[i] = io.pdepth[io.base + i];
  // children: two per branched node, one per node modified by the brancher
  // (reliability branching's one-sided bound change, decision 5)
  const int f = dec == 0 ? 2 : dec == 5 ? 1 : 0;
  s_pos[t] = f;
  s_min[t] = live ? io.cand_obj[i] : INFINITY;
  s_idx[t] = live ? i : INT_MAX;
  for (int k = 0; k < 5; ++k) s_cnt[t][k] = (dec == k || (k == 0 && dec == 5)) ? 1 : 0;
  const bool lp = live && io.status[i] != 12;
  s_cnt[t][5] = lp ? 1 : 0;
  s_cnt[t][6] = lp ? io.iters[i] : 0;
  // (slot 7 unused: the pivots the product-form kernel ran itself come from
  // its own counter, BnbIO::pfi_piv)
  s_cnt[t][7] = 0;
  __syncthreads();
  // Hillis-Steele inclusive scan of the flags
  for (int o = 1; o < kScanBlock; o <<= 1) {
    const int v = t >= o ? s_pos[t - o] : 0;
    __syncthreads();
    s_pos[t] += v;
    __syncthreads();
  }
  if (live) io.pos[i] = s_pos[t] - f;  // exclusive, within the block
  // min / argmin of the incumbent candidates and decision counts
  for (int o = kScanBlock / 2; o > 0; o >>= 1) {
    if (t < o) {
      const double a = s_min[t], b = s_min[t + o];
      const int ia = s_idx[t], ib = s_idx[t + o];
      if (b < a || (b == a && ib < ia)) {
        s_min[t] = b;
        s_idx[t] = ib;
      }
      for (int k = 0; k < 8; ++k) s_cnt[t][k] += s_cnt[t + o][k];
    }
    __syncthreads();
  }
  if (t == 0) {
    io.bsum[blockIdx.x] = s_pos[kScanBlock - 1];
    io.bmin[blockIdx.x] = s_min[0];
    io.bidx[blockIdx.x] = s_idx[0];
    for (int k = 0; k < 8; ++k) io.bcnt[blockIdx.x * 8 + k] = s_cnt[0][k];
  }
}

// One workgroup: exclusive scan of the block sums (any number of blocks,
// 1024 at a time), global min / argmin, decision totals -> io.out.
__global__ __launch_bounds__(1024) void bnb_scan_top(BnbIO io, int nblk) {
  __shared__ int s[1024];
  __shared__ double s_min[1024];
  __shared__ int s_idx[1024];
  __shared__ int s_carry;
  const int t = threadIdx.x;
  if (t == 0) s_carry = 0;
  double my_min = INFINITY;
  int my_idx = INT_MAX;
  long cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int c0 = 0; c0 < nblk; c0 += 1024) {
    const int b = c0 + t;
    const int v = b < nblk ? io.bsum[b] : 0;
    if (b < nblk) {
      const double m = io.bmin[b];
      const int ix = io.bidx[b];
      if (m < my_min || (m == my_min && ix < my_idx)) {
        my_min = m;
        my_idx = ix;
      }
      for (int k = 0; k < 8; ++k) cnt[k] += io.bcnt[b * 8 + k];
    }
    s[t] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int u = t >= o ? s[t - o] : 0;
      __syncthreads();
      s[t] += u;
      __syncthreads();
    }
    if (b < nblk) io.boff[b] = s_carry + s[t] - v;
    __syncthreads();
    if (t == 1023) s_carry += s[1023];
    __syncthreads();
  }
  s_min[t] = my_min;
  s_idx[t] = my_idx;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (t < o) {
      const double a = s_min[t], b = s_min[t + o];
      const int ia = s_idx[t], ib = s_idx[t + o];
      if (b < a || (b == a && ib < ia)) {
        s_min[t] = b;
        s_idx[t] = ib;
      }
    }
    __syncthreads();
  }
  // decision totals: lane-0 atomics into a zeroed slot
  for (int k = 0; k < 5; ++k)
    if (cnt[k]) atomicAdd(reinterpret_cast<unsigned long long *>(&io.out->ndec[k]),
                          (unsigned long long)cnt[k]);
  if (cnt[5]) atomicAdd(reinterpret_cast<unsigned long long *>(&io.out->lps),
                        (unsigned long long)cnt[5]);
  if (cnt[6]) atomicAdd(reinterpret_cast<unsigned long long *>(&io.out->pivots),
                        (unsigned long long)cnt[6]);
  // the product-form kernel's own pivots (K3P counts them: a basis warm
  // start's column replacements are not pivots, a reinversion keeps going,
  // an overflowing LP's later pivots ran in the dense continuation)
  if (t == 0 && io.pfi_piv != nullptr)
    io.out->pfi_pivots = (long long)*io.pfi_piv;
  if (t == 0) {
    io.out->nchild = s_carry;
    io.out->best = s_min[0];
    io.out->best_idx = s_idx[0] == INT_MAX ? -1 : s_idx[0];
  }
}

// One wave per node: copy the node's (FBBT-tightened) box into its two
// children, apply the branching bound, set the children's lower bound (and,
// with parent warm starts, give both children the node's optimal basis).
__global__ __launch_bounds__(256) void bnb_children(BnbIO io, int n) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int dec = i < io.nb ? io.decision[i] : -1;
  if (dec != 0 && dec != 5) return;
  const long p = io.boff[i / kScanBlock] + io.pos[i];  // first child index of the node
  const int j = io.bvar[i];
  const double v = io.bval[i];
  const bool up_first = io.bup[i] != 0;
  // free list F of best-first mode
  auto slot_of = [&](long c) -> size_t {
    if (io.child_slots != nullptr) return (size_t)io.child_slots[c];
    if (c < io.nb) return io.slots[c];
    const long h = c - io.nb, holes = io.hw - io.live;
    if (h < holes) return io.slots[io.live + h];
    return (size_t)(io.hw + (h - holes));
  };
  const double *sl = io.wlb + (size_t)i * n, *su = io.wub + (size_t)i * n;
  if (dec == 5) {
    // the node itself again with the brancher's bound change (up: lb = ceil,
    // else ub = floor), same depth, its LP value as bound, no pseudocost
    // observation when it is solved again (updateAfterSolve only runs on a
    // node's first solve, PCBProcessor.cpp:245-248)
    const size_t c = io.slots == nullptr ? (size_t)io.base + p : slot_of(p);
    double *cl = io.plb + c * n, *cu = io.pub + c * n;
    for (int k = lane; k < n; k += 64) {
      const double l = sl[k], u = su[k];
      cl[k] = (k == j && up_first) ? ceil(v) : l;
      cu[k] = (k == j && !up_first) ? floor(v) : u;
    }
    if (io.ws_head != nullptr) {
      // the engine's basis after the node's strong branching (PCBProcessor
      // resolves the modified node right away, PCBProcessor.cpp:295-310)
      const bool mo = io.mo_head != nullptr;
      const int32_t *sh = mo ? io.mo_head : io.wo_head;
      const int8_t *ss = mo ? io.mo_st : io.wo_st;
      const double *sd = mo ? io.mo_d : io.wo_d, *sb = mo ? io.mo_binv : io.wo_binv;
      const int m = io.m, N = io.N;
      const size_t mm = (size_t)m * m;
      for (int k = lane; k < m; k += 64) io.ws_head[c * m + k] = sh[(size_t)i * m + k];
      for (int k = lane; k < N; k += 64) {
        io.ws_st[c * N + k] = ss[(size_t)i * N + k];
        io.ws_d[c * N + k] = sd[(size_t)i * N + k];
      }
      for (size_t k = lane; k < mm; k += 64) io.ws_binv[c * mm + k] = sb[(size_t)i * mm + k];
    }
    if (lane == 0) {
      io.pnlb[c] = io.obj[i];
      io.pdepth[c] = io.depth_in[i];
      if (io.plive != nullptr) io.plive[c] = 1;
      if (io.ppvar != nullptr) io.ppvar[c] = -1;
    }
    return;
  }
  size_t c_down, c_up;
  if (io.slots == nullptr) {
    // stack order: slot base + p + 1 is popped first
    const size_t c_first = (size_t)io.base + (size_t)p + 1;
    const size_t c_second = c_first - 1;
    c_down = up_first ? c_second : c_first;
    c_up = up_first ? c_first : c_second;
  } else {
    // the preferred child takes the lower child index p
    const size_t c_first = slot_of(p), c_second = slot_of(p + 1);
    c_down = up_first ? c_second : c_first;
    c_up = up_first ? c_first : c_second;
  }
  double *dl = io.plb + c_down * n, *du = io.pub + c_down * n;
  double *ul = io.plb + c_up * n, *uu = io.pub + c_up * n;
  for (int k = lane; k < n; k += 64) {
    const double l = sl[k], u = su[k];
    dl[k] = l;
    du[k] = k == j ? floor(v) : u;
    ul[k] = k == j ? ceil(v) : l;
    uu[k] = u;
  }
  if (io.ws_head != nullptr) {
    const int m = io.m, N = io.N;
    const size_t mm = (size_t)m * m;
    for (int k = lane; k < m; k += 64) {
      const int32_t h = io.wo_head[(size_t)i * m + k];
      io.ws_head[c_down * m + k] = h;
      io.ws_head[c_up * m + k] = h;
    }
    for (int k = lane; k < N; k += 64) {
      const int8_t st = io.wo_st[(size_t)i * N + k];
      const double d = io.wo_d[(size_t)i * N + k];
      io.ws_st[c_down * N + k] = st;
      io.ws_st[c_up * N + k] = st;
      io.ws_d[c_down * N + k] = d;
      io.ws_d[c_up * N + k] = d;
    }
    for (size_t k = lane; k < mm; k += 64) {
      const double b = io.wo_binv[(size_t)i * mm + k];
      io.ws_binv[c_down * mm + k] = b;
      io.ws_binv[c_up * mm + k] = b;
    }
  }
  if (io.opk != nullptr) {
    const int kp = io.opk[i];
    const int N = io.N;
    if (lane < kp) {
      const uint32_t v = io.oppath[(size_t)i * kPathMax + lane];
      io.ppath[c_down * kPathMax + lane] = v;
      io.ppath[c_up * kPathMax + lane] = v;
    }
    if (kp > 0)
      for (int k = lane; k < N; k += 64) {
        const int8_t v = io.opst[(size_t)i * N + k];
        io.ppst[c_down * N + k] = v;
        io.ppst[c_up * N + k] = v;
      }
    if (lane == 0) {
      io.ppk[c_down] = kp;
      io.ppk[c_up] = kp;
    }
  }
  if (lane == 0) {
    const double bound = io.obj[i];
    io.pnlb[c_down] = bound;
    io.pnlb[c_up] = bound;
    io.pdepth[c_down] = io.depth_in[i] + 1;
    io.pdepth[c_up] = io.depth_in[i] + 1;
    if (io.plive != nullptr) {
      io.plive[c_down] = 1;
      io.plive[c_up] = 1;
    }
    if (io.ppvar != nullptr) {  // Branch::getActivity: x_j at the branching
      io.ppvar[c_down] = j;
      io.ppvar[c_up] = j;
      io.ppval[c_down] = v;
      io.ppval[c_up] = v;
    }
  }
}

}  // namespace

hipError_t launch_bnb_tail(const BnbIO &io, int n, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  const int nblk = (io.nb + kScanBlock - 1) / kScanBlock;
  hipLaunchKernelGGL(bnb_scan_block, dim3(nblk), dim3(kScanBlock), 0, stream, io);
  hipLaunchKernelGGL(bnb_scan_top, dim3(1), dim3(1024), 0, stream, io, nblk);
  if (!io.defer_children)
    hipLaunchKernelGGL(bnb_children, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io, n);
  return hipGetLastError();
}

hipError_t launch_bnb_children(const BnbIO &io, int n, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(bnb_children, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io, n);
  return hipGetLastError();
}

}  // namespace mgpu

namespace mgpu {
namespace {

// Keeps pool slots i = rank (mod world) of [0, count) and packs them to
// slots i / world, through a scratch copy (src -> tmp -> pool).
__global__ __launch_bounds__(256) void bnb_shard_copy(const double *slb, const double *sub,
                                                      const double *snlb, const int32_t *sdep,
                                                      double *dlb, double *dub, double *dnlb,
                                                      int32_t *ddep, int count, int n, int rank,
                                                      int world, int to_tmp) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);  // kept node
  const int i = rank + k * world;                      // its pool slot
  if (i >= count) return;
  const size_t from = to_tmp ? (size_t)i : (size_t)k;
  const size_t to = (size_t)k;
  for (int j = lane; j < n; j += 64) {
    dlb[to * n + j] = slb[from * n + j];
    dub[to * n + j] = sub[from * n + j];
  }
  if (lane == 0) {
    dnlb[to] = snlb[from];
    ddep[to] = sdep[from];
  }
}

// Generic per-slot row compaction for the depth-first shard: row k of dst =
// row (rank + k * world) of src (to_tmp) or row k of src (back), one wave
// per row, 4-byte words when the row allows, bytes otherwise.
__global__ __launch_bounds__(256) void bnb_rows_copy(const unsigned char *src, unsigned char *dst,
                                                     size_t row_bytes, int kept, int rank,
                                                     int world, int to_tmp) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= kept) return;
  const size_t from = to_tmp ? (size_t)rank + (size_t)k * world : (size_t)k;
  const unsigned char *a = src + from * row_bytes;
  unsigned char *b = dst + (size_t)k * row_bytes;
  if ((row_bytes & 3) == 0) {
    const uint32_t *a4 = reinterpret_cast<const uint32_t *>(a);
    uint32_t *b4 = reinterpret_cast<uint32_t *>(b);
    for (size_t t = lane; t < row_bytes / 4; t += 64) b4[t] = a4[t];
  } else {
    for (size_t t = lane; t < row_bytes; t += 64) b[t] = a[t];
  }
}

}  // namespace

hipError_t launch_bnb_shard_rows(unsigned char *rows, unsigned char *tmp, size_t row_bytes,
                                 int kept, int rank, int world, hipStream_t stream) {
  if (kept <= 0 || row_bytes == 0) return hipSuccess;
  const dim3 grid((kept + 3) / 4), blk(256);
  hipLaunchKernelGGL(bnb_rows_copy, grid, blk, 0, stream, rows, tmp, row_bytes, kept, rank, world,
                     1);
  hipLaunchKernelGGL(bnb_rows_copy, grid, blk, 0, stream, tmp, rows, row_bytes, kept, rank, world,
                     0);
  return hipGetLastError();
}

hipError_t launch_bnb_shard(double *plb, double *pub, double *pnlb, int32_t *pdep, double *tlb,
                            double *tub, double *tnlb, int32_t *tdep, int count, int n,
                            int rank, int world, int *kept, hipStream_t stream) {
  const int k = count > rank ? (count - rank + world - 1) / world : 0;
  *kept = k;
  if (k == 0) return hipSuccess;
  const dim3 grid((k + 3) / 4), blk(256);
  hipLaunchKernelGGL(bnb_shard_copy, grid, blk, 0, stream, plb, pub, pnlb, pdep, tlb, tub, tnlb,
                     tdep, count, n, rank, world, 1);
  hipLaunchKernelGGL(bnb_shard_copy, grid, blk, 0, stream, tlb, tub, tnlb, tdep, plb, pub, pnlb,
                     pdep, count, n, rank, world, 0);
  return hipGetLastError();
}

}  // namespace mgpu

namespace mgpu {
namespace {

// Child boxes of strong branching (ReliabilityBrancher::strongBranch_,
// ReliabilityBrancher.cpp:469-506 via IntVarHandler::getBrMod,
// IntVarHandler.cpp:111-126): child 2c = down (ub = floor(x)), child 2c+1 =
// up (lb = ceil(x)) of candidate c; one wave per child.
__global__ __launch_bounds__(256) void sb_boxes(const double *plb, const double *pub,
                                                const int32_t *var, const double *val,
                                                int nchild, int n, double *clb, double *cub) {
  const int lane = threadIdx.x & 63;
  const int ch = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ch >= nchild) return;
  const int c = ch >> 1;
  const bool up = ch & 1;
  const int j = var[c];
  const double v = val[c];
  double *dl = clb + (size_t)ch * n, *du = cub + (size_t)ch * n;
  for (int k = lane; k < n; k += 64) {
    double l = plb[k], u = pub[k];
    if (k == j) {
      if (up) l = ceil(v);
      else u = floor(v);
    }
    dl[k] = l;
    du[k] = u;
  }
}

}  // namespace

hipError_t launch_sb_boxes(const double *plb, const double *pub, const int32_t *var,
                           const double *val, int ncand, int n, double *clb, double *cub,
                           hipStream_t stream) {
  if (ncand <= 0) return hipSuccess;
  const int nchild = 2 * ncand;
  hipLaunchKernelGGL(sb_boxes, dim3((nchild + 3) / 4), dim3(256), 0, stream, plb, pub, var, val,
                     nchild, n, clb, cub);
  return hipGetLastError();
}

}  // namespace mgpu
