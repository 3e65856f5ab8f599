// K3 — batched bounded dual simplex, gfx950.
//
// Replaces OsiLPEngine::solve -> Clp resolve() (src/interfaces/
// OsiLPEngine.cpp:571-652): dual simplex from the loaded warm basis
// (OsiDoDualInResolve, :579-583), iteration limit (:561-569) and the status
// map (:592-627) onto EngineStatus numerics (src/base/Types.h:152-166).
// The arithmetic restates oracle/lp_dual.c step for step (same pricing,
// Harris two-pass ratio test, tie-breaks and update order), so the GPU and
// the CPU restatement follow the same pivot sequence.
//
// Mapping (MI355X-first): ONE NODE PER WAVE64, kLpWaves nodes per
// workgroup.
//  * The dense basis inverse lives in VGPRs: lane i holds row i of B^{-1}
//    (64 f64 = 128 VGPRs, fully unrolled, never spilled); basic values,
//    bounds and the basic column index of row i are lane-i registers.
//  * Products with a vector distributed one element per lane (B^{-1} a_q,
//    B^{-1} w) broadcast the vector with v_readlane: no LDS traffic.
//  * The constraint matrix is staged once per workgroup into LDS in both
//    CSC (pivot row rho'A) and CSR (primal recompute) and shared by the
//    waves; per-column state (reduced costs, values, working bounds, pivot
//    row, status) is a per-wave LDS slice, swept lane-strided.
//  * Reductions (pricing arg-max, ratio-test min / arg-max) are xor
//    butterflies with deterministic lowest-index tie-breaks.
//  * Pivots: B^{-1} row r is published to LDS once and read back as a
//    broadcast for both the pivot row and the rank-1 update.
#include "mgpu_internal.h"
#include "sb_rule.h"
#include "wave.h"

namespace mgpu {

#ifdef MGPU_STAMPS
// Diagnostic build only (-DMGPU_STAMPS, tools/lp_stamps.py): s_memtime
// cycles per section summed over all waves; never compiled into the product.
__device__ unsigned long long g_lp_stamps[16];
#define STAMP_KSTART const unsigned long long st_k0 = __builtin_amdgcn_s_memtime();
#define STAMP_DECL unsigned long long st_acc[16] = {0}, st_t = __builtin_amdgcn_s_memtime(); \
  const unsigned long long st_pro = st_t - st_k0;
#define STAMP(i)                                              \
  do {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t_ - st_t;                                   \
    st_t = t_;                                                \
  } while (0)
#define STAMP_FLUSH                                            \
  if ((threadIdx.x & 63) == 0)                                \
    for (int i_ = 0; i_ < 16; ++i_)                            \
      if (i_ < 10 || i_ > 11) atomicAdd(&g_lp_stamps[i_], st_acc[i_]); \
  if ((threadIdx.x & 63) == 0) {                               \
    atomicAdd(&g_lp_stamps[10], __builtin_amdgcn_s_memtime() - st_k0); \
    atomicAdd(&g_lp_stamps[11], st_pro);                       \
  }
#else
#define STAMP_KSTART
#define STAMP_DECL
#define STAMP(i) \
  do {           \
  } while (0)
#define STAMP_FLUSH
#endif

namespace {

constexpr double kPTol = 1e-7;    // primal feasibility (Clp default)
constexpr double kDTol = 1e-7;    // dual feasibility (Clp default)
constexpr double kPivTol = 1e-9;  // smallest |alpha_rq| allowed to pivot
constexpr double kArt0 = 1e7;     // first artificial box half-width
constexpr double kInfB = 1e30;    // |bound| >= this is infinite in the LP

constexpr int kUnknownStatus = 12;  // EngineUnknownStatus: node not solved

enum : int8_t { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };

__host__ __device__ constexpr size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

__host__ __device__ inline size_t shared_a_bytes(int n, int m, int nnz) {
  return al16((size_t)(n + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)(m + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         3 * al16((size_t)n * 8) + 2 * al16((size_t)m * 8);  // c, box (batch 1), row bounds
}
// Shared warm start (one basis for every node, e.g. the root optimum)
// staged once per workgroup: B^-1 (column-major), reduced costs, status,
// basic columns.
__host__ __device__ inline size_t shared_ws_bytes(int n, int m) {
  return al16((size_t)m * m * 8) + al16((size_t)(n + m) * 8) + al16((size_t)(n + m)) +
         al16((size_t)m * 4);
}
__host__ __device__ inline size_t wave_bytes(int N) {
  return 6 * al16((size_t)N * 8) + 2 * al16((size_t)N) + 2 * 64 * 8;
}
// per-node rows: the wave's copy of the matrix values (CSC, CSR) and row
// bounds, with the node's entries written over the loaded ones
__host__ __device__ inline size_t rows_wave_bytes(int m, int nnz) {
  return 2 * al16((size_t)nnz * 8) + 2 * al16((size_t)m * 8);
}

__device__ __forceinline__ double art_lo(double thi, double ab) {
  return (thi < kInfB ? thi : 0.0) - ab;
}
__device__ __forceinline__ double art_hi(double tlo, double ab) {
  return (tlo > -kInfB ? tlo : 0.0) + ab;
}

struct Ctx {
  // shared matrix
  const int *colptr, *rowidx, *rowptr, *ccol;
  const double *cval, *rval;
  // per-wave column state
  double *d, *z, *blo, *bhi, *al, *t2, *rho, *aq;
  int8_t *st, *art;
  // problem
  int n, m, N;
  const double *nlb, *nub, *rlo, *rhi, *c;
  int ocol;        // >= 0: objective is osign * x[ocol] (bound LP), else c
  double osign;
  int lane;
  __device__ __forceinline__ double cj(int j) const {
    return ocol < 0 ? c[j] : (j == ocol ? osign : 0.0);
  }
  __device__ __forceinline__ double tlo(int j) const {
    const double v = j < n ? nlb[j] : rlo[j - n];
    return v < -kInfB ? -INFINITY : v;
  }
  __device__ __forceinline__ double thi(int j) const {
    const double v = j < n ? nub[j] : rhi[j - n];
    return v > kInfB ? INFINITY : v;
  }
};

// rho' a_j over CSC column j in CSC order; four entries' loads are issued
// before their products are summed (the adds keep the sequential order)
__device__ __forceinline__ double col_dot(const Ctx &C, int j) {
  double a = 0.0;
  int t = C.colptr[j];
  const int e = C.colptr[j + 1];
  for (; t + 4 <= e; t += 4) {
    const int i0 = C.rowidx[t], i1 = C.rowidx[t + 1], i2 = C.rowidx[t + 2], i3 = C.rowidx[t + 3];
    const double v0 = C.cval[t], v1 = C.cval[t + 1], v2 = C.cval[t + 2], v3 = C.cval[t + 3];
    const double r0 = C.rho[i0], r1 = C.rho[i1], r2 = C.rho[i2], r3 = C.rho[i3];
    a += v0 * r0;
    a += v1 * r1;
    a += v2 * r2;
    a += v3 * r3;
  }
  for (; t < e; ++t) a += C.cval[t] * C.rho[C.rowidx[t]];
  return a;
}

// oracle place_nonbasic
__device__ __forceinline__ void place_nonbasic(const Ctx &C, int j, double ab) {
  const double lo = C.blo[j], hi = C.bhi[j], dj = C.d[j];
  const bool lo_f = lo > -kInfB, hi_f = hi < kInfB;
  if (lo_f && hi_f && lo == hi) {
    C.st[j] = ST_LB;
    C.z[j] = lo;
    return;
  }
  if (dj > kDTol) {
    if (!lo_f) {
      C.blo[j] = art_lo(hi, ab);
      C.art[j] |= 1;
    }
    C.st[j] = ST_LB;
    C.z[j] = C.blo[j];
  } else if (dj < -kDTol) {
    if (!hi_f) {
      C.bhi[j] = art_hi(lo, ab);
      C.art[j] |= 2;
    }
    C.st[j] = ST_UB;
    C.z[j] = C.bhi[j];
  } else {
    if (lo_f) {
      C.st[j] = ST_LB;
      C.z[j] = lo;
    } else if (hi_f) {
      C.st[j] = ST_UB;
      C.z[j] = hi;
    } else {
      C.st[j] = ST_FREE;
      C.z[j] = 0.0;
    }
  }
}

// oracle grow_art
__device__ __forceinline__ void grow_art(const Ctx &C, double ab) {
  for (int j = C.lane; j < C.N; j += 64) {
    const int8_t a = C.art[j];
    if (!a || C.st[j] == ST_BASIC) continue;
    if (a & 1) C.blo[j] = art_lo(C.thi(j), ab);
    if (a & 2) C.bhi[j] = art_hi(C.tlo(j), ab);
    if (C.st[j] == ST_LB) C.z[j] = C.blo[j];
    if (C.st[j] == ST_UB) C.z[j] = C.bhi[j];
  }
}

// oracle compute_primals: z_B = -B^{-1} (N z_N); lane k forms w_k from CSR
// row k in column order, then lane i takes row i of B^{-1} times w.
template <int M>
__device__ __forceinline__ double compute_primals(const Ctx &C, const double (&binv)[M]) {
  wave_sync();
  double w = 0.0;
  const int k = C.lane;
  if (k < C.m) {
    // four entries' loads in flight (column, then its status and value),
    // the adds in CSR order as before
    int t = C.rowptr[k];
    const int e = C.rowptr[k + 1];
    for (; t + 4 <= e; t += 4) {
      const int j0 = C.ccol[t], j1 = C.ccol[t + 1], j2 = C.ccol[t + 2], j3 = C.ccol[t + 3];
      const double r0 = C.rval[t], r1 = C.rval[t + 1], r2 = C.rval[t + 2], r3 = C.rval[t + 3];
      const int8_t s0 = C.st[j0], s1 = C.st[j1], s2 = C.st[j2], s3 = C.st[j3];
      const double z0 = C.z[j0], z1 = C.z[j1], z2 = C.z[j2], z3 = C.z[j3];
      if (s0 != ST_BASIC && z0 != 0.0) w += r0 * z0;
      if (s1 != ST_BASIC && z1 != 0.0) w += r1 * z1;
      if (s2 != ST_BASIC && z2 != 0.0) w += r2 * z2;
      if (s3 != ST_BASIC && z3 != 0.0) w += r3 * z3;
    }
    for (; t < e; ++t) {
      const int j = C.ccol[t];
      if (C.st[j] == ST_BASIC) continue;
      const double zj = C.z[j];
      if (zj == 0.0) continue;
      w += C.rval[t] * zj;
    }
    const int jl = C.n + k;
    if (C.st[jl] != ST_BASIC) {
      const double zl = C.z[jl];
      if (zl != 0.0) w -= zl;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < M; ++q) s += binv[q] * rld(w, q);
  return -s;
}

// M: basis rows held per lane (m <= M; 8, 16, 32 or 64): the B^-1 row
// registers and every unrolled row loop are sized to the problem's bucket.
template <int W, bool kSharedWs, int M>
__global__ __launch_bounds__(64 * W) void lp_dual_kernel(DevLP lp, LpIO io) {
  STAMP_KSTART
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m, N = n + m, nnz = lp.nnz;
  const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // node list (K3P overflow re-solve): a workgroup with no node of it
  // leaves before staging anything (uniform over the workgroup)
  const int lo = io.node_list != nullptr ? io.list_lo : 0;
  int nsolve = io.batch;
  if (io.node_list != nullptr) {
    nsolve = *io.node_count;
    if (nsolve > io.list_hi) nsolve = io.list_hi;
  }
  // self-resetting node counter: every wave counts itself out, the last one
  // zeroes the counter for the next launch on the stream (no fill kernel)
  auto leave = [&]() {
    if (io.next_exit != nullptr && lane0 == 0 &&
        atomicAdd(io.next_exit, 1) == (int)gridDim.x * W - 1) {
      atomicExch(io.next, 0);
      atomicExch(io.next_exit, 0);
    }
  };
  if (lo + (int)blockIdx.x * W >= nsolve) {
    leave();
    return;
  }

  // ---- stage the constraint matrix (CSC + CSR) once per workgroup ----
  unsigned char *p = smem;
  int *s_colptr = (int *)p;      p += al16((size_t)(n + 1) * 4);
  int *s_rowidx = (int *)p;      p += al16((size_t)nnz * 4);
  double *s_cval = (double *)p;  p += al16((size_t)nnz * 8);
  int *s_rowptr = (int *)p;      p += al16((size_t)(m + 1) * 4);
  int *s_ccol = (int *)p;        p += al16((size_t)nnz * 4);
  double *s_rval = (double *)p;  p += al16((size_t)nnz * 8);
  for (int t = threadIdx.x; t <= n; t += 64 * W) s_colptr[t] = lp.colptr[t];
  for (int t = threadIdx.x; t <= m; t += 64 * W) s_rowptr[t] = lp.rowptr[t];
  for (int t = threadIdx.x; t < nnz; t += 64 * W) {
    s_rowidx[t] = lp.rowidx[t];
    s_cval[t] = lp.cval[t];
    s_ccol[t] = lp.ccol[t];
    s_rval[t] = lp.rval[t];
  }
  // objective and row bounds beside the matrix (the objective sum and the
  // rebuilt reduced costs read them column by column); a single-LP launch
  // (HipLPEngine's route) also stages its box here, so its loads overlap
  // the matrix's instead of following them
  double *s_c = (double *)p;    p += al16((size_t)n * 8);
  double *s_rlo = (double *)p;  p += al16((size_t)m * 8);
  double *s_rhi = (double *)p;  p += al16((size_t)m * 8);
  double *s_blb = (double *)p;  p += al16((size_t)n * 8);
  double *s_bub = (double *)p;  p += al16((size_t)n * 8);
  const bool box1 = io.batch == 1 && io.node_list == nullptr && io.chain_n == nullptr;
  for (int t = threadIdx.x; t < n; t += 64 * W) {
    s_c[t] = lp.objd[t];
    if (box1) {
      s_blb[t] = io.lb[t];
      s_bub[t] = io.ub[t];
    }
  }
  for (int t = threadIdx.x; t < m; t += 64 * W) {
    s_rlo[t] = lp.rlo[t];
    s_rhi[t] = lp.rhi[t];
  }
  double *s_wbinv = nullptr, *s_wd = nullptr;
  int8_t *s_wst = nullptr;
  int32_t *s_whead = nullptr;
  if constexpr (kSharedWs) {
    s_wbinv = (double *)p;  p += al16((size_t)m * m * 8);
    s_wd = (double *)p;     p += al16((size_t)N * 8);
    s_wst = (int8_t *)p;    p += al16((size_t)N);
    s_whead = (int32_t *)p; p += al16((size_t)m * 4);
    for (int t = threadIdx.x; t < m * m; t += 64 * W) s_wbinv[t] = io.ws.binv[t];
    for (int t = threadIdx.x; t < N; t += 64 * W) {
      if (io.ws.d != nullptr) s_wd[t] = io.ws.d[t];  // bound LPs rebuild d
      s_wst[t] = io.ws.st[t];
    }
    for (int t = threadIdx.x; t < m; t += 64 * W) s_whead[t] = io.ws.head[t];
  }
  __syncthreads();

  // Persistent waves: the matrix (and a shared warm start) were staged once
  // for the workgroup; each wave then solves nodes b, b + grid*W, ...
  // (no workgroup barrier below this point).
  STAMP_DECL
  for (int bi = lo + blockIdx.x * W + wave;; bi += gridDim.x * W) {
    if (io.next != nullptr) {  // dynamic schedule: the next unsolved list position
      int t = 0;
      if (lane0 == 0) t = atomicAdd(io.next, 1);
      bi = lo + __builtin_amdgcn_readfirstlane(t);
    }
    if (bi >= nsolve) break;
    const int unit = io.node_list != nullptr ? io.node_list[bi] : bi;
    // chained mode: the unit's LPs one after the other (one LP otherwise)
    const bool chained = io.chain_n != nullptr;
    const int c0 = chained ? 2 * io.chain_off[unit] : unit;
    const int cn = chained ? 2 * io.chain_n[unit] : 1;
    int pst0 = 0, pst1 = 0;        // the chain's last pair: statuses, values
    double pob0 = 0.0, pob1 = 0.0;
    // the basis: B^-1 rows, basic column per lane; in chained mode `held`
    // says the wave still holds the chain slot's basis (the last LP kept its
    // basis and wrote it there), so the next LP need not read it back
    double binv[M];
    int h = -1;
    bool held = false;
    for (int cs = 0; cs < cn; ++cs) {
    if (chained && cs >= 2 && (cs & 1) == 0) {
      const double ov = io.chain_nobj[unit];
      double cd, cu;
      if (sb_verdict(pst0, pob0, pst1, pob1, ov, io.chain_cutoff - ov, cd, cu) > 0) break;
    }
    auto note = [&](int st, double ob) {
      if (cs & 1) {
        pst1 = st;
        pob1 = ob;
      } else {
        pst0 = st;
        pob0 = ob;
      }
    };
    const int b = chained ? c0 + cs : unit;
    // pivots already made by K3P / K3PW (continuation): counted by the
    // iteration limit, the Bland switch and the reported total
    const int ib = io.iter_base_list != nullptr ? io.iter_base_list[bi] : io.iter_base;
    const int bw = io.ws_index != nullptr ? io.ws_index[b] : io.list_ws ? bi : b;  // warm start

    // lane index made opaque per node: otherwise LICM hoists the 64
    // loop-invariant B^-1 init values / LDS addresses out of the node loop
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const bool nrows = io.nr.vals != nullptr;
    unsigned char *wp =
        p + (size_t)wave * (wave_bytes(N) + (nrows ? rows_wave_bytes(m, nnz) : 0));
    Ctx C;
    C.colptr = s_colptr; C.rowidx = s_rowidx; C.cval = s_cval;
    C.rowptr = s_rowptr; C.ccol = s_ccol; C.rval = s_rval;
    C.d = (double *)wp;   wp += al16((size_t)N * 8);
    C.z = (double *)wp;   wp += al16((size_t)N * 8);
    C.blo = (double *)wp; wp += al16((size_t)N * 8);
    C.bhi = (double *)wp; wp += al16((size_t)N * 8);
    C.al = (double *)wp;  wp += al16((size_t)N * 8);
    C.t2 = (double *)wp;  wp += al16((size_t)N * 8);
    C.st = (int8_t *)wp;  wp += al16((size_t)N);
    C.art = (int8_t *)wp; wp += al16((size_t)N);
    C.rho = (double *)wp; wp += 64 * 8;
    C.aq = (double *)wp;  wp += 64 * 8;
    C.n = n; C.m = m; C.N = N;
    C.nlb = box1 ? s_blb : io.lb + (size_t)b * io.box_stride;
    C.nub = box1 ? s_bub : io.ub + (size_t)b * io.box_stride;
    C.rlo = s_rlo; C.rhi = s_rhi; C.c = s_c;
    C.ocol = io.obj_col != nullptr ? io.obj_col[b] : -1;
    C.osign = io.obj_col != nullptr ? io.obj_sign[b] : 0.0;
    C.lane = lane;

    if (io.skip != nullptr && io.skip[b] != 0) {  // pruned by FBBT: not solved
      if (lane == 0) {
        io.status[b] = kUnknownStatus;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      note(kUnknownStatus, INFINITY);
      held = false;
      continue;
    }
    if (nrows) {
      // the node's matrix and row bounds: the loaded values, then its own
      // entries (OsiLPEngine::changeConstraint of the rewritten rows)
      double *wc = (double *)wp;  wp += al16((size_t)nnz * 8);
      double *wr = (double *)wp;  wp += al16((size_t)nnz * 8);
      double *wlo = (double *)wp; wp += al16((size_t)m * 8);
      double *whi = (double *)wp;
      for (int t = lane; t < nnz; t += 64) {
        wc[t] = s_cval[t];
        wr[t] = s_rval[t];
      }
      for (int i = lane; i < m; i += 64) {
        wlo[i] = s_rlo[i];
        whi[i] = s_rhi[i];
      }
      wave_sync();
      const double *rec = io.nr.vals + (size_t)b * io.nr.stride;
      for (int q = lane; q < io.nr.ncoef; q += 64) {
        double v = rec[io.nr.coef_src[q]];
        if (fabs(v) <= kLfTol) v = 0.0;
        wc[io.nr.csc_pos[q]] = v;
        wr[io.nr.csr_pos[q]] = v;
      }
      for (int q = lane; q < io.nr.nrow; q += 64) {
        const int r = io.nr.row[q];
        if (io.nr.lo_src[q] >= 0) wlo[r] = rec[io.nr.lo_src[q]];
        if (io.nr.hi_src[q] >= 0) whi[r] = rec[io.nr.hi_src[q]];
      }
      wave_sync();
      C.cval = wc;
      C.rval = wr;
      C.rlo = wlo;
      C.rhi = whi;
    }

    // ---- working bounds; an empty box is infeasible before any pivot ----
    bool bad = false;
    for (int j = lane; j < N; j += 64) {
      C.blo[j] = C.tlo(j);
      C.bhi[j] = C.thi(j);
      C.art[j] = 0;
      bad |= C.blo[j] > C.bhi[j] + kPTol;
    }
    if (__any(bad)) {
      if (lane == 0) {
        io.status[b] = 2;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      note(2, INFINITY);
      held = false;
      continue;
    }

    // ---- basis: warm start (parent / root optimum) or slack basis ----
    const bool warm = io.ws.head != nullptr;
    if (warm && chained && held) {
      // the chain slot is this wave's own last basis: statuses, reduced
      // costs (0 on basic columns) in LDS and B^-1 / h in registers are what
      // the load below would produce
    } else if (warm) {
      const int32_t *wh = kSharedWs ? s_whead : io.ws.head + (size_t)bw * io.ws.s_head;
      const int8_t *wst = kSharedWs ? s_wst : io.ws.st + (size_t)bw * io.ws.s_st;
      const double *wd = kSharedWs ? s_wd : io.ws.d + (size_t)bw * io.ws.s_d;
      const double *wb = kSharedWs ? s_wbinv : io.ws.binv + (size_t)bw * io.ws.s_binv;
      for (int j = lane; j < N; j += 64) {
        const int8_t s = wst[j];
        C.st[j] = s == ST_BASIC ? ST_LB : s;
      }
      if (lane < m) h = wh[lane];
      wave_sync();
      if (lane < m) C.st[h] = ST_BASIC;
      wave_sync();
  #pragma unroll
      for (int k = 0; k < M; ++k)
        binv[k] = (lane < m && k < m) ? wb[(size_t)k * m + lane] : 0.0;  // column-major: coalesced
      if (C.ocol < 0 && io.ws.d != nullptr) {
        for (int j = lane; j < N; j += 64) C.d[j] = C.st[j] == ST_BASIC ? 0.0 : wd[j];
      } else {
        // reduced costs of the warm basis for the loaded objective (oracle
        // compute_duals): y = c_B' B^-1 accumulated over the basic rows in
        // order -- for a bound LP c_B is osign at ocol's row --, then
        // d_j = c_j - y' a_j.  A solve handed no d (the objective changed
        // since the basis was saved, HipLPEngine's OBBT loop) lands here too.
        const double cb = (lane < m && h < n) ? C.cj(h) : 0.0;
        double yk = 0.0;
        uint64_t rows = __ballot(cb != 0.0);
        while (rows != 0ull) {
          const int i = __builtin_ctzll(rows);
          rows &= rows - 1;
          if (lane == i) {  // publish row i of B^-1
  #pragma unroll
            for (int k = 0; k < M; ++k)
              if (k < m) C.aq[k] = binv[k];
          }
          wave_sync();
          const double bik = lane < m ? C.aq[lane] : 0.0;
          yk += rld(cb, i) * bik;
          wave_sync();
        }
        C.rho[lane] = lane < m ? yk : 0.0;
        wave_sync();
        for (int j = lane; j < N; j += 64) {
          if (C.st[j] == ST_BASIC) {
            C.d[j] = 0.0;
            continue;
          }
          double dot;
          if (j >= n) {
            dot = -C.rho[j - n];
          } else {
            dot = 0.0;
            for (int t = C.colptr[j]; t < C.colptr[j + 1]; ++t) dot += C.cval[t] * C.rho[C.rowidx[t]];
          }
          C.d[j] = (j < n ? C.cj(j) : 0.0) - dot;
        }
      }
    } else {
      if (lane < m) h = n + lane;
      for (int j = lane; j < N; j += 64) {
        C.st[j] = j >= n ? ST_BASIC : ST_LB;
        C.d[j] = j < n ? C.cj(j) : 0.0;  // y = 0 for the slack basis
      }
  #pragma unroll
      for (int k = 0; k < M; ++k) binv[k] = (k == lane && lane < m) ? -1.0 : 0.0;
    }
    wave_sync();
    STAMP(12);
    double art_bound = kArt0;
    for (int j = lane; j < N; j += 64) {
      if (C.st[j] == ST_BASIC) continue;
      const double lo = C.blo[j], hi = C.bhi[j], dj = C.d[j];
      bool keep = false;
      if (warm) {
        const int8_t s = C.st[j];
        if (s == ST_LB && lo > -kInfB && dj >= -kDTol) {
          C.z[j] = lo;
          keep = true;
        } else if (s == ST_UB && hi < kInfB && dj <= kDTol) {
          C.z[j] = hi;
          keep = true;
        } else if (lo == hi && lo > -kInfB) {
          C.st[j] = ST_LB;
          C.z[j] = lo;
          keep = true;
        }
      }
      if (!keep) place_nonbasic(C, j, art_bound);
    }
    wave_sync();
    STAMP(13);
    double lbB = 0.0, ubB = 0.0;
    if (lane < m) {
      lbB = C.blo[h];
      ubB = C.bhi[h];
    }
    double zB = compute_primals(C, binv);

    int status = kUnknownStatus, iters = 0;
    bool fresh = true;
    STAMP(0);
    for (;;) {
      // ---- pricing: most infeasible basic row (Dantzig), lowest row on ties
      double inf = 0.0;
      if (lane < m) {
        if (zB < lbB - kPTol) inf = zB - lbB;
        else if (zB > ubB + kPTol) inf = zB - ubB;
      }
      double best = fabs(inf);
      int r = wave_argmax_lane(best);  // used only when best > 0
      // keep the (wave-uniform) result in a VGPR: as an SGPR value it lets
      // LLVM re-schedule the pivot around it at +100 VGPRs
      asm volatile("" : "+v"(best));
      // anti-cycling (oracle STALL_PIVOTS): past kStallPivots pivots of the
      // solve, Bland's rule: the infeasible row with the lowest basic column,
      // and below the exact minimum ratio with the lowest column on ties
      const bool bland = iters + ib >= kStallPivots;
      if (best == 0.0) {
        if (!fresh) {
          zB = compute_primals(C, binv);
          fresh = true;
          continue;
        }
        bool grow = false;
        for (int j = lane; j < N; j += 64) {
          const int8_t a = C.art[j], s = C.st[j];
          if (s == ST_BASIC || !a) continue;
          if ((s == ST_LB && (a & 1)) || (s == ST_UB && (a & 2))) grow = true;
        }
        if (!__any(grow)) {
          status = 0;
          break;
        }
        if (art_bound >= 1e13) {
          status = 4;
          break;
        }
        art_bound *= 1e3;
        grow_art(C, art_bound);
        zB = compute_primals(C, binv);
        fresh = true;
        continue;
      }
      if (iters + ib >= io.iter_limit) {
        status = 6;
        break;
      }
      if (bland) {
        double key = (lane < m && inf != 0.0) ? -(double)h : -INFINITY;
        int rr = lane;
        wave_argmax_idx(key, rr);
        r = rr;
      }
      const double delta = rld(inf, r);
      STAMP(1);

      // ---- row r of B^{-1} to LDS (read back as a broadcast) ----
      if (lane == r) {
  #pragma unroll
        for (int k = 0; k < M; k += 2) {
          double2 v;
          v.x = binv[k];
          v.y = binv[k + 1];
          *reinterpret_cast<double2 *>(C.rho + k) = v;
        }
      }
      wave_sync();
      const double sigma = delta > 0 ? 1.0 : -1.0;

      STAMP(2);
      // ---- pivot row and Harris pass 1 (pass 2's ratio is cached in t2:
      // +inf for columns that cannot enter) ----
      double tmax = INFINITY;
      for (int j = lane; j < N; j += 64) {
        const int8_t s = C.st[j];
        double a = 0.0, t2 = INFINITY;
        if (s != ST_BASIC && C.blo[j] != C.bhi[j]) {
          if (j >= n) {
            a = -C.rho[j - n];
          } else {
            a = col_dot(C, j);
          }
          // Harris ratios without divergent branches: one numerator pair and
          // denominator per case, two divisions for every lane (the same
          // operands as the per-case formulas, so the same values)
          const double at = sigma * a, dj = C.d[j], fat = fabs(at);
          const bool lb = s == ST_LB && at > kPivTol, ub = s == ST_UB && at < -kPivTol,
                     fr = s == ST_FREE && fat > kPivTol;
          const double n2 = lb ? fmax(dj, 0.0) : ub ? fmin(dj, 0.0) : 0.0;
          const double n1 = lb ? n2 + kDTol : ub ? n2 - kDTol : kDTol;
          const double den = fr ? fat : at;
          if (lb || ub || fr) {
            const double t = n1 / den;
            t2 = fr ? 0.0 : n2 / den;
            if (t < tmax) tmax = t;
          }
        }
        C.al[j] = a;
        C.t2[j] = t2;
      }
      tmax = wave_min_dpp(tmax);
      asm volatile("" : "+v"(tmax));
      if (tmax == INFINITY) {  // dual unbounded
        bool boxed = false;
        for (int j = lane; j < N; j += 64) boxed |= C.st[j] != ST_BASIC && C.art[j] != 0;
        if (!__any(boxed) || art_bound >= 1e13) {
          status = 2;
          break;
        }
        art_bound *= 1e3;
        grow_art(C, art_bound);
        zB = compute_primals(C, binv);
        fresh = true;
        continue;
      }
      STAMP(3);
      // ---- Harris pass 2: largest |alpha| among ratios <= tmax ----
      double qa = 0.0;
      int q = INT_MAX;
      if (!bland) {
        for (int j = lane; j < N; j += 64) {
          if (C.t2[j] <= tmax) {
            const double fa = fabs(C.al[j]);
            if (fa > qa) {
              qa = fa;
              q = j;
            }
          }
        }
        wave_argmax_idx(qa, q);
      } else {
        double key = -INFINITY;
        for (int j = lane; j < N; j += 64) {
          const double t2 = C.t2[j];
          if (t2 != INFINITY && -t2 > key) {
            key = -t2;
            q = j;
          }
        }
        wave_argmax_idx(key, q);
        qa = q != INT_MAX ? fabs(C.al[q]) : 0.0;
      }
      if (qa == 0.0) {
        status = 2;
        break;
      }

      STAMP(4);
      // ---- column q: alpha_q = B^{-1} a_q (a_q one element per lane) ----
      double aqk;
      if (q < n) {
        C.aq[lane] = 0.0;
        wave_sync();
        const int cs = C.colptr[q], deg = C.colptr[q + 1] - cs;
        for (int t = lane; t < deg; t += 64) C.aq[C.rowidx[cs + t]] = C.cval[cs + t];
        wave_sync();
        aqk = C.aq[lane];
      } else {
        aqk = lane == q - n ? -1.0 : 0.0;
      }
      double alq = 0.0;
  #pragma unroll
      for (int k = 0; k < M; ++k) alq += binv[k] * rld(aqk, k);
      const double arq = rld(alq, r);

      STAMP(5);
      // ---- steps ----
      double theta_d = C.d[q] / C.al[q];
      if (sigma * theta_d < 0) theta_d = 0.0;
      const double theta_p = delta / arq;
      const int pl = rl(h, r);
      for (int j = lane; j < N; j += 64) {
        if (C.st[j] == ST_BASIC) continue;
        C.d[j] -= theta_d * C.al[j];
      }
      const double zq = C.z[q] + theta_p;
      const int8_t art_q = C.art[q];
      const double bloq = C.blo[q], bhiq = C.bhi[q];
      const double bound_p = delta < 0 ? C.blo[pl] : C.bhi[pl];
      wave_sync();
      if (lane == 0) {
        C.d[q] = 0.0;
        C.d[pl] = -theta_d;
        C.st[pl] = delta < 0 ? ST_LB : ST_UB;
        C.z[pl] = bound_p;
        C.st[q] = ST_BASIC;
        C.z[q] = zq;
        if (art_q) {  // basic columns keep their true (infinite) bounds
          C.blo[q] = C.tlo(q);
          C.bhi[q] = C.thi(q);
          C.art[q] = 0;
        }
      }
      if (lane < m) zB -= theta_p * alq;
      if (lane == r) {
        h = q;
        zB = zq;
        lbB = art_q ? C.tlo(q) : bloq;
        ubB = art_q ? C.thi(q) : bhiq;
      }
      STAMP(6);
      // ---- rank-1 update of B^{-1} ----
      const double inv = 1.0 / arq;
  #pragma unroll
      for (int k = 0; k < M; ++k) {
        const double nr = C.rho[k] * inv;
        binv[k] = lane == r ? nr : binv[k] - alq * nr;
      }
      STAMP(7);
      ++iters;
      fresh = false;
      if (iters % 64 == 0) {
        zB = compute_primals(C, binv);
        fresh = true;
      }
    }

    // ---- outputs ----
    STAMP(8);
    wave_sync();
    double objv = status == 2 ? INFINITY : -INFINITY;
    if (status == 0 || status == 6) {
      if (lane < m) C.z[h] = zB;
      wave_sync();
      // objective as the oracle sums it: sequentially over the columns, so
      // the value is the oracle's bit for bit (the batched tree's reliability
      // branching compares strong-branching values and pseudocosts exactly)
      // the products lane-parallel (the same roundings: no contraction),
      // then summed in column order through lane reads of the nonzero ones
      // (adding +-0 to a sum that starts at +0 never changes its bits: the
      // sum is never -0, so the value is the full sum's)
      double s = 0.0;
      for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        const double pj = j < n ? C.cj(j) * C.z[j] : 0.0;
        uint64_t nz = __ballot(pj != 0.0);
        while (nz != 0ull) {
          const int l = __builtin_ctzll(nz);
          nz &= nz - 1ull;
          s += rld(pj, l);
        }
      }
      objv = C.ocol < 0 ? s + lp.objoff : s;
      if (lane == 0) io.obj[b] = objv;
      STAMP(14);
      if (io.x != nullptr)
        for (int j = lane; j < n; j += 64) io.x[(size_t)b * n + j] = C.z[j];
      if (io.rc != nullptr)
        for (int j = lane; j < N; j += 64)
          io.rc[(size_t)b * N + j] = C.st[j] == ST_BASIC ? 0.0 : C.d[j];
      if (io.wo_head != nullptr) {
        const size_t bo = io.wo_index != nullptr ? (size_t)io.wo_index[b] : (size_t)b;
        if (lane < m) io.wo_head[bo * m + lane] = h;
        for (int j = lane; j < N; j += 64) {
          io.wo_st[bo * N + j] = C.st[j];
          io.wo_d[bo * N + j] = C.d[j];
        }
        if (lane < m) {
          double *dst = io.wo_binv + bo * m * m + lane;
  #pragma unroll
          for (int k = 0; k < M; ++k)
            if (k < m) dst[(size_t)k * m] = binv[k];   // column-major: coalesced
        }
      }
      STAMP(15);
    } else if (lane == 0) {
      io.obj[b] = objv;
    }
    if (lane == 0) {
      io.status[b] = status;
      io.iters[b] = iters + ib;
    }
    if (chained) {
      note(status, objv);
      held = status == 0 || status == 6;
    }
    STAMP(9);
    }  // the unit's LPs
  }
  leave();
  STAMP_FLUSH
}

}  // namespace

#ifdef MGPU_STAMPS
extern "C" int mgpu_debug_lp_stamps(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lp_stamps), sizeof(unsigned long long) * 16) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lp_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

size_t lp_lds_bytes(int n, int m, int nnz) {
  return shared_a_bytes(n, m, nnz) + (size_t)kLpWaves * wave_bytes(n + m);
}

size_t lp_lds_bytes_rows(int n, int m, int nnz) {
  return lp_lds_bytes(n, m, nnz) + (size_t)kLpWaves * rows_wave_bytes(m, nnz);
}

static size_t lp_lds_bytes_shared(int n, int m, int nnz) {
  return lp_lds_bytes(n, m, nnz) + shared_ws_bytes(n, m);
}

hipError_t launch_lp_dual(const DevLP &lp, const LpIO &io, int num_cus, hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  if (lp.m > kLpMaxM) return hipErrorInvalidValue;
  const bool nrows = io.nr.vals != nullptr;
  const bool shared = !nrows && io.ws.head != nullptr && io.ws.s_head == 0 &&
                      io.ws.s_st == 0 && io.ws.s_d == 0 && io.ws.s_binv == 0 &&
                      lp_lds_bytes_shared(lp.n, lp.m, lp.nnz) <= 160 * 1024;
  const size_t lds = shared  ? lp_lds_bytes_shared(lp.n, lp.m, lp.nnz)
                     : nrows ? lp_lds_bytes_rows(lp.n, lp.m, lp.nnz)
                             : lp_lds_bytes(lp.n, lp.m, lp.nnz);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    const void *fns[] = {
        (const void *)lp_dual_kernel<kLpWaves, false, 8>, (const void *)lp_dual_kernel<kLpWaves, true, 8>,
        (const void *)lp_dual_kernel<kLpWaves, false, 16>, (const void *)lp_dual_kernel<kLpWaves, true, 16>,
        (const void *)lp_dual_kernel<kLpWaves, false, 32>, (const void *)lp_dual_kernel<kLpWaves, true, 32>,
        (const void *)lp_dual_kernel<kLpWaves, false, 64>, (const void *)lp_dual_kernel<kLpWaves, true, 64>};
    for (const void *f : fns) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  // persistent grid: two workgroups (8 waves) per CU is the residency the
  // 214-VGPR / 74-KB LDS budget admits at M = 64; more nodes loop inside the waves
  const int want = (io.batch + kLpWaves - 1) / kLpWaves;
  const int blocks = want < 2 * num_cus ? want : 2 * num_cus;
  auto go = [&](auto mtag) {
    constexpr int Mb = decltype(mtag)::value;
    if (shared)
      hipLaunchKernelGGL((lp_dual_kernel<kLpWaves, true, Mb>), dim3(blocks), dim3(64 * kLpWaves),
                         lds, stream, lp, io);
    else
      hipLaunchKernelGGL((lp_dual_kernel<kLpWaves, false, Mb>), dim3(blocks), dim3(64 * kLpWaves),
                         lds, stream, lp, io);
  };
  if (lp.m <= 8) go(std::integral_constant<int, 8>{});
  else if (lp.m <= 16) go(std::integral_constant<int, 16>{});
  else if (lp.m <= 32) go(std::integral_constant<int, 32>{});
  else go(std::integral_constant<int, 64>{});
  return hipGetLastError();
}

}  // namespace mgpu
