// K3L — batched bounded dual simplex for relaxations with more rows than a
// wave has lanes (m > 64), gfx950.
//
// Same algorithm, arithmetic and tie-breaks as K3 (lp_dual.hip) and its CPU
// restatement oracle/lp_dual.c — the replacement of OsiLPEngine::solve ->
// Clp resolve() (src/interfaces/OsiLPEngine.cpp:571-652): Dantzig pricing,
// Harris two-pass ratio test, explicit basis inverse with rank-1 updates,
// artificial bounds for free columns, primal refresh every 64 pivots,
// EngineStatus numerics (Types.h:152-166).  Every dot product runs in the
// oracle's order (ftran_col, compute_primals, col_dot) and the objective is
// a sequential sum, so a node follows the oracle's pivot sequence and ends
// on the oracle's objective bit for bit.
//
// Mapping (MI355X-first): ONE NODE PER WORKGROUP, persistent over nodes: one
// wave for m <= 256 (wave-level reductions, up to 16 nodes in flight per
// CU), four waves beyond.
//  * B^{-1} (m x m f64) is too large for registers or LDS at these sizes
//    (m = 1025: 8.4 MB): it lives in HBM, COLUMN-major, one slot per
//    workgroup.  Thread i owns basis row i, so every per-row sweep over a
//    column k of B^{-1} — the column alpha_q = B^{-1} a_q, the primal
//    recompute B^{-1} w and the rank-1 update — is a coalesced 512-B wave
//    access; the rank-1 update skips rows with alpha_iq = 0 (no load, no
//    store).  It is the HBM-bound part of the kernel: 16 m^2 bytes per
//    pivot at most.
//  * Per-column state (reduced costs, values, working bounds, pivot row,
//    Harris ratios, status) and the per-row vectors (row r of B^{-1}, the
//    column alpha_q, w, the basis heads) are LDS arrays of the workgroup;
//    the constraint matrix (CSC for rho'A and ftran, CSR for the primal
//    recompute) is read from HBM and stays L2-resident (shared by all
//    workgroups).
//  * Reductions (pricing arg-max, ratio min, pass-2 arg-max) are DPP wave
//    reductions combined across the 4 waves through LDS, with the oracle's
//    lowest-index tie-breaks.
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

constexpr double kPTol = 1e-7;    // primal feasibility (Clp default)
constexpr double kDTol = 1e-7;    // dual feasibility (Clp default)
constexpr double kPivTol = 1e-9;  // smallest |alpha_rq| allowed to pivot
constexpr double kArt0 = 1e7;     // first artificial box half-width
constexpr double kInfB = 1e30;    // |bound| >= this is infinite in the LP
constexpr int kUnknownStatus = 12;

enum : int8_t { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };

__host__ __device__ constexpr size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

__host__ __device__ inline size_t large_lds_bytes(int n, int m) {
  const size_t N = (size_t)n + m;
  return 6 * al16(N * 8) + 2 * al16(N) + 3 * al16((size_t)m * 8) + al16((size_t)m * 4) +
         al16(4 * 8) + al16(4 * 4);  // reduction slots: up to 4 waves
}

template <int kT>  // threads per workgroup = one node
struct S {
  double *d, *z, *blo, *bhi, *al, *t2, *rho, *aq, *w, *redv;
  int8_t *st, *art;
  int *head, *redi;
  double *Bi;                   // HBM, column-major: (i, k) at k * m + i
  const int *colptr, *rowidx, *rowptr, *ccol;
  const double *cval, *rval;
  const double *nlb, *nub, *rlo, *rhi, *c;
  int n, m, N, ocol;
  double osign;
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

// ---- workgroup reductions (every thread calls them) ------------------------
// (not __syncthreads_or: its reduction scratch is static LDS, which would not
// leave the full 160 KiB for the dynamic state)
template <int kT>
__device__ __forceinline__ bool blk_any(bool p, const S<kT> &s) {
  const bool w = __builtin_amdgcn_ballot_w64(p) != 0;
  if constexpr (kT == 64) return w;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.redi[threadIdx.x >> 6] = w ? 1 : 0;
  __syncthreads();
  int any = 0;
  for (int w = 0; w < kT / 64; ++w) any |= s.redi[w];
  return any != 0;
}

template <int kT>
__device__ __forceinline__ double blk_min(double v, const S<kT> &s) {
  v = wave_min_dpp(v);
  if constexpr (kT == 64) return v;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.redv[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = s.redv[0];
  for (int w = 1; w < kT / 64; ++w) r = fmin(r, s.redv[w]);
  return r;
}

template <int kT>
__device__ __forceinline__ void blk_argmax(double &v, int &i, const S<kT> &s) {
  wave_argmax_idx(v, i);
  if constexpr (kT == 64) return;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    s.redv[threadIdx.x >> 6] = v;
    s.redi[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  v = s.redv[0];
  i = s.redi[0];
  for (int w = 1; w < kT / 64; ++w) amax_combine(v, i, s.redv[w], s.redi[w]);
}

// oracle col_dot: v' a_j over CSC column j in CSC order (v in LDS)
template <int kT>
__device__ __forceinline__ double col_dot(const S<kT> &s, const double *v, int j) {
  if (j >= s.n) return -v[j - s.n];
  double a = 0.0;
  for (int t = s.colptr[j]; t < s.colptr[j + 1]; ++t) a += s.cval[t] * v[s.rowidx[t]];
  return a;
}

// oracle place_nonbasic
template <int kT>
__device__ __forceinline__ void place_nonbasic(const S<kT> &s, int j, double ab) {
  const double lo = s.blo[j], hi = s.bhi[j], dj = s.d[j];
  const bool lo_f = lo > -kInfB, hi_f = hi < kInfB;
  if (lo_f && hi_f && lo == hi) {
    s.st[j] = ST_LB;
    s.z[j] = lo;
    return;
  }
  if (dj > kDTol) {
    if (!lo_f) {
      s.blo[j] = (hi < kInfB ? hi : 0.0) - ab;
      s.art[j] |= 1;
    }
    s.st[j] = ST_LB;
    s.z[j] = s.blo[j];
  } else if (dj < -kDTol) {
    if (!hi_f) {
      s.bhi[j] = (lo > -kInfB ? lo : 0.0) + ab;
      s.art[j] |= 2;
    }
    s.st[j] = ST_UB;
    s.z[j] = s.bhi[j];
  } else if (lo_f) {
    s.st[j] = ST_LB;
    s.z[j] = lo;
  } else if (hi_f) {
    s.st[j] = ST_UB;
    s.z[j] = hi;
  } else {
    s.st[j] = ST_FREE;
    s.z[j] = 0.0;
  }
}

// oracle grow_art
template <int kT>
__device__ __forceinline__ void grow_art(const S<kT> &s, double ab) {
  for (int j = threadIdx.x; j < s.N; j += kT) {
    const int8_t a = s.art[j];
    if (!a || s.st[j] == ST_BASIC) continue;
    const double tl = s.tlo(j), th = s.thi(j);
    if (a & 1) s.blo[j] = (th < kInfB ? th : 0.0) - ab;
    if (a & 2) s.bhi[j] = (tl > -kInfB ? tl : 0.0) + ab;
    if (s.st[j] == ST_LB) s.z[j] = s.blo[j];
    if (s.st[j] == ST_UB) s.z[j] = s.bhi[j];
  }
}

// oracle compute_primals: w = N z_N per row (CSR row k in column order, the
// logical last), then z_B = -B^{-1} w with k ascending.
template <int kT>
__device__ __forceinline__ void compute_primals(const S<kT> &s) {
  __syncthreads();
  for (int k = threadIdx.x; k < s.m; k += kT) {
    double w = 0.0;
    for (int t = s.rowptr[k]; t < s.rowptr[k + 1]; ++t) {
      const int j = s.ccol[t];
      if (s.st[j] == ST_BASIC) continue;
      const double zj = s.z[j];
      if (zj == 0.0) continue;
      w += s.rval[t] * zj;
    }
    const int jl = s.n + k;
    if (s.st[jl] != ST_BASIC) {
      const double zl = s.z[jl];
      if (zl != 0.0) w -= zl;
    }
    s.w[k] = w;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < s.m; i += kT) {
    double acc = 0.0;
    const double *col = s.Bi + i;
    int k0 = 0;
    for (; k0 + 8 <= s.m; k0 += 8) {  // loads first, adds in k order
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = col[(size_t)(k0 + u) * s.m];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u] * s.w[k0 + u];
    }
    for (; k0 < s.m; ++k0) acc += col[(size_t)k0 * s.m] * s.w[k0];
    s.z[s.head[i]] = -acc;
  }
  __syncthreads();
}

// Per-node refactorisation of a warm basis for the node's own matrix (the
// glob path with m > 64; K3R's job for m <= 64): oracle/lp_dual.c
// invert_basis -- Gauss-Jordan on [B | I] with partial pivoting (first row
// of largest |pivot| at or below the diagonal; |pivot| < 1e-12 = singular),
// the same element operations -- with B in this workgroup's HBM slot and I
// becoming B^-1 in the inverse slot, both column-major (thread r owns rows
// r, r + kT, ...).  Returns false when singular (the caller takes the slack
// basis, as the oracle does).
template <int kT>
__device__ bool refactor_basis(S<kT> &s, double *Bm) {
  const int n = s.n, m = s.m, tid = threadIdx.x;
  const size_t mm = (size_t)m * m;
  for (size_t e = tid; e < mm; e += kT) {
    Bm[e] = 0.0;
    s.Bi[e] = (e / m) == (e % m) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int i = tid; i < m; i += kT) {   // column i of B = the column of head[i]
    const int h = s.head[i];
    if (h >= n) {
      Bm[(size_t)i * m + (h - n)] = -1.0;
    } else {
      for (int t = s.colptr[h]; t < s.colptr[h + 1]; ++t)
        Bm[(size_t)i * m + s.rowidx[t]] = s.cval[t];
    }
  }
  __syncthreads();
  for (int c = 0; c < m; ++c) {
    double bv = -1.0;
    int br = INT_MAX;
    for (int r = c + tid; r < m; r += kT) {
      const double a = fabs(Bm[(size_t)c * m + r]);
      if (a > bv) {
        bv = a;
        br = r;
      }
    }
    blk_argmax(bv, br, s);
    if (!(bv >= 1e-12)) return false;
    if (br != c) {
      for (int k = tid; k < m; k += kT) {
        const size_t o = (size_t)k * m;
        double t = Bm[o + c];
        Bm[o + c] = Bm[o + br];
        Bm[o + br] = t;
        t = s.Bi[o + c];
        s.Bi[o + c] = s.Bi[o + br];
        s.Bi[o + br] = t;
      }
      __syncthreads();
    }
    const double inv = 1.0 / Bm[(size_t)c * m + c];
    __syncthreads();
    for (int k = tid; k < m; k += kT) {
      Bm[(size_t)k * m + c] *= inv;
      s.Bi[(size_t)k * m + c] *= inv;
    }
    __syncthreads();
    for (int r = tid; r < m; r += kT) {
      if (r == c) continue;
      const double f = Bm[(size_t)c * m + r];
      if (f == 0.0) continue;
      for (int k = 0; k < m; ++k) {
        const size_t o = (size_t)k * m;
        Bm[o + r] -= f * Bm[o + c];
        s.Bi[o + r] -= f * s.Bi[o + c];
      }
    }
    __syncthreads();
  }
  return true;
}

// K3R's column replacement for m > 64 (oracle colrep_refactor): from the
// root inverse, each basic structural column the node's rows changed is
// swapped in by one product-form update (alpha = B^-1 a' in CSC order, row
// i / alpha_i, row r -= alpha_r row i), B^-1 column-major in the inverse
// slot.  Returns false when a pivot is below 1e-12 (the caller refactors
// from scratch).
template <int kT>
__device__ bool colrep_basis(S<kT> &s, const double *cval0, const double *binv0) {
  const int n = s.n, m = s.m, tid = threadIdx.x;
  const size_t mm = (size_t)m * m;
  for (size_t e = tid; e < mm; e += kT) s.Bi[e] = binv0[e];
  __syncthreads();
  for (int i = 0; i < m; ++i) {
    const int h = s.head[i];
    if (h >= n) continue;
    bool ch = false;
    for (int t = s.colptr[h] + tid; t < s.colptr[h + 1]; t += kT) ch |= s.cval[t] != cval0[t];
    if (!blk_any(ch, s)) continue;
    for (int r = tid; r < m; r += kT) {
      double al = 0.0;
      for (int t = s.colptr[h]; t < s.colptr[h + 1]; ++t)
        al += s.Bi[(size_t)s.rowidx[t] * m + r] * s.cval[t];
      s.aq[r] = al;
    }
    __syncthreads();
    const double piv = s.aq[i];
    if (fabs(piv) < 1e-12) return false;
    const double inv = 1.0 / piv;
    for (int k = tid; k < m; k += kT) s.Bi[(size_t)k * m + i] *= inv;
    __syncthreads();
    for (int r = tid; r < m; r += kT) {
      if (r == i) continue;
      const double f = s.aq[r];
      if (f == 0.0) continue;
      for (int k = 0; k < m; ++k) s.Bi[(size_t)k * m + r] -= f * s.Bi[(size_t)k * m + i];
    }
    __syncthreads();
  }
  return true;
}

template <int kT>
__global__ __launch_bounds__(kT) void lp_large_kernel(DevLP lp, LpIO io, double *binv_slots) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m, N = n + m;
  const int tid = threadIdx.x;
  S<kT> s;
  {
    unsigned char *p = smem;
    s.d = (double *)p;    p += al16((size_t)N * 8);
    s.z = (double *)p;    p += al16((size_t)N * 8);
    s.blo = (double *)p;  p += al16((size_t)N * 8);
    s.bhi = (double *)p;  p += al16((size_t)N * 8);
    s.al = (double *)p;   p += al16((size_t)N * 8);
    s.t2 = (double *)p;   p += al16((size_t)N * 8);
    s.st = (int8_t *)p;   p += al16((size_t)N);
    s.art = (int8_t *)p;  p += al16((size_t)N);
    s.rho = (double *)p;  p += al16((size_t)m * 8);
    s.aq = (double *)p;   p += al16((size_t)m * 8);
    s.w = (double *)p;    p += al16((size_t)m * 8);
    s.head = (int *)p;    p += al16((size_t)m * 4);
    s.redv = (double *)p; p += al16(4 * 8);
    s.redi = (int *)p;
  }
  s.Bi = binv_slots + (size_t)blockIdx.x * m * m;
  s.colptr = lp.colptr; s.rowidx = lp.rowidx; s.cval = lp.cval;
  s.rowptr = lp.rowptr; s.ccol = lp.ccol; s.rval = lp.rval;
  s.rlo = lp.rlo; s.rhi = lp.rhi; s.c = lp.objd;
  s.n = n; s.m = m; s.N = N;
  const size_t mm = (size_t)m * m;

  // node list (the product-form kernels' overflow re-solve, as K3's):
  // positions list_lo .. min(*node_count, list_hi) of node_list
  const int lo = io.node_list != nullptr ? io.list_lo : 0;
  int nsolve = io.batch;
  if (io.node_list != nullptr) {
    nsolve = *io.node_count;
    if (nsolve > io.list_hi) nsolve = io.list_hi;
  }
  // nodes from a device counter when the host gives one (dynamic schedule:
  // a workgroup that finishes early takes the next node), else a static stride
  __shared__ int s_next;
  for (int bi = lo + blockIdx.x;; bi += gridDim.x) {
    __syncthreads();  // the previous node's LDS state is dead
    if (io.next != nullptr) {
      if (tid == 0) s_next = atomicAdd(io.next, 1);
      __syncthreads();
      bi = lo + s_next;
    }
    if (bi >= nsolve) break;
    const int b = io.node_list != nullptr ? io.node_list[bi] : bi;
    // pivots already made by K3P / K3PW (continuation): counted by the
    // iteration limit, the Bland switch and the reported total
    const int ib = io.iter_base_list != nullptr ? io.iter_base_list[bi] : io.iter_base;
    s.nlb = io.lb + (size_t)b * io.box_stride;
    s.nub = io.ub + (size_t)b * io.box_stride;
    s.ocol = io.obj_col != nullptr ? io.obj_col[b] : -1;
    s.osign = io.obj_col != nullptr ? io.obj_sign[b] : 0.0;

    if (io.skip != nullptr && io.skip[b] != 0) {  // pruned by FBBT: not solved
      if (tid == 0) {
        io.status[b] = kUnknownStatus;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      continue;
    }
    const bool nrows = io.nr.vals != nullptr;
    double *wg = nrows ? io.nr.wg + (size_t)blockIdx.x * io.nr.wg_stride : nullptr;
    if (nrows) {
      // the node's matrix and row bounds (K3's per-node rows): the loaded
      // values, then its own entries (OsiLPEngine::changeConstraint of the
      // rewritten rows), in this workgroup's HBM slot
      const int nnz = lp.nnz;
      double *wc = wg, *wr = wc + nnz, *wlo = wr + nnz, *whi = wlo + m;
      for (int t = tid; t < nnz; t += kT) {
        wc[t] = lp.cval[t];
        wr[t] = lp.rval[t];
      }
      for (int i = tid; i < m; i += kT) {
        wlo[i] = lp.rlo[i];
        whi[i] = lp.rhi[i];
      }
      __syncthreads();
      const double *rec = io.nr.vals + (size_t)b * io.nr.stride;
      for (int q = tid; q < io.nr.ncoef; q += kT) {
        double v = rec[io.nr.coef_src[q]];
        if (fabs(v) <= kLfTol) v = 0.0;
        wc[io.nr.csc_pos[q]] = v;
        wr[io.nr.csr_pos[q]] = v;
      }
      for (int q = tid; q < io.nr.nrow; q += kT) {
        const int r = io.nr.row[q];
        if (io.nr.lo_src[q] >= 0) wlo[r] = rec[io.nr.lo_src[q]];
        if (io.nr.hi_src[q] >= 0) whi[r] = rec[io.nr.hi_src[q]];
      }
      __syncthreads();
      s.cval = wc;
      s.rval = wr;
      s.rlo = wlo;
      s.rhi = whi;
    }
    // ---- working bounds; an empty box is infeasible before any pivot ----
    bool bad = false;
    for (int j = tid; j < N; j += kT) {
      s.blo[j] = s.tlo(j);
      s.bhi[j] = s.thi(j);
      s.art[j] = 0;
      bad |= s.blo[j] > s.bhi[j] + kPTol;
    }
    if (blk_any(bad, s)) {
      if (tid == 0) {
        io.status[b] = 2;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      continue;
    }

    // ---- basis: warm start or slack basis (B = -I) ----
    bool warm = io.ws.head != nullptr;
    const size_t bw = io.ws_index != nullptr ? (size_t)io.ws_index[b]
                      : io.list_ws ? (size_t)bi : (size_t)b;
    if (warm) {
      const int32_t *wh = io.ws.head + bw * io.ws.s_head;
      const int8_t *wst = io.ws.st + bw * io.ws.s_st;
      for (int j = tid; j < N; j += kT) {
        const int8_t v = wst[j];
        s.st[j] = v == ST_BASIC ? ST_LB : v;
      }
      for (int i = tid; i < m; i += kT) s.head[i] = wh[i];
      if (io.ws.binv != nullptr) {
        const double *wb = io.ws.binv + bw * io.ws.s_binv;
        for (size_t e = tid; e < mm; e += kT) s.Bi[e] = wb[e];  // column-major both
      }
      __syncthreads();
      for (int i = tid; i < m; i += kT) s.st[s.head[i]] = ST_BASIC;
      __syncthreads();
      if (io.ws.binv == nullptr && nrows)
        warm = (io.nr.binv0 != nullptr && colrep_basis(s, lp.cval, io.nr.binv0)) ||
               refactor_basis(s, wg + 2 * (size_t)lp.nnz + 2 * (size_t)m);
    }
    if (warm) {
      if (s.ocol < 0 && io.ws.d != nullptr) {
        const double *wd = io.ws.d + bw * io.ws.s_d;
        for (int j = tid; j < N; j += kT) s.d[j] = s.st[j] == ST_BASIC ? 0.0 : wd[j];
      } else if (s.ocol < 0) {
        // no d with the warm start (objective changed since the basis was
        // saved): oracle compute_duals, y = c_B' B^-1 over the basic rows in
        // order (thread k owns y_k), d_j = c_j - y' a_j
        for (int k = tid; k < m; k += kT) {
          double y = 0.0;
          for (int i = 0; i < m; ++i) {
            const int hi = s.head[i];
            const double cb = hi < n ? s.c[hi] : 0.0;
            if (cb != 0.0) y += cb * s.Bi[(size_t)k * m + i];
          }
          s.rho[k] = y;
        }
        __syncthreads();
        for (int j = tid; j < N; j += kT)
          s.d[j] = s.st[j] == ST_BASIC ? 0.0 : (j < n ? s.c[j] : 0.0) - col_dot(s, s.rho, j);
      } else {
        // bound LP (oracle compute_duals): y = c_B' B^-1 = osign * row r of
        // B^-1 when ocol is basic in row r, else 0; d_j = c_j - y' a_j
        int rr = INT_MAX;
        for (int i = tid; i < m; i += kT)
          if (s.head[i] == s.ocol) rr = i;
        double one = rr != INT_MAX ? 1.0 : 0.0;
        blk_argmax(one, rr, s);
        for (int k = tid; k < m; k += kT)
          s.rho[k] = rr != INT_MAX ? 0.0 + s.osign * s.Bi[(size_t)k * m + rr] : 0.0;
        __syncthreads();
        for (int j = tid; j < N; j += kT)
          s.d[j] = s.st[j] == ST_BASIC ? 0.0 : s.cj(j) - col_dot(s, s.rho, j);
      }
    } else {
      for (int i = tid; i < m; i += kT) s.head[i] = n + i;
      for (int j = tid; j < N; j += kT) {
        s.st[j] = j >= n ? ST_BASIC : ST_LB;
        s.d[j] = j < n ? s.cj(j) : 0.0;  // y = 0 for the slack basis
      }
      for (int k = 0; k < m; ++k)
        for (int i = tid; i < m; i += kT) s.Bi[(size_t)k * m + i] = i == k ? -1.0 : 0.0;
    }
    __syncthreads();
    double art_bound = kArt0;
    for (int j = tid; j < N; j += kT) {
      if (s.st[j] == ST_BASIC) continue;
      const double lo = s.blo[j], hi = s.bhi[j], dj = s.d[j];
      bool keep = false;
      if (warm) {
        const int8_t v = s.st[j];
        if (v == ST_LB && lo > -kInfB && dj >= -kDTol) {
          s.z[j] = lo;
          keep = true;
        } else if (v == ST_UB && hi < kInfB && dj <= kDTol) {
          s.z[j] = hi;
          keep = true;
        } else if (lo == hi && lo > -kInfB) {
          s.st[j] = ST_LB;
          s.z[j] = lo;
          keep = true;
        }
      }
      if (!keep) place_nonbasic(s, j, art_bound);
    }
    compute_primals(s);

    int status = kUnknownStatus, iters = 0;
    bool fresh = true;
    for (;;) {
      // ---- pricing: most infeasible basic row, lowest row on ties; past
      // kStallPivots pivots (oracle STALL_PIVOTS) Bland's rule: the
      // infeasible row with the lowest basic column ----
      const bool bland = iters + ib >= kStallPivots;
      double best = 0.0, key = -INFINITY;
      int r = INT_MAX;
      for (int i = tid; i < m; i += kT) {
        const int h = s.head[i];
        const double v = s.z[h];
        double inf = 0.0;
        if (v < s.blo[h] - kPTol) inf = v - s.blo[h];
        else if (v > s.bhi[h] + kPTol) inf = v - s.bhi[h];
        if (bland) {
          if (inf != 0.0 && -(double)h > key) {
            key = -(double)h;
            r = i;
          }
        } else if (fabs(inf) > best) {
          best = fabs(inf);
          r = i;
        }
      }
      if (bland) {
        blk_argmax(key, r, s);
        best = key == -INFINITY ? 0.0 : 1.0;   // only "some row is infeasible" is used
      } else {
        blk_argmax(best, r, s);
      }
      if (best == 0.0) {
        if (!fresh) {
          compute_primals(s);
          fresh = true;
          continue;
        }
        bool grow = false;
        for (int j = tid; j < N; j += kT) {
          const int8_t a = s.art[j], v = s.st[j];
          if (v == ST_BASIC || !a) continue;
          if ((v == ST_LB && (a & 1)) || (v == ST_UB && (a & 2))) grow = true;
        }
        if (!blk_any(grow, s)) {
          status = 0;
          break;
        }
        if (art_bound >= 1e13) {
          status = 4;
          break;
        }
        art_bound *= 1e3;
        grow_art(s, art_bound);
        compute_primals(s);
        fresh = true;
        continue;
      }
      if (iters + ib >= io.iter_limit) {
        status = 6;
        break;
      }
      double delta;
      {
        const int h = s.head[r];
        const double v = s.z[h];
        delta = v < s.blo[h] - kPTol ? v - s.blo[h] : v - s.bhi[h];
      }
      // ---- row r of B^{-1} ----
      for (int k = tid; k < m; k += kT) s.rho[k] = s.Bi[(size_t)k * m + r];
      __syncthreads();
      const double sigma = delta > 0 ? 1.0 : -1.0;

      // ---- pivot row and Harris pass 1 (pass 2's ratio cached in t2) ----
      double tmax = INFINITY;
      for (int j = tid; j < N; j += kT) {
        const int8_t v = s.st[j];
        double a = 0.0, t2 = INFINITY;
        if (v != ST_BASIC && s.blo[j] != s.bhi[j]) {
          a = col_dot(s, s.rho, j);
          const double at = sigma * a, dj = s.d[j];
          if (v == ST_LB && at > kPivTol) {
            const double t = (fmax(dj, 0.0) + kDTol) / at;
            t2 = fmax(dj, 0.0) / at;
            if (t < tmax) tmax = t;
          } else if (v == ST_UB && at < -kPivTol) {
            const double t = (fmin(dj, 0.0) - kDTol) / at;
            t2 = fmin(dj, 0.0) / at;
            if (t < tmax) tmax = t;
          } else if (v == ST_FREE && fabs(at) > kPivTol) {
            const double t = kDTol / fabs(at);
            t2 = 0.0;
            if (t < tmax) tmax = t;
          }
        }
        s.al[j] = a;
        s.t2[j] = t2;
      }
      tmax = blk_min(tmax, s);
      if (tmax == INFINITY) {  // dual unbounded
        bool boxed = false;
        for (int j = tid; j < N; j += kT) boxed |= s.st[j] != ST_BASIC && s.art[j] != 0;
        if (!blk_any(boxed, s) || art_bound >= 1e13) {
          status = 2;
          break;
        }
        art_bound *= 1e3;
        grow_art(s, art_bound);
        compute_primals(s);
        fresh = true;
        continue;
      }
      // ---- Harris pass 2: largest |alpha| among ratios <= tmax ----
      double qa = 0.0;
      int q = INT_MAX;
      if (!bland) {
        for (int j = tid; j < N; j += kT) {
          if (s.t2[j] <= tmax) {
            const double fa = fabs(s.al[j]);
            if (fa > qa) {
              qa = fa;
              q = j;
            }
          }
        }
        blk_argmax(qa, q, s);
      } else {  // Bland: the exact minimum ratio, lowest column on ties
        double key = -INFINITY;
        for (int j = tid; j < N; j += kT) {
          const double t2 = s.t2[j];
          if (t2 != INFINITY && -t2 > key) {
            key = -t2;
            q = j;
          }
        }
        blk_argmax(key, q, s);
        qa = q != INT_MAX ? fabs(s.al[q]) : 0.0;
      }
      if (qa == 0.0) {
        status = 2;
        break;
      }
      // ---- column q: alpha_q = B^{-1} a_q (oracle ftran_col order) ----
      for (int i = tid; i < m; i += kT) {
        double v;
        if (q < n) {
          v = 0.0;
          for (int t = s.colptr[q]; t < s.colptr[q + 1]; ++t)
            v += s.Bi[(size_t)s.rowidx[t] * m + i] * s.cval[t];
        } else {
          v = -s.Bi[(size_t)(q - n) * m + i];
        }
        s.aq[i] = v;
      }
      __syncthreads();
      const double arq = s.aq[r];
      double theta_d = s.d[q] / s.al[q];
      if (sigma * theta_d < 0) theta_d = 0.0;
      const double theta_p = delta / arq;
      const int pl = s.head[r];
      for (int j = tid; j < N; j += kT)
        if (s.st[j] != ST_BASIC) s.d[j] -= theta_d * s.al[j];
      for (int i = tid; i < m; i += kT) s.z[s.head[i]] -= theta_p * s.aq[i];
      const double inv = 1.0 / arq;
      for (int k = tid; k < m; k += kT) s.rho[k] *= inv;  // row r of the new B^{-1}
      __syncthreads();
      if (tid == 0) {
        const double zq = s.z[q] + theta_p;
        s.d[q] = 0.0;
        s.d[pl] = -theta_d;
        if (delta < 0) {
          s.st[pl] = ST_LB;
          s.z[pl] = s.blo[pl];
        } else {
          s.st[pl] = ST_UB;
          s.z[pl] = s.bhi[pl];
        }
        s.head[r] = q;
        s.st[q] = ST_BASIC;
        s.z[q] = zq;
        if (s.art[q]) {  // basic columns keep their true (infinite) bounds
          s.blo[q] = s.tlo(q);
          s.bhi[q] = s.thi(q);
          s.art[q] = 0;
        }
      }
      // ---- rank-1 update of B^{-1} (HBM): rows with alpha_iq = 0 untouched
      // (8 independent loads in flight per thread, then the 8 stores: the
      // column walk is a chain of HBM round trips otherwise)
      for (int i = tid; i < m; i += kT) {
        const double f = s.aq[i];
        double *col = s.Bi + i;
        if (i == r) {
          for (int k = 0; k < m; ++k) col[(size_t)k * m] = s.rho[k];
        } else if (f != 0.0) {
          int k0 = 0;
          for (; k0 + 8 <= m; k0 += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = col[(size_t)(k0 + u) * m];
#pragma unroll
            for (int u = 0; u < 8; ++u) col[(size_t)(k0 + u) * m] = v[u] - f * s.rho[k0 + u];
          }
          for (; k0 < m; ++k0) col[(size_t)k0 * m] -= f * s.rho[k0];
        }
      }
      __syncthreads();
      ++iters;
      fresh = false;
      if (iters % 64 == 0) {
        compute_primals(s);
        fresh = true;
      }
    }

    // ---- outputs ----
    __syncthreads();
    if (status == 0 || status == 6) {
      if (tid == 0) {
        double obj = 0.0;  // oracle order: sequential over the structurals
        for (int j = 0; j < n; ++j) obj += s.cj(j) * s.z[j];
        io.obj[b] = s.ocol < 0 ? obj + lp.objoff : obj;
      }
      if (io.x != nullptr)
        for (int j = tid; j < n; j += kT) io.x[(size_t)b * n + j] = s.z[j];
      if (io.rc != nullptr)
        for (int j = tid; j < N; j += kT)
          io.rc[(size_t)b * N + j] = s.st[j] == ST_BASIC ? 0.0 : s.d[j];
      if (io.wo_head != nullptr) {
        const size_t bo = io.wo_index != nullptr ? (size_t)io.wo_index[b] : (size_t)b;
        for (int i = tid; i < m; i += kT) io.wo_head[bo * m + i] = s.head[i];
        for (int j = tid; j < N; j += kT) {
          io.wo_st[bo * N + j] = s.st[j];
          io.wo_d[bo * N + j] = s.d[j];
        }
        double *dst = io.wo_binv + bo * mm;
        for (size_t e = tid; e < mm; e += kT) dst[e] = s.Bi[e];
      }
    } else if (tid == 0) {
      io.obj[b] = status == 2 ? INFINITY : -INFINITY;
    }
    if (tid == 0) {
      io.status[b] = status;
      io.iters[b] = iters + ib;
    }
  }
}

}  // namespace

size_t lp_large_lds_bytes(int n, int m) { return large_lds_bytes(n, m); }

// Workgroup size: one wave per node up to m = 256 rows (wave-level
// reductions, no cross-wave barriers, many nodes in flight per CU); four
// waves per node beyond, where the per-pivot sweeps over m rows dominate.
int lp_large_threads(int m) { return m <= 256 ? 64 : 256; }

int lp_large_grid(int batch, int n, int m, int num_cus) {
  const size_t lds = large_lds_bytes(n, m);
  const int waves = lp_large_threads(m) / 64;
  int per_cu = (int)((160 * 1024) / (lds > 0 ? lds : 1));
  const int cap = 16 / waves;  // 16 waves per CU
  if (per_cu > cap) per_cu = cap;
  if (per_cu < 1) per_cu = 1;
  const int g = per_cu * num_cus;
  return batch < g ? batch : g;
}

hipError_t lp_large_prepare() {
  static bool attr_set = false;  // dynamic LDS above 64 KiB must be opted in
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)lp_large_kernel<64>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLargeLdsMax);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void *)lp_large_kernel<256>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLargeLdsMax);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  return hipSuccess;
}

hipError_t launch_lp_large(const DevLP &lp, const LpIO &io, double *binv_slots, int grid,
                           hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  const size_t lds = large_lds_bytes(lp.n, lp.m);
  if (lds > (size_t)kLargeLdsMax || grid <= 0 || binv_slots == nullptr) return hipErrorInvalidValue;
  if (lp_large_threads(lp.m) == 64)
    hipLaunchKernelGGL(lp_large_kernel<64>, dim3(grid), dim3(64), lds, stream, lp, io,
                       binv_slots);
  else
    hipLaunchKernelGGL(lp_large_kernel<256>, dim3(grid), dim3(256), lds, stream, lp, io,
                       binv_slots);
  return hipGetLastError();
}

}  // namespace mgpu
