// K3P — batched bounded dual simplex in product form, gfx950.
//
// Same solve as K3 (repo:minotaur_amd/csrc/lp_dual.hip; OsiLPEngine::solve ->
// Clp resolve(), src/interfaces/OsiLPEngine.cpp:571-652) for the case the
// B&B hot path actually runs: every node of a batch warm-starts from ONE
// basis (the root optimum / the parent of a strong-branching batch), so the
// starting inverse B0^{-1} is the same for all of them and only the few
// pivots each node makes (5.9 on average for tls4-lin, 99.9 % <= 24) differ.
//
// MI355X-first mapping:
//  * B0^{-1} is staged ONCE per workgroup in LDS, in both layouts (column
//    major for B^{-1} a_q, row major for rho' = u' B0^{-1}); a node's own
//    inverse is B^{-1} = E_{k-1} ... E_0 B0^{-1}: k eta columns in VGPRs
//    (lane i holds eta_t[i]; at most kPfiMax of them).  The dense inverse of
//    K3 (128 VGPRs per node, 60 FMAs per lane per pivot to update) is gone,
//    which takes the kernel from 2 to 4 waves per SIMD.
//  * Column state (reduced costs, values, working bounds, status, pivot row,
//    Harris ratios) lives in VGPRs too: column j = s*64 + lane is slot s of
//    that lane (S slots, N = n + m <= 64*S).  Only the broadcast vectors (rho,
//    the nonbasic values for the primal recompute) go through LDS.
//  * BTRAN visits only the nonzeros of u (a ballot mask, ascending rows) with
//    v_readlane broadcasts; FTRAN reads the CSC column of a_q from LDS and
//    applies the etas lane-parallel.
//  * A node that would need more than kmax pivots stops and is appended to an
//    overflow list; the dense K3 then re-solves exactly those nodes from the
//    same warm start (launch_lp_dual with a node list, same stream).
//
// Arithmetic: oracle/lp_dual.c in product-form mode (dual_simplex_impl with
// pfi > 0: pfi_btran, ftran_col, pfi_apply_etas, compute_primals), loop for
// loop, so the GPU follows the oracle pivot for pivot (tests/test_lp_pfi_gpu.py).
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {

#ifdef MGPU_STAMPS
// Diagnostic build only (-DMGPU_STAMPS, tools/lp_stamps.py --pfi): s_memtime
// cycles per section summed over all waves; never compiled into the product.
__device__ unsigned long long g_pfi_stamps[16];
#define PSTAMP_DECL unsigned long long st_acc[10] = {0}, st_t = __builtin_amdgcn_s_memtime();
#define PSTAMP(i)                                             \
  do {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t_ - st_t;                                   \
    st_t = t_;                                                \
  } while (0)
#define PSTAMP_FLUSH                                           \
  if ((threadIdx.x & 63) == 0)                                \
    for (int i_ = 0; i_ < 10; ++i_) atomicAdd(&g_pfi_stamps[i_], st_acc[i_]);
#else
#define PSTAMP_DECL
#define PSTAMP(i) \
  do {            \
  } while (0)
#define PSTAMP_FLUSH
#endif

namespace {

constexpr double kPTol = 1e-7;
constexpr double kDTol = 1e-7;
constexpr double kPivTol = 1e-9;
constexpr double kArt0 = 1e7;
constexpr double kInfB = 1e30;
constexpr int kUnknownStatus = 12;
constexpr int kWaves = 12;  // one 768-thread workgroup per CU: 3 waves per SIMD (<= 168 VGPRs)

enum : int { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };

static_assert(kPfiMax < 64, "K3P never reaches K3's 64-pivot primal refresh");

__host__ __device__ constexpr size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

// matrix (CSC + CSR), B0^{-1} both ways, warm-start d / status / head
__host__ __device__ inline size_t pfi_shared_bytes(int n, int m, int nnz) {
  const int N = n + m;
  return al16((size_t)(n + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)(m + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         2 * al16((size_t)m * m * 8) + al16((size_t)N * 8) + al16((size_t)N * 4) +
         al16((size_t)m * 4);
}
// per wave: rho [64] + two column vectors [N] (values; basic-row bounds)
__host__ __device__ inline size_t pfi_wave_bytes(int N) { return 64 * 8 + 2 * al16((size_t)N * 8); }

__device__ __forceinline__ double art_lo(double thi, double ab) {
  return (thi < kInfB ? thi : 0.0) - ab;
}
__device__ __forceinline__ double art_hi(double tlo, double ab) {
  return (tlo > -kInfB ? tlo : 0.0) + ab;
}

// value of column j (wave-uniform j) held in slot j>>6 of lane j&63
template <int S>
__device__ __forceinline__ double colget(const double (&a)[S], int j) {
  const int s = j >> 6;
  double v = a[0];
#pragma unroll
  for (int t = 1; t < S; ++t)
    if (s == t) v = a[t];
  return rld(v, j & 63);
}
template <int S>
__device__ __forceinline__ int colget(const int (&a)[S], int j) {
  const int s = j >> 6;
  int v = a[0];
#pragma unroll
  for (int t = 1; t < S; ++t)
    if (s == t) v = a[t];
  return rl(v, j & 63);
}
template <int S, class T>
__device__ __forceinline__ void colset(T (&a)[S], int j, T v, int lane) {
#pragma unroll
  for (int t = 0; t < S; ++t)
    if (t == (j >> 6) && lane == (j & 63)) a[t] = v;
}

struct Prob {
  const int *colptr, *rowidx, *rowptr, *ccol;
  const double *cval, *rval;
  const double *b0c, *b0r;  // B0^{-1}: b0c[k*m + i] = b0r[i*m + k] = (B0^{-1})_{ik}
  int n, m, N;
  const double *nlb, *nub, *rlo, *rhi, *c;
  int ocol;
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
  // rho' a_j over CSC column j (K3's col_dot: four loads in flight, the
  // adds in CSC order)
  __device__ __forceinline__ double col_dot(const double *rho, int j) const {
    double a = 0.0;
    int t = colptr[j];
    const int e = colptr[j + 1];
    for (; t + 4 <= e; t += 4) {
      const int i0 = rowidx[t], i1 = rowidx[t + 1], i2 = rowidx[t + 2], i3 = rowidx[t + 3];
      const double v0 = cval[t], v1 = cval[t + 1], v2 = cval[t + 2], v3 = cval[t + 3];
      const double r0 = rho[i0], r1 = rho[i1], r2 = rho[i2], r3 = rho[i3];
      a += v0 * r0;
      a += v1 * r1;
      a += v2 * r2;
      a += v3 * r3;
    }
    for (; t < e; ++t) a += cval[t] * rho[rowidx[t]];
    return a;
  }
};

// v <- E_{k-1} ... E_0 v (oracle pfi_apply_etas); lanes >= m hold eta 0
// (pivot row of eta t = lane t of prow)
__device__ __forceinline__ double apply_etas(double v, const double (&eta)[kPfiMax], int prow,
                                             int k, int lane) {
#pragma unroll
  for (int t = 0; t < kPfiMax; ++t) {
    if (t < k) {
      const int p = rl(prow, t);
      const double vp = rld(v, p);
      if (vp != 0.0) v = lane == p ? eta[t] * vp : v + eta[t] * vp;
    }
  }
  return v;
}

template <int S>
__global__ __launch_bounds__(64 * kWaves) void lp_pfi_kernel(DevLP lp, LpIO io, PfiIO px) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m, N = n + m, nnz = lp.nnz;
  const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kmax = px.kmax;

  // ---- stage the matrix, B0^{-1} (both layouts) and the warm start once ----
  unsigned char *p = smem;
  int *s_colptr = (int *)p;      p += al16((size_t)(n + 1) * 4);
  int *s_rowidx = (int *)p;      p += al16((size_t)nnz * 4);
  double *s_cval = (double *)p;  p += al16((size_t)nnz * 8);
  int *s_rowptr = (int *)p;      p += al16((size_t)(m + 1) * 4);
  int *s_ccol = (int *)p;        p += al16((size_t)nnz * 4);
  double *s_rval = (double *)p;  p += al16((size_t)nnz * 8);
  double *s_b0c = (double *)p;   p += al16((size_t)m * m * 8);
  double *s_b0r = (double *)p;   p += al16((size_t)m * m * 8);
  double *s_wd = (double *)p;    p += al16((size_t)N * 8);
  int *s_wst = (int *)p;         p += al16((size_t)N * 4);
  int *s_whead = (int *)p;       p += al16((size_t)m * 4);
  constexpr int T = 64 * kWaves;
  for (int t = threadIdx.x; t <= n; t += T) s_colptr[t] = lp.colptr[t];
  for (int t = threadIdx.x; t <= m; t += T) s_rowptr[t] = lp.rowptr[t];
  for (int t = threadIdx.x; t < nnz; t += T) {
    s_rowidx[t] = lp.rowidx[t];
    s_cval[t] = lp.cval[t];
    s_ccol[t] = lp.ccol[t];
    s_rval[t] = lp.rval[t];
  }
  for (int t = threadIdx.x; t < m * m; t += T) {
    const double v = io.ws.binv[t];  // column-major: t = k*m + i
    s_b0c[t] = v;
    s_b0r[(t % m) * m + t / m] = v;
  }
  for (int t = threadIdx.x; t < N; t += T) {
    s_wd[t] = io.ws.d != nullptr ? io.ws.d[t] : 0.0;  // bound LPs rebuild d
    const int8_t s = io.ws.st[t];
    s_wst[t] = s == ST_BASIC ? ST_LB : s;
  }
  for (int t = threadIdx.x; t < m; t += T) s_whead[t] = io.ws.head[t];
  __syncthreads();
  for (int t = threadIdx.x; t < m; t += T) s_wst[s_whead[t]] = ST_BASIC;  // basic = in head
  __syncthreads();

  Prob P;
  P.colptr = s_colptr; P.rowidx = s_rowidx; P.cval = s_cval;
  P.rowptr = s_rowptr; P.ccol = s_ccol; P.rval = s_rval;
  P.b0c = s_b0c; P.b0r = s_b0r;
  P.n = n; P.m = m; P.N = N;
  P.rlo = lp.rlo; P.rhi = lp.rhi; P.c = lp.objd;
  double *rho = (double *)(p + (size_t)wave * pfi_wave_bytes(N));
  double *zbuf = rho + 64;
  double *ybuf = zbuf + al16((size_t)N * 8) / 8;

  // persistent waves over nodes (no workgroup barrier below this point)
  PSTAMP_DECL
  for (int b = blockIdx.x * kWaves + wave; b < io.batch; b += gridDim.x * kWaves) {
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    P.nlb = io.lb + (size_t)b * io.box_stride;
    P.nub = io.ub + (size_t)b * io.box_stride;
    P.ocol = io.obj_col != nullptr ? io.obj_col[b] : -1;
    P.osign = io.obj_col != nullptr ? io.obj_sign[b] : 0.0;

    if (io.skip != nullptr && io.skip[b] != 0) {
      if (lane == 0) {
        io.status[b] = kUnknownStatus;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      PSTAMP(9);
      continue;
    }

    // ---- column slots: working bounds; an empty box is infeasible ----
    double d[S], z[S], blo[S], bhi[S], al[S], t2[S];
    int st[S], art[S];
    bool bad = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = s * 64 + lane;
      const bool valid = j < N;
      blo[s] = valid ? P.tlo(j) : 0.0;
      bhi[s] = valid ? P.thi(j) : 0.0;
      art[s] = 0;
      z[s] = 0.0;
      al[s] = 0.0;
      t2[s] = INFINITY;
      st[s] = valid ? s_wst[j] : ST_BASIC;  // slots past N act as basic: never touched
      bad |= valid && blo[s] > bhi[s] + kPTol;
    }
    if (__any(bad)) {
      if (lane == 0) {
        io.status[b] = 2;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      PSTAMP(9);
      continue;
    }

    // ---- basis rows: head, bounds (basic columns carry no artificial box;
    // read back through LDS, not a second HBM gather) ----
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = s * 64 + lane;
      if (j < N) {
        zbuf[j] = blo[s];
        ybuf[j] = bhi[s];
      }
    }
    wave_sync();
    int h = lane < m ? s_whead[lane] : -1;
    double lbB = 0.0, ubB = 0.0;
    if (lane < m) {
      lbB = zbuf[h];
      ubB = ybuf[h];
    }
    wave_sync();
    if (P.ocol < 0) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = (j < N && st[s] != ST_BASIC) ? s_wd[j] : 0.0;
      }
    } else {
      // bound LP (oracle compute_duals at B = B0): y = osign * row r of B0^{-1}
      // when ocol is basic in row r, else 0; d_j = c_j - y' a_j
      const uint64_t on = __ballot(lane < m && h == P.ocol);
      double y = 0.0;
      if (on != 0ull && lane < m) y = 0.0 + P.osign * s_b0r[(size_t)__builtin_ctzll(on) * m + lane];
      rho[lane] = y;
      wave_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = 0.0;
        if (j < N && st[s] != ST_BASIC)
          d[s] = P.cj(j) - (j >= n ? -rho[j - n] : P.col_dot(rho, j));
      }
      wave_sync();
    }

    // ---- nonbasic placement: keep the warm status when dual feasible ----
    double art_bound = kArt0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (st[s] == ST_BASIC) continue;
      const double lo = blo[s], hi = bhi[s], dj = d[s];
      const bool lo_f = lo > -kInfB, hi_f = hi < kInfB;
      if (st[s] == ST_LB && lo_f && dj >= -kDTol) {
        z[s] = lo;
      } else if (st[s] == ST_UB && hi_f && dj <= kDTol) {
        z[s] = hi;
      } else if (lo == hi && lo_f) {
        st[s] = ST_LB;
        z[s] = lo;
      } else if (dj > kDTol) {  // oracle place_nonbasic
        if (!lo_f) {
          blo[s] = art_lo(hi, art_bound);
          art[s] |= 1;
        }
        st[s] = ST_LB;
        z[s] = blo[s];
      } else if (dj < -kDTol) {
        if (!hi_f) {
          bhi[s] = art_hi(lo, art_bound);
          art[s] |= 2;
        }
        st[s] = ST_UB;
        z[s] = bhi[s];
      } else if (lo_f) {
        st[s] = ST_LB;
        z[s] = lo;
      } else if (hi_f) {
        st[s] = ST_UB;
        z[s] = hi;
      } else {
        st[s] = ST_FREE;
        z[s] = 0.0;
      }
    }

    double eta[kPfiMax];
#pragma unroll
    for (int t = 0; t < kPfiMax; ++t) eta[t] = 0.0;
    int prow = 0;  // lane t: pivot row of eta t
    int iters = 0;

    // oracle compute_primals (product form): z_B = -E...E B0^{-1} (N z_N)
    auto primals = [&]() -> double {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        if (j < N) zbuf[j] = st[s] == ST_BASIC ? 0.0 : z[s];
      }
      wave_sync();
      double w = 0.0;
      if (lane < m) {
        for (int t = P.rowptr[lane]; t < P.rowptr[lane + 1]; ++t) {
          const double zj = zbuf[P.ccol[t]];
          if (zj == 0.0) continue;
          w += P.rval[t] * zj;
        }
        const double zl = zbuf[n + lane];
        if (zl != 0.0) w -= zl;
      }
      wave_sync();
      double sacc = 0.0;
      const int li = lane < m ? lane : 0;
      int k = 0;
      for (; k + 4 <= m; k += 4) {  // four LDS loads in flight, adds in order
        const double b0 = P.b0c[(size_t)k * m + li], b1 = P.b0c[(size_t)(k + 1) * m + li];
        const double b2 = P.b0c[(size_t)(k + 2) * m + li], b3 = P.b0c[(size_t)(k + 3) * m + li];
        sacc += b0 * rld(w, k);
        sacc += b1 * rld(w, k + 1);
        sacc += b2 * rld(w, k + 2);
        sacc += b3 * rld(w, k + 3);
      }
      for (; k < m; ++k) sacc += P.b0c[(size_t)k * m + li] * rld(w, k);
      if (lane >= m) sacc = 0.0;
      sacc = apply_etas(sacc, eta, prow, iters, lane);
      return -sacc;
    };
    auto grow = [&](double ab) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        if (!art[s] || st[s] == ST_BASIC) continue;
        if (art[s] & 1) blo[s] = art_lo(P.thi(j), ab);
        if (art[s] & 2) bhi[s] = art_hi(P.tlo(j), ab);
        if (st[s] == ST_LB) z[s] = blo[s];
        if (st[s] == ST_UB) z[s] = bhi[s];
      }
    };

    PSTAMP(0);
    double zB = primals();
    PSTAMP(1);
    int status = kUnknownStatus;
    bool fresh = true;
    for (;;) {
      // ---- pricing: most infeasible basic row, lowest row on ties ----
      double inf = 0.0;
      if (lane < m) {
        if (zB < lbB - kPTol) inf = zB - lbB;
        else if (zB > ubB + kPTol) inf = zB - ubB;
      }
      double best = fabs(inf);
      int r = best > 0.0 ? lane : INT_MAX;
      wave_argmax_dpp(best, r);
      asm volatile("" : "+v"(best));
      PSTAMP(2);
      if (best == 0.0) {
        if (!fresh) {
          zB = primals();
          PSTAMP(1);
          fresh = true;
          continue;
        }
        bool g = false;
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (st[s] != ST_BASIC && art[s] &&
              ((st[s] == ST_LB && (art[s] & 1)) || (st[s] == ST_UB && (art[s] & 2))))
            g = true;
        if (!__any(g)) {
          status = 0;
          break;
        }
        if (art_bound >= 1e13) {
          status = 4;
          break;
        }
        art_bound *= 1e3;
        grow(art_bound);
        zB = primals();
        PSTAMP(1);
        fresh = true;
        continue;
      }
      if (iters >= io.iter_limit) {
        status = 6;
        break;
      }
      if (iters >= kmax) {  // eta file full: the dense K3 re-solves this node
        status = -1;
        break;
      }
      const double delta = rld(inf, r);
      const double sigma = delta > 0 ? 1.0 : -1.0;

      // ---- BTRAN: u = e_r' E_{k-1} ... E_0 over the nonzeros of u ----
      double u = lane == r ? 1.0 : 0.0;
#pragma unroll
      for (int t = kPfiMax - 1; t >= 0; --t) {
        if (t < iters) {
          uint64_t mask = __ballot(u != 0.0);
          double acc = 0.0;
          while (mask) {
            const int i = __builtin_ctzll(mask);
            mask &= mask - 1;
            acc += rld(u, i) * rld(eta[t], i);
          }
          if (lane == rl(prow, t)) u = acc;
        }
      }
      {  // rho' = u' B0^{-1} (ascending nonzero rows), published to LDS
        uint64_t mask = __ballot(u != 0.0);
        double rk = 0.0;
        const int lk = lane < m ? lane : 0;
        while (mask) {  // up to four rows per round: loads first, adds in order
          int ii[4];
          int c = 0;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            ii[t] = mask ? __builtin_ctzll(mask) : 0;
            c += mask ? 1 : 0;
            mask &= mask - 1;
          }
          double bv[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) bv[t] = P.b0r[(size_t)ii[t] * m + lk];
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < c) rk += rld(u, ii[t]) * bv[t];
        }
        rho[lane] = lane < m ? rk : 0.0;
      }
      wave_sync();
      PSTAMP(3);

      // ---- pivot row and Harris pass 1 (pass-2 ratio cached in t2) ----
      double tmax = INFINITY;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        double a = 0.0, tt = INFINITY;
        if (st[s] != ST_BASIC && blo[s] != bhi[s]) {
          a = j >= n ? -rho[j - n] : P.col_dot(rho, j);
          const double at = sigma * a, dj = d[s], fat = fabs(at);
          const bool lb = st[s] == ST_LB && at > kPivTol, ub = st[s] == ST_UB && at < -kPivTol,
                     fr = st[s] == ST_FREE && fat > kPivTol;
          const double n2 = lb ? fmax(dj, 0.0) : ub ? fmin(dj, 0.0) : 0.0;
          const double n1 = lb ? n2 + kDTol : ub ? n2 - kDTol : kDTol;
          const double den = fr ? fat : at;
          if (lb || ub || fr) {
            const double tr = n1 / den;
            tt = fr ? 0.0 : n2 / den;
            if (tr < tmax) tmax = tr;
          }
        }
        al[s] = a;
        t2[s] = tt;
      }
      tmax = wave_min_dpp(tmax);
      asm volatile("" : "+v"(tmax));
      PSTAMP(4);
      if (tmax == INFINITY) {  // dual unbounded
        bool boxed = false;
#pragma unroll
        for (int s = 0; s < S; ++s) boxed |= st[s] != ST_BASIC && art[s] != 0;
        if (!__any(boxed) || art_bound >= 1e13) {
          status = 2;
          break;
        }
        art_bound *= 1e3;
        grow(art_bound);
        zB = primals();
        fresh = true;
        continue;
      }
      // ---- Harris pass 2: largest |alpha| among ratios <= tmax ----
      double qa = 0.0;
      int q = INT_MAX;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (t2[s] <= tmax) {
          const double fa = fabs(al[s]);
          if (fa > qa) {
            qa = fa;
            q = s * 64 + lane;
          }
        }
      }
      wave_argmax_dpp(qa, q);
      PSTAMP(5);
      if (qa == 0.0) {
        status = 2;
        break;
      }

      // ---- FTRAN: alpha_q = E...E B0^{-1} a_q ----
      double alq = 0.0;
      {
        const int li = lane < m ? lane : 0;
        if (q < n) {
          for (int t = P.colptr[q]; t < P.colptr[q + 1]; ++t)
            alq += P.b0c[(size_t)P.rowidx[t] * m + li] * P.cval[t];
        } else {
          alq = -P.b0c[(size_t)(q - n) * m + li];
        }
        if (lane >= m) alq = 0.0;
      }
      alq = apply_etas(alq, eta, prow, iters, lane);
      const double arq = rld(alq, r);
      PSTAMP(6);

      // ---- steps ----
      double theta_d = colget(d, q) / colget(al, q);
      if (sigma * theta_d < 0) theta_d = 0.0;
      const double theta_p = delta / arq;
      const int pl = rl(h, r);
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (st[s] != ST_BASIC) d[s] -= theta_d * al[s];
      const double zq = colget(z, q) + theta_p;
      const int art_q = colget(art, q);
      double bloq = colget(blo, q), bhiq = colget(bhi, q);
      const double bound_p = delta < 0 ? colget(blo, pl) : colget(bhi, pl);
      colset(d, q, 0.0, lane);
      colset(d, pl, -theta_d, lane);
      colset(st, pl, delta < 0 ? (int)ST_LB : (int)ST_UB, lane);
      colset(z, pl, bound_p, lane);
      colset(st, q, (int)ST_BASIC, lane);
      colset(z, q, zq, lane);
      if (art_q) {  // basic columns keep their true (infinite) bounds
        bloq = P.tlo(q);
        bhiq = P.thi(q);
        colset(blo, q, bloq, lane);
        colset(bhi, q, bhiq, lane);
        colset(art, q, 0, lane);
      }
      if (lane < m) zB -= theta_p * alq;
      if (lane == r) {
        h = q;
        zB = zq;
        lbB = bloq;
        ubB = bhiq;
      }
      // ---- eta column of this pivot (oracle: -alpha_q/alpha_rq, 1/alpha_rq at r)
      const double inv = 1.0 / arq;
      const double e = lane == r ? inv : -alq * inv;
#pragma unroll
      for (int t = 0; t < kPfiMax; ++t)
        if (t == iters) eta[t] = e;
      if (lane == iters) prow = r;
      ++iters;
      fresh = false;
      PSTAMP(7);
    }

    // ---- outputs ----
    if (status == -1) {
      if (lane == 0) px.ovf_list[atomicAdd(px.ovf_count, 1)] = b;
      continue;
    }
    if (status == 0 || status == 6) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        if (j < N) zbuf[j] = z[s];
      }
      wave_sync();
      if (lane < m) zbuf[h] = zB;
      wave_sync();
      double sum = 0.0;
      for (int j = lane; j < n; j += 64) sum += P.cj(j) * zbuf[j];
      sum = wave_sum(sum);
      if (lane == 0) io.obj[b] = P.ocol < 0 ? sum + lp.objoff : sum;
      if (io.x != nullptr)
        for (int j = lane; j < n; j += 64) io.x[(size_t)b * n + j] = zbuf[j];
      wave_sync();
    } else if (lane == 0) {
      io.obj[b] = status == 2 ? INFINITY : -INFINITY;
    }
    if (lane == 0) {
      io.status[b] = status;
      io.iters[b] = iters;
    }
    PSTAMP(8);
  }
  PSTAMP_FLUSH
}

template <int S>
hipError_t launch_s(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                    hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)lp_pfi_kernel<S>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const size_t lds = lp_pfi_lds_bytes(lp.n, lp.m, lp.nnz);
  const int want = (io.batch + kWaves - 1) / kWaves;
  const int blocks = want < num_cus ? want : num_cus;
  hipLaunchKernelGGL((lp_pfi_kernel<S>), dim3(blocks), dim3(64 * kWaves), lds, stream, lp, io,
                     px);
  return hipGetLastError();
}

}  // namespace

#ifdef MGPU_STAMPS
extern "C" int mgpu_debug_pfi_stamps(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pfi_stamps), sizeof(unsigned long long) * 16) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pfi_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

size_t lp_pfi_lds_bytes(int n, int m, int nnz) {
  return pfi_shared_bytes(n, m, nnz) + (size_t)kWaves * pfi_wave_bytes(n + m);
}

bool lp_pfi_fits(int n, int m, int nnz) {
  return m <= kLpMaxM && n + m <= 64 * kPfiSlots && lp_pfi_lds_bytes(n, m, nnz) <= 160 * 1024;
}

hipError_t launch_lp_pfi(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                         hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  if (!lp_pfi_fits(lp.n, lp.m, lp.nnz) || io.ws.head == nullptr || px.kmax < 1 ||
      px.kmax > kPfiMax)
    return hipErrorInvalidValue;
  const int S = (lp.n + lp.m + 63) / 64;
  switch (S) {
    case 1: return launch_s<1>(lp, io, px, num_cus, stream);
    case 2: return launch_s<2>(lp, io, px, num_cus, stream);
    case 3: return launch_s<3>(lp, io, px, num_cus, stream);
    default: return launch_s<4>(lp, io, px, num_cus, stream);
  }
}

}  // namespace mgpu
