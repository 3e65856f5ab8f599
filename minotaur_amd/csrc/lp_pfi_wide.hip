// K3PW — the product-form dual simplex of K3P for relaxations with 64 < m
// <= 128 rows (two basis rows per lane), gfx950.
//
// Same solve and arithmetic as K3P (repo:minotaur_amd/csrc/lp_pfi.hip), i.e.
// oracle/lp_dual.c in product-form mode (dual_simplex_impl with pfi > 0:
// pfi_btran, ftran_col, pfi_apply_etas, compute_primals, loop for loop), the
// replacement of OsiLPEngine::solve -> Clp resolve()
// (src/interfaces/OsiLPEngine.cpp:571-652) for the batches that share one
// warm start: the root basis of the batched tree's node LPs, the relaxation
// basis of root OBBT.  The dense K3L it replaces for these batches copies
// the m x m warm-start inverse into an HBM slot for every LP and rewrites
// the rows of that copy on every pivot (16 m^2 bytes at most); here the
// starting inverse B0^{-1} is staged ONCE per workgroup in LDS and a node
// only keeps its eta columns.
//
// MI355X-first mapping:
//  * Basis row i = rs*64 + lane, rs < 2: every per-row quantity (basic
//    column, its bounds and value, u of BTRAN, alpha_q, the eta columns) is a
//    pair of registers per lane; a wave-uniform row p is broadcast from slot
//    p >> 6 with v_readlane.
//  * B0^{-1} column-major in LDS with the odd leading dimension m + 1 (both
//    column walks and row walks are bank-spread); 8 waves per workgroup, one
//    workgroup per CU (the inverse takes 76-103 KB for m = 97..113).
//  * Eta columns in VGPRs (kPfiWideMax of them, 2 registers pairs each): the
//    convex trees' node LPs from the root basis take 12-25 pivots (deeper
//    nodes more), so the file holds 32; a node that needs more stops and
//    writes its basis with the explicit inverse E...E B0^{-1} to a
//    continuation slot, and K3L continues exactly those nodes (node list,
//    same stream, no host sync).
//  * Column state (reduced cost, pivot-row entry, Harris ratio, status bits)
//    in VGPRs for column j = s*64 + lane (n + m <= 64*S), values and working
//    bounds in a per-wave LDS slice, as in K3P.
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

constexpr double kPTol = 1e-7;
constexpr double kDTol = 1e-7;
constexpr double kPivTol = 1e-9;
constexpr double kArt0 = 1e7;
constexpr double kInfB = 1e30;
constexpr int kUnknownStatus = 12;
constexpr int kR = 2;            // basis rows per lane
constexpr int kKE = kPfiWideMax; // eta file
constexpr int kWaves = 8;        // waves per workgroup (2 per SIMD)

static_assert(kKE < 64, "K3PW never reaches the dense 64-pivot primal refresh");

enum : int { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };
constexpr int kArtLo = 4, kArtHi = 8, kFixed = 16;

__host__ __device__ constexpr size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

__host__ __device__ inline size_t pfiw_shared_bytes(int n, int m, int nnz) {
  const int N = n + m;
  return al16((size_t)(n + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)(m + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)m * (m + 1) * 8) + al16((size_t)N * 8) + al16((size_t)N * 4) +
         al16((size_t)m * 4);
}
// per wave: rho [128] + column values, lower and upper working bounds [N]
__host__ __device__ inline size_t pfiw_wave_bytes(int N) {
  return 64 * kR * 8 + 3 * al16((size_t)N * 8);
}

__device__ __forceinline__ double art_lo(double thi, double ab) {
  return (thi < kInfB ? thi : 0.0) - ab;
}
__device__ __forceinline__ double art_hi(double tlo, double ab) {
  return (tlo > -kInfB ? tlo : 0.0) + ab;
}

// row p's value of a per-row register pair (p wave-uniform)
__device__ __forceinline__ double rrow(const double (&v)[kR], int p) {
  return rld(p < 64 ? v[0] : v[1], p & 63);
}
__device__ __forceinline__ int rrowi(const int (&v)[kR], int p) {
  return rl(p < 64 ? v[0] : v[1], p & 63);
}

struct Prob {
  const int *colptr, *rowidx, *rowptr, *ccol;
  const double *cval, *rval;
  const double *b0;  // (B0^{-1})_{ik} = b0[k*ld + i]
  int n, m, N, ld;
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
  // rho' a_j over CSC column j (four loads in flight, adds in CSC order)
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

// v <- E_{k-1} ... E_0 v (oracle pfi_apply_etas): out_p' = eta_p out_p,
// out_i' = out_i + eta_i out_p; rows >= m hold 0 in v and in every eta
__device__ __forceinline__ void apply_etas(double (&v)[kR], const double (&eta)[kKE][kR],
                                           int prow, int k, int lane) {
#pragma unroll
  for (int t = 0; t < kKE; ++t) {
    if (t < k) {
      const int p = rl(prow, t);
      const double vp = rrow(v, p);
      if (vp != 0.0) {
#pragma unroll
        for (int rs = 0; rs < kR; ++rs)
          v[rs] = rs * 64 + lane == p ? eta[t][rs] * vp : v[rs] + eta[t][rs] * vp;
      }
    }
  }
}

template <int S>
__global__ __launch_bounds__(64 * kWaves) void lp_pfiw_kernel(DevLP lp, LpIO io, PfiIO px) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m, N = n + m, nnz = lp.nnz, ld = m + 1;
  const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kmax = px.kmax;

  // ---- stage the matrix, B0^{-1} and the warm start once per workgroup ----
  unsigned char *p = smem;
  int *s_colptr = (int *)p;      p += al16((size_t)(n + 1) * 4);
  int *s_rowidx = (int *)p;      p += al16((size_t)nnz * 4);
  double *s_cval = (double *)p;  p += al16((size_t)nnz * 8);
  int *s_rowptr = (int *)p;      p += al16((size_t)(m + 1) * 4);
  int *s_ccol = (int *)p;        p += al16((size_t)nnz * 4);
  double *s_rval = (double *)p;  p += al16((size_t)nnz * 8);
  double *s_b0 = (double *)p;    p += al16((size_t)m * ld * 8);
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
  for (int t = threadIdx.x; t < m * m; t += T)  // ABI: column-major, t = k*m + i
    s_b0[(t / m) * ld + t % m] = io.ws.binv[t];
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
  P.b0 = s_b0;
  P.n = n; P.m = m; P.N = N; P.ld = ld;
  P.rlo = lp.rlo; P.rhi = lp.rhi; P.c = lp.objd;
  double *rho = (double *)(p + (size_t)wave * pfiw_wave_bytes(N));
  const size_t Np = al16((size_t)N * 8) / 8;
  double *zc = rho + 64 * kR;  // value of each nonbasic column, 0 for basic ones
  double *lo = zc + Np;        // working bounds (artificial where marked)
  double *hi = lo + Np;

  // persistent waves over nodes from a device counter (no workgroup barrier
  // below this point)
  for (;;) {
    int b = 0;
    if (lane0 == 0) b = atomicAdd(px.next, 1);
    b = __builtin_amdgcn_readfirstlane(b);
    if (b >= io.batch) break;
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
      continue;
    }

    // ---- working bounds; an empty box is infeasible before any pivot ----
    double tl[S], th[S];
    int sa[S];
    bool bad = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = s * 64 + lane;
      const bool valid = j < N;
      tl[s] = valid ? P.tlo(j) : 0.0;
      th[s] = valid ? P.thi(j) : 0.0;
      sa[s] = valid ? s_wst[j] : ST_BASIC;  // slots past N act as basic: never touched
      bad |= valid && tl[s] > th[s] + kPTol;
      if (valid) {
        lo[j] = tl[s];
        hi[j] = th[s];
      }
    }
    if (__any(bad)) {
      if (lane == 0) {
        io.status[b] = 2;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
      }
      continue;
    }
    wave_sync();

    // ---- basis rows: head and bounds (basic columns carry no artificial box)
    int h[kR];
    double lbB[kR], ubB[kR];
#pragma unroll
    for (int rs = 0; rs < kR; ++rs) {
      const int i = rs * 64 + lane;
      h[rs] = i < m ? s_whead[i] : -1;
      lbB[rs] = i < m ? lo[h[rs]] : 0.0;
      ubB[rs] = i < m ? hi[h[rs]] : 0.0;
    }
    double d[S];
    if (P.ocol < 0) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = (j < N && sa[s] != ST_BASIC) ? s_wd[j] : 0.0;
      }
    } else {
      // bound LP (oracle compute_duals at B = B0): y = osign * row r of B0^{-1}
      // when ocol is basic in row r, else 0; d_j = c_j - y' a_j
      int rb = -1;
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        const uint64_t on = __ballot(rs * 64 + lane < m && h[rs] == P.ocol);
        if (rb < 0 && on != 0ull) rb = rs * 64 + (int)__builtin_ctzll(on);
      }
#pragma unroll
      for (int ks = 0; ks < kR; ++ks) {
        const int k = ks * 64 + lane;
        double y = 0.0;
        if (rb >= 0 && k < m) y = 0.0 + P.osign * P.b0[(size_t)k * ld + rb];
        rho[k] = y;
      }
      wave_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = 0.0;
        if (j < N && sa[s] != ST_BASIC)
          d[s] = P.cj(j) - (j >= n ? -rho[j - n] : P.col_dot(rho, j));
      }
      wave_sync();
    }

    // ---- nonbasic placement: keep the warm status when dual feasible ----
    double art_bound = kArt0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = s * 64 + lane;
      if (j >= N) continue;
      if (sa[s] == ST_BASIC) {  // the fixed bit matters once it leaves the basis
        zc[j] = 0.0;
        sa[s] = ST_BASIC | (tl[s] == th[s] ? kFixed : 0);
        continue;
      }
      double lo_j = tl[s], hi_j = th[s], z;
      const double dj = d[s];
      const bool lo_f = lo_j > -kInfB, hi_f = hi_j < kInfB;
      int st = sa[s], art = 0;
      if (st == ST_LB && lo_f && dj >= -kDTol) {
        z = lo_j;
      } else if (st == ST_UB && hi_f && dj <= kDTol) {
        z = hi_j;
      } else if (lo_j == hi_j && lo_f) {
        st = ST_LB;
        z = lo_j;
      } else if (dj > kDTol) {  // oracle place_nonbasic
        if (!lo_f) {
          lo_j = art_lo(hi_j, art_bound);
          lo[j] = lo_j;
          art = kArtLo;
        }
        st = ST_LB;
        z = lo_j;
      } else if (dj < -kDTol) {
        if (!hi_f) {
          hi_j = art_hi(lo_j, art_bound);
          hi[j] = hi_j;
          art = kArtHi;
        }
        st = ST_UB;
        z = hi_j;
      } else if (lo_f) {
        st = ST_LB;
        z = lo_j;
      } else if (hi_f) {
        st = ST_UB;
        z = hi_j;
      } else {
        st = ST_FREE;
        z = 0.0;
      }
      zc[j] = z;
      sa[s] = st | art | (lo_j == hi_j ? kFixed : 0);
    }

    double eta[kKE][kR];
#pragma unroll
    for (int t = 0; t < kKE; ++t)
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) eta[t][rs] = 0.0;
    int prow = 0;  // lane t: pivot row of eta t
    int iters = 0;
    double zB[kR];

    // oracle compute_primals (product form): z_B = -E...E B0^{-1} (N z_N)
    auto primals = [&]() {
      wave_sync();
      double w[kR];
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        const int k = rs * 64 + lane;
        double acc = 0.0;
        if (k < m) {
          for (int t = P.rowptr[k]; t < P.rowptr[k + 1]; ++t) {
            const double zj = zc[P.ccol[t]];
            if (zj == 0.0) continue;
            acc += P.rval[t] * zj;
          }
          const double zl = zc[n + k];
          if (zl != 0.0) acc -= zl;
        }
        w[rs] = acc;
      }
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        const int i = rs * 64 + lane;
        const int li = i < m ? i : 0;
        double sacc = 0.0;
        int k = 0;
        const int k1 = m < 64 ? m : 64;
        for (; k + 4 <= k1; k += 4) {  // four LDS loads in flight, adds in order
          const double b0 = P.b0[(size_t)k * ld + li], b1 = P.b0[(size_t)(k + 1) * ld + li];
          const double b2 = P.b0[(size_t)(k + 2) * ld + li], b3 = P.b0[(size_t)(k + 3) * ld + li];
          sacc += b0 * rld(w[0], k);
          sacc += b1 * rld(w[0], k + 1);
          sacc += b2 * rld(w[0], k + 2);
          sacc += b3 * rld(w[0], k + 3);
        }
        for (; k < k1; ++k) sacc += P.b0[(size_t)k * ld + li] * rld(w[0], k);
        for (; k + 4 <= m; k += 4) {
          const double b0 = P.b0[(size_t)k * ld + li], b1 = P.b0[(size_t)(k + 1) * ld + li];
          const double b2 = P.b0[(size_t)(k + 2) * ld + li], b3 = P.b0[(size_t)(k + 3) * ld + li];
          sacc += b0 * rld(w[1], k - 64);
          sacc += b1 * rld(w[1], k - 63);
          sacc += b2 * rld(w[1], k - 62);
          sacc += b3 * rld(w[1], k - 61);
        }
        for (; k < m; ++k) sacc += P.b0[(size_t)k * ld + li] * rld(w[1], k - 64);
        zB[rs] = i < m ? sacc : 0.0;
      }
      apply_etas(zB, eta, prow, iters, lane);
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) zB[rs] = -zB[rs];
    };
    // oracle grow_art
    auto grow = [&](double ab) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        const int st = sa[s] & 3;
        if (!(sa[s] & (kArtLo | kArtHi)) || st == ST_BASIC) continue;
        double lo_j = lo[j], hi_j = hi[j];
        if (sa[s] & kArtLo) lo_j = lo[j] = art_lo(P.thi(j), ab);
        if (sa[s] & kArtHi) hi_j = hi[j] = art_hi(P.tlo(j), ab);
        if (st == ST_LB) zc[j] = lo_j;
        if (st == ST_UB) zc[j] = hi_j;
        sa[s] = (sa[s] & ~kFixed) | (lo_j == hi_j ? kFixed : 0);
      }
    };

    primals();
    int status = kUnknownStatus;
    for (;;) {
      // ---- pricing: most infeasible basic row, lowest row on ties ----
      double inf[kR];
      double best = 0.0;
      int r = INT_MAX;
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        inf[rs] = 0.0;
        if (rs * 64 + lane < m) {
          if (zB[rs] < lbB[rs] - kPTol) inf[rs] = zB[rs] - lbB[rs];
          else if (zB[rs] > ubB[rs] + kPTol) inf[rs] = zB[rs] - ubB[rs];
        }
        if (fabs(inf[rs]) > best) {
          best = fabs(inf[rs]);
          r = rs * 64 + lane;
        }
      }
      wave_argmax_idx(best, r);  // r used only when best > 0
      asm volatile("" : "+v"(best));
      if (best == 0.0) {
        // optimal on the maintained primal values (K3P's rule, oracle pfi mode)
        bool g = false;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int st = sa[s] & 3;
          if (st != ST_BASIC && (((st == ST_LB) && (sa[s] & kArtLo)) ||
                                 ((st == ST_UB) && (sa[s] & kArtHi))))
            g = true;
        }
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
        primals();
        continue;
      }
      if (iters >= io.iter_limit) {
        status = 6;
        break;
      }
      if (iters >= kmax) {  // eta file full: K3L continues this node
        status = -1;
        break;
      }
      const double delta = rrow(inf, r);
      const double sigma = delta > 0 ? 1.0 : -1.0;

      // ---- BTRAN: u = e_r' E_{k-1} ... E_0 over the nonzeros of u (rows
      // ascending: slot 0's lanes, then slot 1's) ----
      double u[kR];
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) u[rs] = rs * 64 + lane == r ? 1.0 : 0.0;
#pragma unroll
      for (int t = kKE - 1; t >= 0; --t) {
        if (t < iters) {
          // u' eta_t: lane products (row lane + row 64 + lane), summed by the
          // symmetric DPP butterfly (oracle eta_dot).  All products zero
          // and u_pt zero: the sum would write a zero back, so the eta is
          // skipped (K3P's btran_etas); a nonzero u_pt whose product
          // underflowed is still rewritten, as the oracle does
          const int pt = rl(prow, t);
          const double p0 = u[0] * eta[t][0], p1 = u[1] * eta[t][1];
          const bool upt = (lane == pt && u[0] != 0.0) || (64 + lane == pt && u[1] != 0.0);
          if (__ballot(p0 != 0.0 || p1 != 0.0 || upt) != 0ull) {
            const double acc = wave_sum_sym(p0 + p1);
#pragma unroll
            for (int rs = 0; rs < kR; ++rs)
              if (rs * 64 + lane == pt) u[rs] = acc;
          }
        }
      }
      {  // rho' = u' B0^{-1} (ascending nonzero rows), published to LDS
        double rk[kR];
        size_t lk[kR];
#pragma unroll
        for (int ks = 0; ks < kR; ++ks) {
          rk[ks] = 0.0;
          const int k = ks * 64 + lane;
          lk[ks] = (size_t)(k < m ? k : 0) * ld;
        }
#pragma unroll
        for (int rs = 0; rs < kR; ++rs) {
          uint64_t mask = __ballot(u[rs] != 0.0);
          while (mask) {  // up to four rows per round: loads first, adds in order
            int ii[4];
            int c = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              ii[t] = mask ? __builtin_ctzll(mask) : 0;
              c += mask ? 1 : 0;
              mask &= mask - 1;
            }
            double uv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) uv[t] = rld(u[rs], ii[t]);
#pragma unroll
            for (int ks = 0; ks < kR; ++ks) {
              double bv[4];
#pragma unroll
              for (int t = 0; t < 4; ++t) bv[t] = P.b0[lk[ks] + rs * 64 + ii[t]];
#pragma unroll
              for (int t = 0; t < 4; ++t)
                if (t < c) rk[ks] += uv[t] * bv[t];
            }
          }
        }
#pragma unroll
        for (int ks = 0; ks < kR; ++ks) {
          const int k = ks * 64 + lane;
          rho[k] = k < m ? rk[ks] : 0.0;
        }
      }
      wave_sync();

      // ---- pivot row and Harris pass 1 (pass-2 ratio kept per slot) ----
      double al[S], t2[S];
      double tmax = INFINITY;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        double a = 0.0, tt = INFINITY;
        const int st = sa[s] & 3;
        if (st != ST_BASIC && !(sa[s] & kFixed)) {
          a = j >= n ? -rho[j - n] : P.col_dot(rho, j);
          const double at = sigma * a, dj = d[s], fat = fabs(at);
          const bool lb = st == ST_LB && at > kPivTol, ub = st == ST_UB && at < -kPivTol,
                     fr = st == ST_FREE && fat > kPivTol;
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
      if (tmax == INFINITY) {  // dual unbounded
        bool boxed = false;
#pragma unroll
        for (int s = 0; s < S; ++s)
          boxed |= (sa[s] & 3) != ST_BASIC && (sa[s] & (kArtLo | kArtHi)) != 0;
        if (!__any(boxed) || art_bound >= 1e13) {
          status = 2;
          break;
        }
        art_bound *= 1e3;
        grow(art_bound);
        primals();
        continue;
      }
      // ---- Harris pass 2: largest |alpha| among ratios <= tmax; the owner
      // lane keeps its candidate's reduced cost, alpha and status bits ----
      double qa = 0.0, cd = 0.0, cal = 0.0;
      int q = INT_MAX, csa = 0;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (t2[s] <= tmax) {
          const double fa = fabs(al[s]);
          if (fa > qa) {
            qa = fa;
            q = s * 64 + lane;
            cd = d[s];
            cal = al[s];
            csa = sa[s];
          }
        }
      }
      wave_argmax_idx(qa, q);
      if (qa == 0.0) {
        status = 2;
        break;
      }
      const int ql = q & 63, qs = q >> 6;

      // ---- FTRAN: alpha_q = E...E B0^{-1} a_q ----
      double alq[kR];
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        const int i = rs * 64 + lane;
        const int li = i < m ? i : 0;
        double v = 0.0;
        if (q < n) {  // four entries' loads in flight, adds in CSC order
          int t = P.colptr[q];
          const int e = P.colptr[q + 1];
          for (; t + 4 <= e; t += 4) {
            const int r0 = P.rowidx[t], r1 = P.rowidx[t + 1], r2 = P.rowidx[t + 2],
                      r3 = P.rowidx[t + 3];
            const double c0 = P.cval[t], c1 = P.cval[t + 1], c2 = P.cval[t + 2],
                         c3 = P.cval[t + 3];
            const double b0 = P.b0[(size_t)r0 * ld + li], b1 = P.b0[(size_t)r1 * ld + li];
            const double b2 = P.b0[(size_t)r2 * ld + li], b3 = P.b0[(size_t)r3 * ld + li];
            v += b0 * c0;
            v += b1 * c1;
            v += b2 * c2;
            v += b3 * c3;
          }
          for (; t < e; ++t) v += P.b0[(size_t)P.rowidx[t] * ld + li] * P.cval[t];
        } else {
          v = -P.b0[(size_t)(q - n) * ld + li];
        }
        alq[rs] = i < m ? v : 0.0;
      }
      apply_etas(alq, eta, prow, iters, lane);
      const double arq = rrow(alq, r);

      // ---- steps ----
      double theta_d = rld(cd, ql) / rld(cal, ql);
      if (sigma * theta_d < 0) theta_d = 0.0;
      const double theta_p = delta / arq;
      const int pl = rrowi(h, r);
      const int pls = pl >> 6, pll = pl & 63;
#pragma unroll
      for (int s = 0; s < S; ++s)
        if ((sa[s] & 3) != ST_BASIC) d[s] -= theta_d * al[s];
      const double zq = zc[q] + theta_p;
      const bool art_q = (rl(csa, ql) & (kArtLo | kArtHi)) != 0;
      double bloq = lo[q], bhiq = hi[q];
      const double bound_p = delta < 0 ? lo[pl] : hi[pl];
      wave_sync();
      if (art_q) {  // basic columns keep their true (infinite) bounds
        bloq = P.tlo(q);
        bhiq = P.thi(q);
      }
      if (lane == 0) {
        zc[q] = 0.0;        // basic now (its value is zB of row r)
        zc[pl] = bound_p;   // leaving column to its violated bound
        lo[q] = bloq;
        hi[q] = bhiq;
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s == qs && lane == ql) {
          d[s] = 0.0;
          sa[s] = ST_BASIC | (bloq == bhiq ? kFixed : 0);
        }
        if (s == pls && lane == pll) {
          d[s] = -theta_d;
          sa[s] = (delta < 0 ? ST_LB : ST_UB) | (sa[s] & kFixed);
        }
      }
      const double inv = 1.0 / arq;
#pragma unroll
      for (int rs = 0; rs < kR; ++rs) {
        const int i = rs * 64 + lane;
        if (i < m) zB[rs] -= theta_p * alq[rs];
        // eta column of this pivot (oracle: -alpha_q/alpha_rq, 1/alpha_rq at r)
        const double e = i == r ? inv : -alq[rs] * inv;
#pragma unroll
        for (int t = 0; t < kKE; ++t)
          if (t == iters) eta[t][rs] = e;
        if (i == r) {
          h[rs] = q;
          zB[rs] = zq;
          lbB[rs] = bloq;
          ubB[rs] = bhiq;
        }
      }
      if (lane == iters) prow = r;
      ++iters;
    }

    // ---- outputs ----
    if (status == -1) {
      // overflow: take a list slot; within the slot capacity, hand K3L this
      // basis with its explicit inverse (oracle: the same loops) so it
      // continues instead of restarting
      int slot = 0;
      if (lane == 0) slot = atomicAdd(px.ovf_count, 1);
      slot = rl(slot, 0);
      if (lane == 0) px.ovf_list[slot] = b;
      if (slot < px.ovf_cap) {
#pragma unroll
        for (int rs = 0; rs < kR; ++rs) {
          const int i = rs * 64 + lane;
          if (i < m) px.c_head[(size_t)slot * m + i] = h[rs];
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = s * 64 + lane;
          if (j < N) {
            px.c_st[(size_t)slot * N + j] = (int8_t)(sa[s] & 3);
            px.c_d[(size_t)slot * N + j] = d[s];
          }
        }
        double *cb = px.c_binv + (size_t)slot * m * m;
        for (int c = 0; c < m; ++c) {
          double v[kR];
#pragma unroll
          for (int rs = 0; rs < kR; ++rs) {
            const int i = rs * 64 + lane;
            v[rs] = i < m ? P.b0[(size_t)c * ld + i] : 0.0;
          }
          apply_etas(v, eta, prow, iters, lane);
#pragma unroll
          for (int rs = 0; rs < kR; ++rs) {
            const int i = rs * 64 + lane;
            if (i < m) cb[(size_t)c * m + i] = v[rs];  // column-major (ABI layout)
          }
        }
      }
      wave_sync();
      continue;
    }
    if (status == 0 || status == 6) {
      wave_sync();
#pragma unroll
      for (int rs = 0; rs < kR; ++rs)
        if (rs * 64 + lane < m) zc[h[rs]] = zB[rs];
      wave_sync();
      if (lane == 0) {
        double sum = 0.0;  // oracle order: sequential over the structurals
        for (int j = 0; j < n; ++j) sum += P.cj(j) * zc[j];
        io.obj[b] = P.ocol < 0 ? sum + lp.objoff : sum;
      }
      if (io.x != nullptr)
        for (int j = lane; j < n; j += 64) io.x[(size_t)b * n + j] = zc[j];
    } else if (lane == 0) {
      io.obj[b] = status == 2 ? INFINITY : -INFINITY;
    }
    if (lane == 0) {
      io.status[b] = status;
      io.iters[b] = iters;
    }
    wave_sync();
  }
}

template <int S>
hipError_t launch_s(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                    hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)lp_pfiw_kernel<S>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const size_t lds = lp_pfiw_lds_bytes(lp.n, lp.m, lp.nnz);
  const int want = (io.batch + kWaves - 1) / kWaves;
  const int blocks = want < num_cus ? want : num_cus;
  hipLaunchKernelGGL((lp_pfiw_kernel<S>), dim3(blocks), dim3(64 * kWaves), lds, stream, lp, io,
                     px);
  return hipGetLastError();
}

}  // namespace

size_t lp_pfiw_lds_bytes(int n, int m, int nnz) {
  return pfiw_shared_bytes(n, m, nnz) + (size_t)kWaves * pfiw_wave_bytes(n + m);
}

bool lp_pfiw_fits(int n, int m, int nnz) {
  return m > kLpMaxM && m <= 64 * kR && n + m <= 64 * kPfiSlots &&
         lp_pfiw_lds_bytes(n, m, nnz) <= 160 * 1024;
}

hipError_t launch_lp_pfiw(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                          hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  if (!lp_pfiw_fits(lp.n, lp.m, lp.nnz) || io.ws.head == nullptr || px.kmax < 1 ||
      px.kmax > kKE)
    return hipErrorInvalidValue;
  const int S = (lp.n + lp.m + 63) / 64;
  switch (S) {
    case 2: return launch_s<2>(lp, io, px, num_cus, stream);
    case 3: return launch_s<3>(lp, io, px, num_cus, stream);
    default: return launch_s<4>(lp, io, px, num_cus, stream);
  }
}

}  // namespace mgpu
