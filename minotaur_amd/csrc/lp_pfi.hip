// K3P — batched bounded dual simplex in product form, gfx950.
//
// Same solve as K3 (repo:minotaur_amd/csrc/lp_dual.hip; OsiLPEngine::solve ->
// Clp resolve(), src/interfaces/OsiLPEngine.cpp:571-652) for the case the
// B&B hot path actually runs: every node of a batch warm-starts from ONE
// basis (the root optimum / the parent of a strong-branching batch), so the
// starting inverse B0^{-1} is the same for all of them and only the few
// pivots each node makes (5.9 on average for tls4-lin, 99.9 % <= 24) differ.
//
// MI355X-first mapping (the kernel is latency-bound, so the design goal is
// waves per SIMD: few VGPRs per node, LDS sized for 16 waves per CU):
//  * B0^{-1} is staged ONCE per workgroup in LDS, column-major with an odd
//    leading dimension m+1, so lanes reading a column (B0^{-1} a_q, the
//    primal recompute) and lanes reading a row (rho' = u' B0^{-1}) both hit
//    distinct banks.  A node's inverse is B^{-1} = E_{k-1} ... E_0 B0^{-1}:
//    k eta columns in VGPRs (lane i holds eta_t[i]; at most kPfiMax).  The
//    dense inverse of K3 (128 VGPRs per node, m FMAs per lane per pivot to
//    update) is gone.
//  * Per column j = s*64 + lane (slot s of that lane, N = n + m <= 64*S):
//    reduced cost, pivot-row entry, Harris ratio and packed status bits stay
//    in VGPRs; value and working bounds live in a per-wave LDS slice (they
//    are read by wave-uniform index or rarely).  The entering column's data
//    is captured by its owner lane during pass 2 and broadcast with
//    v_readlane: no dynamically indexed register arrays (those were demoted
//    to scratch).
//  * BTRAN visits only the nonzeros of u (a ballot mask, ascending rows) with
//    v_readlane broadcasts; FTRAN reads the CSC column of a_q from LDS and
//    applies the etas lane-parallel.
//  * A node that would need more than kmax pivots stops, is appended to an
//    overflow list and writes its basis with the explicit inverse to a
//    continuation slot; the dense K3 then continues exactly those nodes
//    (launch_lp_dual with a node list, same stream, no host sync).
//
// Arithmetic: oracle/lp_dual.c in product-form mode (dual_simplex_impl with
// pfi > 0: pfi_btran, ftran_col, pfi_apply_etas, compute_primals), loop for
// loop, so the GPU follows the oracle pivot for pivot (tests/test_lp_pfi_gpu.py).
#include <type_traits>

#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {

#ifdef MGPU_STAMPS
// Diagnostic build only (-DMGPU_STAMPS, tools/lp_stamps.py --pfi): s_memtime
// cycles per section summed over all waves; never compiled into the product.
__device__ unsigned long long g_pfi_stamps[16];
#define PSTAMP_DECL unsigned long long st_acc[12] = {0}, st_t = __builtin_amdgcn_s_memtime();
#define PSTAMP(i)                                             \
  do {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t_ - st_t;                                   \
    st_t = t_;                                                \
  } while (0)
#define PSTAMP_FLUSH                                           \
  if ((threadIdx.x & 63) == 0)                                \
    for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_pfi_stamps[i_], st_acc[i_]);
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
constexpr double kColrepTol = 1e-9;  // oracle COLREP_TOL
constexpr double kArt0 = 1e7;
constexpr double kInfB = 1e30;
constexpr int kUnknownStatus = 12;
// waves per workgroup (one workgroup per CU): 16 = 4 per SIMD (<= 128 VGPRs)
// up to 3 column slots; the 4-slot build keeps 12 (3 per SIMD).  The 32-eta
// file does not fit 128 VGPRs (168 at 3 waves per SIMD): at 4 waves per SIMD
// the compiler spills ~60 VGPRs (156 B per lane of scratch) and is still
// faster: headline K3P 15.6 -> 14.5 ms (profiles/r04f_ab).  A/B on tls4-lin
// (S = 3): 12 waves with a 24-eta file 2.12 ms, 16 waves with a 16-eta file
// 1.75 ms + a longer overflow tail (0.16 ms).
// The 48-eta build (caps above 32: narrow tree rounds, where a few LPs
// would otherwise run dense past 32 etas) at two waves per SIMD.
template <int S, int K>
constexpr int waves_for() { return K > 32 ? 8 : S <= 3 ? 16 : 12; }
__host__ __device__ inline int slots_for(int N) { return (N + 63) / 64; }

// packed column status: bits 0-1 status, 2-3 artificial-bound flags, 4 fixed
enum : int { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };
constexpr int kArtLo = 4, kArtHi = 8, kFixed = 16;

static_assert(kPfiBig < 64, "K3P never reaches K3's 64-pivot primal refresh");
// (a reinversion is taken only while the refresh stays out of reach, below)
constexpr int kPfiSmall = 16;   // the 16-eta build (4 waves per SIMD)

__host__ __device__ constexpr size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

// matrix (CSC + CSR), B0^{-1} (column-major, leading dimension m + 1),
// warm-start d / status / head
__host__ __device__ inline size_t pfi_shared_bytes(int n, int m, int nnz) {
  const int N = n + m;
  return al16((size_t)(n + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)(m + 1) * 4) + al16((size_t)nnz * 4) + al16((size_t)nnz * 8) +
         al16((size_t)m * (m + 1) * 8) + al16((size_t)N * 8) + al16((size_t)N * 4) +
         al16((size_t)m * 4) + al16((size_t)n * 4) + al16((size_t)n * 8) + 16;
}
// per wave: rho [64] + column values, lower and upper working bounds [N],
// a node pair's reduced costs [N] and head [64]
__host__ __device__ inline size_t pfi_wave_bytes(int N) {
  return 64 * 8 + 4 * al16((size_t)N * 8) + 64 * 4;
}

__device__ __forceinline__ double art_lo(double thi, double ab) {
  return (thi < kInfB ? thi : 0.0) - ab;
}
__device__ __forceinline__ double art_hi(double tlo, double ab) {
  return (tlo > -kInfB ? tlo : 0.0) + ab;
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

// v <- E_{k-1} ... E_0 v (oracle pfi_apply_etas); lanes >= m hold eta 0;
// the pivot row of eta t is lane t of prow
template <int K>
__device__ __forceinline__ double apply_etas(double v, const double (&eta)[K], int prow,
                                             int k, int lane) {
#pragma unroll
  for (int t = 0; t < K; ++t) {
    if (t < k) {
      // select, not a (wave-uniform) branch: consecutive etas overlap
      const int p = rl(prow, t);
      const double vp = rld(v, p);
      const double nv = lane == p ? eta[t] * vp : v + eta[t] * vp;
      v = vp != 0.0 ? nv : v;
    }
  }
  return v;
}

// apply_etas on G columns at once: the same operations, in the same order,
// on each column (bit for bit G apply_etas calls), as G independent chains
template <int K, int G>
__device__ __forceinline__ void apply_etas_n(double (&v)[G], const double (&eta)[K], int prow,
                                             int k, int lane) {
#pragma unroll
  for (int t = 0; t < K; ++t) {
    if (t < k) {
      const int p = rl(prow, t);
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const double vp = rld(v[i], p);
        const double nv = lane == p ? eta[t] * vp : v[i] + eta[t] * vp;
        v[i] = vp != 0.0 ? nv : v[i];
      }
    }
  }
}

// B0^{-1} a_q (oracle ftran_col, product form, before the etas): four CSC
// entries' loads in flight, adds in CSC order; lanes >= m give 0
__device__ __forceinline__ double ftran_b0(const Prob &P, int q, int lane) {
  const int li = lane < P.m ? lane : 0, ld = P.ld;
  double alq = 0.0;
  if (q < P.n) {
    int t = P.colptr[q];
    const int e = P.colptr[q + 1];
    for (; t + 4 <= e; t += 4) {
      const int r0 = P.rowidx[t], r1 = P.rowidx[t + 1], r2 = P.rowidx[t + 2],
                r3 = P.rowidx[t + 3];
      const double c0 = P.cval[t], c1 = P.cval[t + 1], c2 = P.cval[t + 2], c3 = P.cval[t + 3];
      const double b0 = P.b0[(size_t)r0 * ld + li], b1 = P.b0[(size_t)r1 * ld + li];
      const double b2 = P.b0[(size_t)r2 * ld + li], b3 = P.b0[(size_t)r3 * ld + li];
      alq += b0 * c0;
      alq += b1 * c1;
      alq += b2 * c2;
      alq += b3 * c3;
    }
    for (; t < e; ++t) alq += P.b0[(size_t)P.rowidx[t] * ld + li] * P.cval[t];
  } else {
    alq = -P.b0[(size_t)(q - P.n) * ld + li];
  }
  return lane < P.m ? alq : 0.0;
}

// B0^{-1} a_q from the launch's precomputed columns (launch_pfi_t0: the same
// ftran_b0 arithmetic, once per column instead of once per use)
__device__ __forceinline__ double ftran_col0(const Prob &P, const double *t0, int q, int lane) {
  if (t0 == nullptr) return ftran_b0(P, q, lane);
  return lane < P.m ? t0[(size_t)q * P.m + lane] : 0.0;
}

// t0[q][i] = (B0^{-1} a_q)_i, one wave per column, B0^{-1} read in place
// (column-major, leading dimension m: the ABI layout) with ftran_b0's loop
__global__ __launch_bounds__(256) void pfi_t0_kernel(DevLP lp, const double *binv, double *t0) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = lp.n, m = lp.m;
  if (q >= n + m) return;
  const int li = lane < m ? lane : 0;
  double alq = 0.0;
  if (q < n) {
    int t = lp.colptr[q];
    const int e = lp.colptr[q + 1];
    for (; t + 4 <= e; t += 4) {
      const int r0 = lp.rowidx[t], r1 = lp.rowidx[t + 1], r2 = lp.rowidx[t + 2],
                r3 = lp.rowidx[t + 3];
      const double c0 = lp.cval[t], c1 = lp.cval[t + 1], c2 = lp.cval[t + 2], c3 = lp.cval[t + 3];
      const double b0 = binv[(size_t)r0 * m + li], b1 = binv[(size_t)r1 * m + li];
      const double b2 = binv[(size_t)r2 * m + li], b3 = binv[(size_t)r3 * m + li];
      alq += b0 * c0;
      alq += b1 * c1;
      alq += b2 * c2;
      alq += b3 * c3;
    }
    for (; t < e; ++t) alq += binv[(size_t)lp.rowidx[t] * m + li] * lp.cval[t];
  } else {
    alq = -binv[(size_t)(q - n) * m + li];
  }
  if (lane < m) t0[(size_t)q * m + lane] = alq;
}

// u <- u' E_{k-1} ... E_0 (oracle pfi_btran's eta loop): each E_t' rewrites
// component prow[t] with u' eta_t, the lane products summed by the
// symmetric DPP butterfly (oracle eta_dot)
template <int K>
__device__ __forceinline__ double btran_etas(double u, const double (&eta)[K], int prow, int k,
                                             int lane) {
#pragma unroll
  for (int t = K - 1; t >= 0; --t) {
    if (t < k) {
      // all products zero and u_p zero: the sum would write a zero back;
      // skipping changes at most the sign of a zero, which no later step
      // reads (sums, and u_b0 skips zeros).  A nonzero u_p whose product
      // underflowed is still rewritten (to the sum's zero, as the oracle)
      const int p = rl(prow, t);
      const double pr = u * eta[t];
      if (__ballot(pr != 0.0 || (lane == p && u != 0.0)) != 0ull) {
        const double acc = wave_sum_sym(pr);
        if (lane == p) u = acc;
      }
    }
  }
  return u;
}

// (u' B0^{-1})_lane over the nonzero rows of u, ascending (four loads in
// flight, adds in order)
__device__ __forceinline__ double u_b0(const Prob &P, double u, int lane) {
  uint64_t mask = __ballot(u != 0.0);
  double rk = 0.0;
  const size_t lk = (size_t)(lane < P.m ? lane : 0) * P.ld;
  while (mask) {
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
    for (int t = 0; t < 4; ++t) bv[t] = P.b0[lk + ii[t]];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < c) rk += rld(u, ii[t]) * bv[t];
  }
  return rk;
}

template <int S, int K>
__global__ __launch_bounds__((64 * waves_for<S, K>())) void lp_pfi_kernel(DevLP lp, LpIO io,
                                                                       PfiIO px) {
  constexpr int kWaves = waves_for<S, K>();
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
  int *s_oidx = (int *)p;        p += al16((size_t)n * 4);    // nonzero objective columns
  double *s_oval = (double *)p;  p += al16((size_t)n * 8);
  int *s_onnz = (int *)p;        p += 16;
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
  if (wave == 0) {
    // the objective's nonzero columns in column order: the objective sum
    // skips the zero terms (adding +-0 to a sum that starts at +0 never
    // changes its bits, so the value is the oracle's full sum)
    int cnt = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane0;
      const double cv = j < n ? lp.objd[j] : 0.0;
      const uint64_t mask = __ballot(cv != 0.0);
      if (cv != 0.0) {
        const int pos = cnt + __popcll(mask & ((1ull << lane0) - 1ull));
        s_oidx[pos] = j;
        s_oval[pos] = cv;
      }
      cnt += __popcll(mask);
    }
    if (lane0 == 0) *s_onnz = cnt;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < m; t += T) s_wst[s_whead[t]] = ST_BASIC;  // basic = in head
  __syncthreads();

  Prob P;
  P.colptr = s_colptr; P.rowidx = s_rowidx; P.cval = s_cval;
  P.rowptr = s_rowptr; P.ccol = s_ccol; P.rval = s_rval;
  P.b0 = s_b0;
  P.n = n; P.m = m; P.N = N; P.ld = ld;
  P.rlo = lp.rlo; P.rhi = lp.rhi; P.c = lp.objd;
  double *rho = (double *)(p + (size_t)wave * pfi_wave_bytes(N));
  const size_t Np = al16((size_t)N * 8) / 8;
  double *zc = rho + 64;   // value of each nonbasic column, 0 for basic ones
  double *lo = zc + Np;    // working bounds (artificial where marked)
  double *hi = lo + Np;
  double *sib_d = hi + Np;                            // a pair's shared reduced costs
  int *sib_h = reinterpret_cast<int *>(sib_d + Np);   // and basis head [64]

  // persistent waves over nodes (no workgroup barrier below this point)
  PSTAMP_DECL
  unsigned long long wave_piv = 0;   // pivots this wave ran (PfiIO::pivots)
  // Nodes are taken from a device counter: a wave that finishes early takes
  // the next node, so the kernel ends with the last node, not with the wave
  // that drew the longest static share (pivot counts range 0..24+).
  //
  // Nodes come in PAIRS (2p, 2p + 1): the batched tree pops children pairs
  // that start from the same parent basis, and the column replacements of a
  // basis warm start and the reduced costs they give depend on the basis
  // alone, so the second node of a pair with the first's basis reuses them
  // (eta columns [0, k) stay intact under the first node's pivots; head and
  // reduced costs are kept in the wave's LDS slice).  The same operations,
  // so the same bits as computing them again.
  double eta[K];
#pragma unroll
  for (int t = 0; t < K; ++t) eta[t] = 0.0;
  int prow = 0;      // lane t: pivot row of eta t
  int sib = -1;      // the node whose column replacements eta [0, ksib) hold
  int ksib = 0;
  for (;;) {
    int pr = 0;
    if (lane0 == 0) pr = atomicAdd(px.next, 1);
    pr = __builtin_amdgcn_readfirstlane(pr);
    if (2 * pr >= io.batch) break;
  for (int b = 2 * pr; b < 2 * pr + 2 && b < io.batch; ++b) {
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int prev_sib = sib;   // reusable by this node only
    sib = -1;
    P.nlb = io.lb + (size_t)b * io.box_stride;
    P.nub = io.ub + (size_t)b * io.box_stride;
    P.ocol = io.obj_col != nullptr ? io.obj_col[b] : -1;
    P.osign = io.obj_col != nullptr ? io.obj_sign[b] : 0.0;

    if (io.skip != nullptr && io.skip[b] != 0) {
      if (lane == 0) {
        io.status[b] = kUnknownStatus;
        io.obj[b] = INFINITY;
        io.iters[b] = 0;
        if (io.path.k_out != nullptr) io.path.k_out[b] = 0;
        if (px.decide) {   // presolveNode found it infeasible (node_decide: 1)
          px.dec.decision[b] = 1;
          if (px.dec.cand_obj != nullptr) px.dec.cand_obj[b] = INFINITY;
        }
      }
      PSTAMP(9);
      continue;
    }

    // basis warm start (the batched tree's warm mode 2): the parent's
    // optimal basis as its statuses plus the kpath basic columns outside the
    // shared basis (ascending); kpath 0 = the shared basis itself
    int kpath = io.path.k != nullptr ? io.path.k[b] : 0;
    // a basis difference larger than this launch's eta file (a cap lowered
    // after the tree handed it on, a row imported from a rank with a larger
    // cap) cannot be rebuilt: the shared basis, as the oracle does
    if (kpath > px.kmax) kpath = 0;
    const uint32_t *ppath = io.path.path + (size_t)b * kPathMax;
    const int8_t *pst = io.path.st + (size_t)b * N;
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
      // slots past N act as basic: never touched
      sa[s] = valid ? (kpath > 0 ? (int)pst[j] : s_wst[j]) : ST_BASIC;
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
        if (io.path.k_out != nullptr) io.path.k_out[b] = 0;
        if (px.decide) {   // ProvenInfeasible (node_decide: 1)
          px.dec.decision[b] = 1;
          if (px.dec.cand_obj != nullptr) px.dec.cand_obj[b] = INFINITY;
        }
      }
      PSTAMP(9);
      continue;
    }
    wave_sync();

    int ne = 0;    // eta columns: the warm start's column replacements, then this solve's

    // Column replacement with partial pivoting (oracle colrep_basis), from
    // the shared basis (head s_whead, no etas): the shared basis's columns
    // that are nonbasic in the target basis free their rows (freem); each
    // listed column q = colq(i), ascending (FTRAN through B0^{-1} and the etas
    // so far) takes the free row with the largest |alpha| (lowest row on
    // ties) and becomes an eta exactly as a pivot on it would.  kRG columns
    // at a time: the etas of the earlier groups go into them as kRG
    // independent chains (apply_etas_n); inside the group each new eta is
    // applied to the group's later columns, so every column sees the
    // operations of one apply_etas call in order.  false: no usable pivot
    // (< kColrepTol) for some column.  Used by the basis warm start and by
    // the reinversion when the eta file is full.
    int h = lane < m ? s_whead[lane] : -1;
    auto colrep = [&](int k, uint64_t freem, auto colq, auto group) -> bool {
      constexpr int kRG = decltype(group)::value;
      bool ok = true;
#pragma unroll 1
      for (int g = 0; g < k && ok; g += kRG) {
        double v[kRG];
        int qg[kRG];
#pragma unroll
        for (int i = 0; i < kRG; ++i) {
          const bool in = g + i < k;  // wave-uniform
          qg[i] = in ? colq(g + i) : 0;
          v[i] = in ? ftran_col0(P, px.t0, qg[i], lane) : 0.0;
        }
        apply_etas_n(v, eta, prow, g, lane);
#pragma unroll
        for (int i = 0; i < kRG; ++i) {
          if (ok && g + i < k) {
            const int s = g + i, q = qg[i];
            double best = ((freem >> lane) & 1ull) ? fabs(v[i]) : 0.0;
            const int r = wave_argmax_lane(best);
            if (!(best >= kColrepTol)) {
              ok = false;
              break;
            }
            freem &= ~(1ull << r);
            const double inv = 1.0 / rld(v[i], r);
            const double e = lane == r ? inv : -v[i] * inv;
#pragma unroll
            for (int t = 0; t < K; ++t)
              if (t == s) eta[t] = e;
            if (lane == s) prow = r;
            if (lane == r) h = q;
#pragma unroll
            for (int i2 = i + 1; i2 < kRG; ++i2) {
              const double vp = rld(v[i2], r);
              const double nv = lane == r ? e * vp : v[i2] + e * vp;
              v[i2] = vp != 0.0 ? nv : v[i2];
            }
          }
        }
      }
      return ok;
    };

    // ---- basis rows: head, the warm start's column replacements, bounds
    // (basic columns carry no artificial box)
    bool reuse = false;
    if (kpath > 0 && prev_sib == b - 1 && ksib == kpath) {
      // the previous node's basis?  (path columns and statuses equal)
      const uint32_t *pp1 = ppath - kPathMax;
      const int8_t *ps1 = pst - N;
      bool diff = lane < kpath && ppath[lane] != pp1[lane];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        diff |= j < N && pst[j] != ps1[j];
      }
      reuse = !__any(diff);
    }
    if (reuse) {
      ne = kpath;
      h = lane < m ? sib_h[lane] : -1;
      sib = b;
    } else if (kpath > 0) {
      const uint64_t freem = __ballot(lane < m && pst[h] != ST_BASIC);
      // (two columns per group: four measured 0.8 % slower, profiles/r05f)
      if (colrep(kpath, freem, [&](int i) { return (int)(ppath[i] & 0xFFFFu); },
                 std::integral_constant<int, 2>())) {
        ne = kpath;
        if (lane < m) sib_h[lane] = h;
        sib = b;
        ksib = kpath;
      } else {  // the shared basis, its statuses and reduced costs
        kpath = 0;
        h = lane < m ? s_whead[lane] : -1;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = s * 64 + lane;
          if (j < N) sa[s] = s_wst[j];
        }
      }
    }
    PSTAMP(10);
    // the basic rows' bounds are lo[h] / hi[h] (a basic column keeps its
    // working bounds; grow() skips basic columns), read at pricing
    double d[S];
    if (reuse) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = j < N ? sib_d[j] : 0.0;
      }
    } else if (kpath > 0) {
      // reduced costs of the path's basis (oracle pfi_compute_duals): u = c_B
      // through the etas backwards (BTRAN), rho = u' B0^{-1}, d = c - rho' A
      double u = (lane < m && h < n) ? P.c[h] : 0.0;
      u = btran_etas(u, eta, prow, ne, lane);
      rho[lane] = lane < m ? u_b0(P, u, lane) : 0.0;
      wave_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = 0.0;
        if (j < N && sa[s] != ST_BASIC)
          d[s] = (j < n ? P.c[j] : 0.0) - (j >= n ? -rho[j - n] : P.col_dot(rho, j));
        if (j < N) sib_d[j] = d[s];
      }
      wave_sync();
      PSTAMP(11);
    } else if (P.ocol < 0) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        d[s] = (j < N && sa[s] != ST_BASIC) ? s_wd[j] : 0.0;
      }
    } else {
      // bound LP (oracle compute_duals at B = B0): y = osign * row r of B0^{-1}
      // when ocol is basic in row r, else 0; d_j = c_j - y' a_j
      const uint64_t on = __ballot(lane < m && h == P.ocol);
      double y = 0.0;
      if (on != 0ull && lane < m)
        y = 0.0 + P.osign * P.b0[(size_t)lane * ld + __builtin_ctzll(on)];
      rho[lane] = y;
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

    int iters = 0;  // this solve's own pivots

    // oracle compute_primals (product form): z_B = -E...E B0^{-1} (N z_N)
    auto primals = [&]() -> double {
      wave_sync();
      // row sums of N z_N in CSR (= ascending column) order.  Zero values
      // are not skipped: a product a*0 = +-0 added to a sum that starts at
      // +0 never changes its bits (cancellation gives +0), so the value is
      // the oracle's; four columns' loads in flight (the tangent rows of an
      // OA-LP hold 40+ terms).
      double w = 0.0;
      if (lane < m) {
        int t = P.rowptr[lane];
        const int e = P.rowptr[lane + 1];
        for (; t + 4 <= e; t += 4) {
          const int c0 = P.ccol[t], c1 = P.ccol[t + 1], c2 = P.ccol[t + 2], c3 = P.ccol[t + 3];
          const double a0 = P.rval[t], a1 = P.rval[t + 1], a2 = P.rval[t + 2],
                       a3 = P.rval[t + 3];
          const double z0 = zc[c0], z1 = zc[c1], z2 = zc[c2], z3 = zc[c3];
          w += a0 * z0;
          w += a1 * z1;
          w += a2 * z2;
          w += a3 * z3;
        }
        for (; t < e; ++t) w += P.rval[t] * zc[P.ccol[t]];
        const double zl = zc[n + lane];
        if (zl != 0.0) w -= zl;
      }
      // over the rows with w_k != 0 only, ascending (a zero w_k adds +-0,
      // which never changes a sum that starts at +0): four LDS loads in
      // flight, adds in order
      double sacc = 0.0;
      const int li = lane < m ? lane : 0;
      uint64_t nzw = __ballot(lane < m && w != 0.0);
      while (nzw) {
        int ii[4];
        int c = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          ii[t] = nzw ? __builtin_ctzll(nzw) : 0;
          c += nzw ? 1 : 0;
          nzw &= nzw - 1;
        }
        double bv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[t] = P.b0[(size_t)ii[t] * ld + li];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (t < c) sacc += bv[t] * rld(w, ii[t]);
      }
      if (lane >= m) sacc = 0.0;
      sacc = apply_etas(sacc, eta, prow, ne, lane);
      return -sacc;
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

    PSTAMP(0);
    // primal values are recomputed at ONE place (the top of the loop) so the
    // eta pass inside primals() is inlined once
    double zB = 0.0;
    bool need = true;   // recompute before pricing
    int status = kUnknownStatus;
    for (;;) {
      // lane-derived addresses recomputed per pivot (not hoisted and spilled)
      lane = lane0;
      asm volatile("" : "+v"(lane));
      if (need) {
        zB = primals();
        PSTAMP(1);
        need = false;
      }
      // ---- pricing: most infeasible basic row, lowest row on ties ----
      double inf = 0.0;
      if (lane < m) {
        const double lbB = lo[h], ubB = hi[h];
        if (zB < lbB - kPTol) inf = zB - lbB;
        else if (zB > ubB + kPTol) inf = zB - ubB;
      }
      double best = fabs(inf);
      const int r = wave_argmax_lane(best);  // used only when best > 0
      asm volatile("" : "+v"(best));
      PSTAMP(2);
      if (best == 0.0) {
        // optimal on the maintained primal values: the product form holds at
        // most kmax etas since the recompute at the solve's start, so no
        // second recompute confirms them (oracle: pfi mode)
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
        need = true;
        continue;
      }
      if (iters >= io.iter_limit) {
        status = 6;
        break;
      }
      if (ne >= kmax) {
        // eta file full.  Reinversion (oracle: the same rule): the current
        // basis rebuilt as column replacements on B0 -- its basic columns
        // outside the shared basis, ascending, exactly as a basis warm start
        // -- when that difference leaves an eighth of the file free and the
        // solve stays short of the 64-pivot primal refresh; the primal values
        // are then recomputed, the reduced costs kept.  Otherwise (or for
        // bound LPs, whose reduced costs are rebuilt per objective) the dense
        // K3 continues this node from its basis and explicit inverse.
        bool again = false;
        if (io.ws.d != nullptr) {
          uint64_t bm[S], nrm[S];
          int kb = 0;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const int j = s * 64 + lane;
            bm[s] = __ballot(j < N && (sa[s] & 3) == ST_BASIC);
            nrm[s] = bm[s] & ~__ballot(j < N && s_wst[j] == ST_BASIC);
            kb += __popcll(nrm[s]);
          }
          const int room = kmax / 8 > 1 ? kmax / 8 : 1;
          if (kb <= kmax - room && iters + (kmax - kb) < 64) {
            // the listed columns into the (free) rho slice, ascending
            int *cl = reinterpret_cast<int *>(rho);
            int base = 0;
#pragma unroll
            for (int s = 0; s < S; ++s) {
              if ((nrm[s] >> lane) & 1ull)
                cl[base + __popcll(nrm[s] & ((1ull << lane) - 1ull))] = s * 64 + lane;
              base += __popcll(nrm[s]);
            }
            wave_sync();
            // rows whose shared-basis column is nonbasic now are free
            const int hc = lane < m ? s_whead[lane] : 0;
            bool bnow = false;
#pragma unroll
            for (int s = 0; s < S; ++s)
              if ((hc >> 6) == s) bnow = ((bm[s] >> (hc & 63)) & 1ull) != 0;
            const uint64_t freem = __ballot(lane < m && !bnow);
            h = lane < m ? s_whead[lane] : -1;
            ne = 0;
            sib = -1;   // the column replacements are gone
            // (one column at a time: the main loop's state is live here)
            if (colrep(kb, freem, [&](int i) { return cl[i]; },
                       std::integral_constant<int, 1>())) {
              ne = kb;
              again = true;
            } else {
              // no usable pivot: the dense continuation restarts from the
              // shared basis (head, statuses, reduced costs), the pivots counted
              h = lane < m ? s_whead[lane] : -1;
#pragma unroll
              for (int s = 0; s < S; ++s) {
                const int j = s * 64 + lane;
                if (j < N) {
                  sa[s] = s_wst[j];
                  d[s] = s_wst[j] == ST_BASIC ? 0.0 : s_wd[j];
                }
              }
            }
            wave_sync();
          }
        }
        if (again) {
          need = true;
          continue;
        }
        status = -1;
        break;
      }
      const double delta = rld(inf, r);
      const double sigma = delta > 0 ? 1.0 : -1.0;

      // ---- BTRAN: u = e_r' E_{k-1} ... E_0 over the nonzeros of u, then
      // rho' = u' B0^{-1}, published to LDS ----
      {
        const double u = btran_etas(lane == r ? 1.0 : 0.0, eta, prow, ne, lane);
        rho[lane] = lane < m ? u_b0(P, u, lane) : 0.0;
      }
      wave_sync();
      PSTAMP(3);

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
      PSTAMP(4);
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
        need = true;
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
      PSTAMP(5);
      if (qa == 0.0) {
        status = 2;
        break;
      }
      const int ql = q & 63, qs = q >> 6;

      // ---- FTRAN: alpha_q = E...E B0^{-1} a_q ----
      const double alq = apply_etas(ftran_col0(P, px.t0, q, lane), eta, prow, ne, lane);
      const double arq = rld(alq, r);
      PSTAMP(6);

      // ---- steps ----
      double theta_d = rld(cd, ql) / rld(cal, ql);
      if (sigma * theta_d < 0) theta_d = 0.0;
      const double theta_p = delta / arq;
      const int pl = rl(h, r);
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
      if (lane < m) zB -= theta_p * alq;
      if (lane == r) {
        h = q;
        zB = zq;
      }
      // ---- eta column of this pivot (oracle: -alpha_q/alpha_rq, 1/alpha_rq at r)
      const double inv = 1.0 / arq;
      const double e = lane == r ? inv : -alq * inv;
#pragma unroll
      for (int t = 0; t < K; ++t)
        if (t == ne) eta[t] = e;
      if (lane == ne) prow = r;
      ++ne;
      ++iters;
      PSTAMP(7);
    }

    wave_piv += (unsigned long long)iters;   // this kernel's own pivots
    // ---- outputs ----
    if (status == -1) {
      // overflow: take a list slot; within the slot capacity, hand K3 this
      // basis with its explicit inverse (oracle: the same loops) so it
      // continues instead of restarting
      int slot = 0;
      if (lane == 0) slot = atomicAdd(px.ovf_count, 1);
      slot = rl(slot, 0);
      if (lane == 0) {
        px.ovf_list[slot] = b;
        if (io.path.k_out != nullptr) io.path.k_out[b] = 0;   // children: from the root
      }
      if (slot < px.ovf_cap) {
        if (lane == 0) px.c_iters[slot] = iters;
        if (lane < m) px.c_head[(size_t)slot * m + lane] = h;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = s * 64 + lane;
          if (j < N) {
            px.c_st[(size_t)slot * N + j] = (int8_t)(sa[s] & 3);
            px.c_d[(size_t)slot * N + j] = d[s];
          }
        }
        double *cb = px.c_binv + (size_t)slot * m * m;
        const int li = lane < m ? lane : 0;
        for (int c = 0; c < m; ++c) {
          double v = lane < m ? P.b0[(size_t)c * ld + li] : 0.0;
          v = apply_etas(v, eta, prow, ne, lane);
          if (lane < m) cb[(size_t)c * m + lane] = v;  // column-major (ABI layout)
        }
      }
      wave_sync();
      PSTAMP(8);
      continue;
    }
    if (status == 0 || status == 6) {
      wave_sync();
      if (lane < m) zc[h] = zB;
      wave_sync();
      // objective as the oracle sums it: sequentially over the columns, so
      // the value is the oracle's bit for bit (best-first search orders nodes
      // by these bounds; a last-bit difference reorders ties)
      // the products lane-parallel (64 nonzero columns per pass), the sum
      // sequential in column order through readlanes of the nonzero products
      // (a zero value gives +-0, which the sum skips for the same reason)
      double sum = 0.0;
      if (P.ocol >= 0) {
        sum += P.osign * zc[P.ocol];
      } else {
        const int no = *s_onnz;
        for (int k0 = 0; k0 < no; k0 += 64) {
          const int k = k0 + lane;
          const double pr = k < no ? s_oval[k] * zc[s_oidx[k]] : 0.0;
          uint64_t nz = __ballot(pr != 0.0);
          while (nz != 0ull) {
            const int i = __builtin_ctzll(nz);
            nz &= nz - 1ull;
            sum += rld(pr, i);
          }
        }
      }
      const double solval = P.ocol < 0 ? sum + lp.objoff : sum;
      if (lane == 0) io.obj[b] = solval;
      int dec = -1;
      if (px.decide) {
        // node_decide_kernel's decision on the values in LDS (the same
        // tests in the same order): the bound test of shouldPrune_, then
        // IntVarHandler::isFeasible, then MaxVioBrancher's choice
        const DecideIO &dd = px.dec;
        const double cut = dd.incumbent;
        if (solval >= cut - dd.abs_tol || solval >= cut - fabs(cut) * dd.rel_tol ||
            solval >= dd.cutoff) {
          dec = 2;
        } else {
          bool frac = false;
          for (int j = lane; j < n; j += 64) {
            const uint8_t t = lp.vtype[j];
            if (t == kBinary || t == kInteger) {
              const double v = zc[j];
              frac |= fabs(v - floor(v + 0.5)) > dd.int_tol;
            }
          }
          dec = __any(frac) ? 0 : 3;
          if (dec == 0 && dd.bvar != nullptr) {
            double best = -INFINITY;
            int bj = INT_MAX;
            for (int j = lane; j < n; j += 64) {
              const uint8_t t = lp.vtype[j];
              if (t != kBinary && t != kInteger) continue;
              const double v = zc[j];
              if (!(fabs(floor(v + 0.5) - v) > dd.int_tol)) continue;
              const double dn = v - floor(v), up = ceil(v) - v;
              const double lo_ = (up < dn) ? up : dn, hi_ = (dn < up) ? up : dn;
              const double sc = 0.1 * (0.8 * lo_ + 0.2 * hi_);
              if (sc > best) {
                best = sc;
                bj = j;
              }
            }
            wave_argmax(best, bj);
            if (lane == 0) {
              const double v = zc[bj];
              dd.bvar[b] = bj;
              dd.bval[b] = v;
              dd.bup[b] = (v - floor(v)) > (ceil(v) - v) ? 1 : 0;
            }
          }
        }
        if (lane == 0) {
          dd.decision[b] = dec;
          if (dd.cand_obj != nullptr) dd.cand_obj[b] = dec == 3 ? solval : INFINITY;
        }
      }
      // x for the caller; with the fused decision only an incumbent
      // candidate's (the tree reads no other node's x)
      if (io.x != nullptr && (!px.decide || dec == 3))
        for (int j = lane; j < n; j += 64) io.x[(size_t)b * n + j] = zc[j];
    } else {
      if (lane == 0) io.obj[b] = status == 2 ? INFINITY : -INFINITY;
      if (px.decide && lane == 0) {   // 2 infeasible -> 1; 4 unbounded -> 4 (engine)
        px.dec.decision[b] = status == 2 ? 1 : 4;
        if (px.dec.cand_obj != nullptr) px.dec.cand_obj[b] = INFINITY;
      }
    }
    if (lane == 0) {
      io.status[b] = status;
      io.iters[b] = iters;
    }
    if (io.path.k_out != nullptr) {
      // the node's final basis for its children: its statuses and its basic
      // columns outside the shared basis in ascending order (optimal, at
      // most `inherit` of them; else k_out 0: the children start from the
      // shared basis)
      int ko = 0;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = s * 64 + lane;
        ko += __popcll(__ballot(j < N && (sa[s] & 3) == ST_BASIC && s_wst[j] != ST_BASIC));
      }
      if (status != 0 || ko > io.path.inherit) ko = 0;
      if (lane == 0) io.path.k_out[b] = ko;
      if (ko > 0) {
        int base = 0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = s * 64 + lane;
          const bool e = j < N && (sa[s] & 3) == ST_BASIC && s_wst[j] != ST_BASIC;
          const uint64_t em = __ballot(e);
          if (e) io.path.path_out[(size_t)b * kPathMax + base +
                                  __popcll(em & ((1ull << lane) - 1ull))] = (uint32_t)j;
          base += __popcll(em);
          if (j < N) io.path.st_out[(size_t)b * N + j] = (int8_t)(sa[s] & 3);
        }
      }
    }
    wave_sync();
    PSTAMP(8);
  }
  }
  if (lane0 == 0 && px.pivots != nullptr && wave_piv != 0) atomicAdd(px.pivots, wave_piv);
  PSTAMP_FLUSH
}

template <int S, int K>
hipError_t launch_s(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                    hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)lp_pfi_kernel<S, K>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  constexpr int kWaves = waves_for<S, K>();
  const size_t lds = lp_pfi_lds_bytes(lp.n, lp.m, lp.nnz, px.kmax);
  const int want = (io.batch + kWaves - 1) / kWaves;
  const int blocks = want < num_cus ? want : num_cus;
  hipLaunchKernelGGL((lp_pfi_kernel<S, K>), dim3(blocks), dim3(64 * kWaves), lds, stream, lp,
                     io, px);
  return hipGetLastError();
}

template <int K>
hipError_t launch_k(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                    hipStream_t stream) {
  switch ((lp.n + lp.m + 63) / 64) {
    case 1: return launch_s<1, K>(lp, io, px, num_cus, stream);
    case 2: return launch_s<2, K>(lp, io, px, num_cus, stream);
    case 3: return launch_s<3, K>(lp, io, px, num_cus, stream);
    default: return launch_s<4, K>(lp, io, px, num_cus, stream);
  }
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

hipError_t launch_pfi_t0(const DevLP &lp, const double *binv, double *t0, hipStream_t stream) {
  const int N = lp.n + lp.m;
  hipLaunchKernelGGL(pfi_t0_kernel, dim3((N + 3) / 4), dim3(256), 0, stream, lp, binv, t0);
  return hipGetLastError();
}

size_t lp_pfi_lds_bytes(int n, int m, int nnz, int kmax) {
  const bool small = kmax <= kPfiSmall, big = kmax > kPfiMax;
  const int waves = big ? waves_for<3, kPfiBig>()
                    : slots_for(n + m) <= 3 ? (small ? waves_for<3, kPfiSmall>()
                                                     : waves_for<3, kPfiMax>())
                                            : waves_for<4, kPfiMax>();
  return pfi_shared_bytes(n, m, nnz) + (size_t)waves * pfi_wave_bytes(n + m);
}

bool lp_pfi_fits(int n, int m, int nnz) {
  return m <= kLpMaxM && n + m <= 64 * kPfiSlots &&
         lp_pfi_lds_bytes(n, m, nnz, kPfiSmall) <= 160 * 1024 &&
         lp_pfi_lds_bytes(n, m, nnz, kPfiMax) <= 160 * 1024;
}

hipError_t launch_lp_pfi(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                         hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  if (!lp_pfi_fits(lp.n, lp.m, lp.nnz) || io.ws.head == nullptr || px.kmax < 1 ||
      px.kmax > kPfiBig)
    return hipErrorInvalidValue;
  // the eta file in VGPRs is sized at compile time: 16 when the cap allows,
  // 32 (the default cap), 48 above it
  if (px.kmax <= kPfiSmall) return launch_k<kPfiSmall>(lp, io, px, num_cus, stream);
  if (px.kmax <= kPfiMax) return launch_k<kPfiMax>(lp, io, px, num_cus, stream);
  return launch_k<kPfiBig>(lp, io, px, num_cus, stream);
}

}  // namespace mgpu
