// K3R — per-node refactorisation of the warm basis when every node has its
// own rows, gfx950.
//
// The glob path rewrites the secant / McCormick rows at every node
// (QuadHandler::upSqCon_ / upBilCon_, src/base/QuadHandler.cpp:3322-3419)
// and OsiLPEngine::changeConstraint loads them (src/interfaces/
// OsiLPEngine.cpp:206-243); Clp then refactors the kept basis for the new
// matrix before the dual simplex.  Here the batch shares the sparsity
// pattern and each node brings its values (NodeRowsIO), so one kernel builds
// every node's warm start for K3: the oracle's invert_basis (Gauss-Jordan
// with partial pivoting over [B | I], largest |pivot| with the first row on
// ties, a pivot below 1e-12 = singular -> the slack basis) and compute_duals
// (y = c_B' B^-1, d_j = c_j - y' a_j in CSC order), in the oracle's
// arithmetic order, so K3 then follows oracle/lp_dual.c pivot for pivot.
//
// Mapping: one node per wave64 (one wave per workgroup).  Lane r holds
// constraint row r of B and of I in VGPRs.  The pivot column is always
// register 0: each elimination step shifts the B row left by one (columns
// already pivoted are unit vectors that are never read again), so the
// dynamic step loop indexes registers only with compile-time constants.
// The I part is kept in PIVOT order: register k holds the column of the row
// pivoted at step k, and a row's own identity entry (exactly 1 until that
// row is pivoted) is implicit.  At step c only registers 0..c of I and
// 0..m-c-1 of B can be nonzero, so both updates run over 8-register chunks
// below those bounds (wave-uniform branches): half the work of the dense
// [B | I] sweep.  The values are the oracle's (the skipped entries are the
// zeros it updates); only the sign of a zero entry of B^-1 can differ, which
// no consumer distinguishes.  The pivot row is broadcast through LDS.  Steps
// whose column has no other nonzero (slack columns) skip the elimination with
// a wave-uniform branch.
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

constexpr double kSingTol = 1e-12;  // oracle invert_basis: |pivot| < 1e-12 = singular
enum : int8_t { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };

__host__ __device__ constexpr size_t al16r(size_t b) { return (b + 15) & ~(size_t)15; }

template <int M>
__global__ __launch_bounds__(64) void lp_refactor_kernel(DevLP lp, RefacIO io) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = lp.n, m = lp.m, N = n + m, nnz = lp.nnz, ld = m + 1;
  if (io.skip != nullptr && io.skip[b] != 0) return;  // K3 skips the node too

  unsigned char *p = smem;
  double *wc = (double *)p;   p += al16r((size_t)nnz * 8);      // node CSC values
  double *Ls = (double *)p;   p += al16r((size_t)m * ld * 8);   // dense B, then B^-1 rows
  double *prow = (double *)p; p += al16r((size_t)2 * M * 8);    // pivot row broadcast
  int32_t *pord = (int32_t *)p; p += al16r((size_t)M * 4);       // row pivoted at step k
  double *y = (double *)p;    p += al16r((size_t)m * 8);
  int32_t *hd = (int32_t *)p; p += al16r((size_t)m * 4);
  int8_t *st = (int8_t *)p;

  // the node's matrix: the loaded values, then its own entries
  for (int t = lane; t < nnz; t += 64) wc[t] = lp.cval[t];
  wave_sync();
  const double *rec = io.nr.vals + (size_t)b * io.nr.stride;
  for (int q = lane; q < io.nr.ncoef; q += 64) {
    double v = rec[io.nr.coef_src[q]];
    if (fabs(v) <= kLfTol) v = 0.0;
    wc[io.nr.csc_pos[q]] = v;
  }
  // warm basis: statuses with the basic columns from head (oracle: st of the
  // non-basic columns, ST_BASIC -> ST_LB, then head[i] basic)
  const int32_t *wh = io.head + (size_t)b * io.s_head;
  const int8_t *wst = io.st + (size_t)b * io.s_st;
  for (int i = lane; i < m; i += 64) hd[i] = wh[i];
  for (int j = lane; j < N; j += 64) {
    const int8_t s = wst[j];
    st[j] = s == ST_BASIC ? ST_LB : s;
  }
  wave_sync();
  for (int i = lane; i < m; i += 64) st[hd[i]] = ST_BASIC;
  const bool row = lane < m;
  const size_t mm = (size_t)m * m;
  bool done = false;
  if (io.binv0 != nullptr) {
    // column replacement from the root inverse (oracle colrep_refactor):
    // only the basic structural columns whose entries this node rewrote
    // differ from the root basis; each takes its node column by one
    // product-form update of B^-1, held row-major in Ls (stride ld)
    for (size_t t = lane; t < mm; t += 64) Ls[(t % m) * ld + t / m] = io.binv0[t];
    wave_sync();
    done = true;
    for (int i = 0; i < m; ++i) {
      const int h = hd[i];
      if (h >= n) continue;
      bool ch = false;
      for (int t = lp.colptr[h] + lane; t < lp.colptr[h + 1]; t += 64) ch |= wc[t] != lp.cval[t];
      if (!__any(ch)) continue;
      double al = 0.0;
      if (row)
        for (int t = lp.colptr[h]; t < lp.colptr[h + 1]; ++t)
          al += Ls[(size_t)lane * ld + lp.rowidx[t]] * wc[t];
      const double piv = rld(al, i);
      if (fabs(piv) < kSingTol) {
        done = false;  // refactor from scratch below
        break;
      }
      const double inv = 1.0 / piv;
      for (int k = lane; k < m; k += 64) Ls[(size_t)i * ld + k] *= inv;
      wave_sync();
      if (row && lane != i && al != 0.0)
        for (int k = 0; k < m; ++k) Ls[(size_t)lane * ld + k] -= al * Ls[(size_t)i * ld + k];
      wave_sync();
    }
  }
  int32_t *oh = io.o_head + (size_t)b * m;
  int8_t *ost = io.o_st + (size_t)b * N;
  double *od = io.o_d + (size_t)b * N;
  double *ob = io.o_binv + mm * b;
  if (!done) {
  for (int t = lane; t < m * ld; t += 64) Ls[t] = 0.0;
  wave_sync();
  // dense basis matrix: column i of B = column head[i] of [A | -I]
  for (int i = lane; i < m; i += 64) {
    const int h = hd[i];
    if (h >= n) {
      Ls[(size_t)(h - n) * ld + i] = -1.0;
    } else {
      for (int t = lp.colptr[h]; t < lp.colptr[h + 1]; ++t) Ls[(size_t)lp.rowidx[t] * ld + i] = wc[t];
    }
  }
  wave_sync();

  constexpr int kC = 8;          // register chunk of the skipped updates
  constexpr int NQ = M / kC;
  static_assert(M % kC == 0, "register rows are whole chunks");
  double Bv[M], Iv[M];  // Iv[k]: the column of the row pivoted at step k
#pragma unroll
  for (int k = 0; k < M; ++k) {
    Bv[k] = (row && k < m) ? Ls[(size_t)lane * ld + k] : 0.0;
    Iv[k] = 0.0;
  }
  int lpos = lane;  // logical row (row swaps move logical positions, not data)
  bool sing = false;
  for (int c = 0; c < m; ++c) {
    // pivot: the largest |B_rc| over logical rows r >= c, the first on ties
    // (oracle: strictly greater than the best so far, starting from 0)
    const double a = fabs(Bv[0]);
    double v = (row && lpos >= c && a > 0.0) ? a : -1.0;
    const double mx = wave_max_dpp(v);
    if (mx < kSingTol) {  // no candidate, or below the tolerance
      sing = true;
      break;
    }
    const uint64_t hit = __ballot(v == mx);
    int P;
    if (__popcll(hit) == 1) {
      P = (int)__builtin_ctzll(hit);
    } else {
      const int lmin = wave_min_i32_dpp(v == mx ? lpos : INT_MAX);
      P = (int)__builtin_ctzll(__ballot(v == mx && lpos == lmin));
    }
    const int Q = (int)__builtin_ctzll(__ballot(row && lpos == c));
    const int lp_P = rl(lpos, P);
    if (lane == Q) lpos = lp_P;  // swap rows c and piv
    if (lane == P) lpos = c;
    // scale the pivot row by 1 / pivot (a product, as the oracle); its own
    // identity entry (1) becomes inv at pivot position c
    const double inv = 1.0 / rld(Bv[0], P);
    if (lane == 0) pord[c] = P;
    if (lane == P) {
#pragma unroll
      for (int k = 0; k < M; ++k) Bv[k] *= inv;
#pragma unroll
      for (int k = 1; k < M; ++k) prow[k] = Bv[k];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q * kC <= c) {
#pragma unroll
          for (int k = q * kC; k < q * kC + kC; ++k) {
            Iv[k] = k < c ? Iv[k] * inv : k == c ? inv : Iv[k];
            prow[M + k] = Iv[k];
          }
        }
      }
    }
    wave_sync();
    // eliminate column c from every other row with f = B_rc != 0
    const double f = Bv[0];
    const bool upd = row && lane != P && f != 0.0;
    if (__any(upd)) {
#pragma unroll
      for (int k = 0; k + 1 < M; ++k) {
        const double t = Bv[k + 1] - f * prow[k + 1];
        Bv[k] = upd ? t : Bv[k + 1];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q * kC <= c) {
#pragma unroll
          for (int k = q * kC; k < q * kC + kC; ++k) {
            const double t = Iv[k] - f * prow[M + k];
            Iv[k] = upd ? t : Iv[k];
          }
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k + 1 < M; ++k) Bv[k] = Bv[k + 1];
    }
    Bv[M - 1] = 0.0;
    wave_sync();  // prow is rewritten by the next step
  }

  if (io.o_sing != nullptr && lane == 0) io.o_sing[b] = sing ? 1 : 0;
  if (sing) {
    // oracle: the warm start is dropped for the slack basis (B^-1 = -I,
    // y = 0: d_j = c_j for the structurals, 0 for the basic slacks)
    for (int i = lane; i < m; i += 64) oh[i] = n + i;
    for (int j = lane; j < N; j += 64) {
      ost[j] = j < n ? ST_LB : ST_BASIC;
      od[j] = j < n ? lp.objd[j] : 0.0;
    }
    for (int k = 0; k < m; ++k)
      for (int i = lane; i < m; i += 64) ob[(size_t)k * m + i] = i == k ? -1.0 : 0.0;
    return;
  }
  // row lpos of B^-1 (basis position lpos) to LDS, row-major: pivot
  // position k is column pord[k] of the identity part
  if (row) {
#pragma unroll
    for (int k = 0; k < M; ++k)
      if (k < m) Ls[(size_t)lpos * ld + pord[k]] = Iv[k];
  }
  wave_sync();
  } else if (io.o_sing != nullptr && lane == 0) {
    io.o_sing[b] = 0;
  }
  // column-major B^-1: column k is one coalesced store over the lanes
  for (int k = 0; k < m; ++k)
    for (int i = lane; i < m; i += 64) ob[(size_t)k * m + i] = Ls[(size_t)i * ld + k];
  // y_k = sum over basis positions i (ascending) of c_B[i] * B^-1[i][k]
  for (int k = lane; k < m; k += 64) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) {
      const int h = hd[i];
      const double cb = h < n ? lp.objd[h] : 0.0;
      if (cb != 0.0) s += cb * Ls[(size_t)i * ld + k];
    }
    y[k] = s;
  }
  wave_sync();
  for (int i = lane; i < m; i += 64) oh[i] = hd[i];
  for (int j = lane; j < N; j += 64) {
    ost[j] = st[j];
    double d = 0.0;
    if (st[j] != ST_BASIC) {
      double dot;
      if (j >= n) {
        dot = -y[j - n];
      } else {
        dot = 0.0;
        for (int t = lp.colptr[j]; t < lp.colptr[j + 1]; ++t) dot += wc[t] * y[lp.rowidx[t]];
      }
      d = (j < n ? lp.objd[j] : 0.0) - dot;
    }
    od[j] = d;
  }
}

template <int M>
size_t refactor_lds(int n, int m, int nnz) {
  return al16r((size_t)nnz * 8) + al16r((size_t)m * (m + 1) * 8) + al16r((size_t)2 * M * 8) +
         al16r((size_t)M * 4) + al16r((size_t)m * 8) + al16r((size_t)m * 4) +
         al16r((size_t)(n + m));
}

template <int M>
hipError_t launch_m(const DevLP &lp, const RefacIO &io, hipStream_t stream) {
  const size_t lds = refactor_lds<M>(lp.n, lp.m, lp.nnz);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)lp_refactor_kernel<M>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(lp_refactor_kernel<M>, dim3(io.batch), dim3(64), lds, stream, lp, io);
  return hipGetLastError();
}

}  // namespace

// register rows sized to the basis: M <= 56 keeps the two rows of B and I
// under 256 VGPRs (two waves per SIMD), M = 64 needs AGPRs (one wave)
size_t lp_refactor_lds_bytes(int n, int m, int nnz) {
  return m <= 32 ? refactor_lds<32>(n, m, nnz)
       : m <= 56 ? refactor_lds<56>(n, m, nnz) : refactor_lds<64>(n, m, nnz);
}

hipError_t launch_lp_refactor(const DevLP &lp, const RefacIO &io, hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  if (lp.m > kLpMaxM || lp.m <= 0) return hipErrorInvalidValue;
  return lp.m <= 32 ? launch_m<32>(lp, io, stream)
       : lp.m <= 56 ? launch_m<56>(lp, io, stream) : launch_m<64>(lp, io, stream);
}

}  // namespace mgpu
