// K5 — batched QP relaxation solve with an MFMA KKT block, gfx950
// (QPDRelaxer / BqpdEngine, src/interfaces/
// BqpdEngine.cpp:449-534).
//
//   min 1/2 x'Qx + c'x + k   s.t.  A x = b,  l <= x <= u   (node box)
//
// Mehrotra predictor-corrector interior point, one node per workgroup.  The
// Newton system is the KKT block [Q + D, A'; A, 0] (D = Z_l/S_l + Z_u/S_u),
// reduced through its Schur complement:
//   K = Q + D = L L'        qp_potrf_ll blocked left-looking Cholesky:
//                                       16x16 tiles, each tile's update
//                                       over all earlier column blocks on
//                                       v_mfma_f64_16x16x4_f64, L written
//                                       once (qp_potrf: the right-looking
//                                       form, for n past its LDS panel)
//   W = L^-1 A', M = W'W    qp_trsm_syrk  blocked forward substitution and
//                                       the Gram product, both on MFMA
//   M = Lm Lm', steps       qp_step    Lm in LDS, predictor + corrector
//                                       solves, ratio tests, updates
// Layout: n, m padded to multiples of 16 (np, mp); padded variables are
// fixed at 0 (identity rows of K), padded rows of A are zero.  Per node in
// HBM: K [np][np] (lower triangle = L after qp_potrf), W [np][mp], M
// [mp][mp] and the iterate (x, y, zl, zu).  The arithmetic follows the CPU
// restatement oracle/qp_ipm.py step for step (objectives agree to 1e-6;
// iterates up to rounding).
#include "mgpu_internal.h"
#include "qp_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;  // threads per workgroup (4 waves)

__device__ __forceinline__ double block_sum(double v, double *red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
__device__ __forceinline__ double block_min(double v, double *red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if (t < o) red[t] = fmin(red[t], red[t + o]);
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
__device__ __forceinline__ double block_max(double v, double *red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if (t < o) red[t] = fmax(red[t], red[t + o]);
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// ---- init ------------------------------------------------------------------
__global__ __launch_bounds__(kT) void qp_init(DevQP q, QpWork w) {
  __shared__ int s_empty;
  const int b = blockIdx.x;
  const size_t o = (size_t)b * q.np;
  if (threadIdx.x == 0) s_empty = 0;
  __syncthreads();
  for (int j = threadIdx.x; j < q.np; j += kT) {
    const double l = w.l[o + j], u = w.u[o + j];
    const bool fr = l < u;
    if (l > u) s_empty = 1;
    w.x[o + j] = fr ? 0.5 * (l + u) : l;
    w.zl[o + j] = fr ? 1.0 : 0.0;
    w.zu[o + j] = fr ? 1.0 : 0.0;
  }
  for (int i = threadIdx.x; i < q.mp; i += kT) w.y[(size_t)b * q.mp + i] = 0.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    // a skipped node (presolve found it infeasible) is not solved; an empty
    // box is infeasible before any iteration
    const bool skip = w.skip != nullptr && w.skip[b] != 0;
    w.done[b] = skip || s_empty ? 1 : 0;
    w.iters[b] = 0;
    w.status[b] = skip ? 12 : s_empty ? 2 : 6;
  }
}

// ---- residuals, convergence test, K and W assembly --------------------------
__global__ __launch_bounds__(kT) void qp_prep(DevQP q, QpWork w, int assemble) {
  __shared__ double red[kT];
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x;
  if (w.done[b]) return;
  const int np = q.np, mp = q.mp;
  const size_t o = (size_t)b * np, oy = (size_t)b * mp;
  double *x = sm, *y = sm + np;
  for (int j = t; j < np; j += kT) x[j] = w.x[o + j];
  for (int i = t; i < mp; i += kT) y[i] = w.y[oy + i];
  __syncthreads();
  // rd = Qx + c - A'y - zl + zu on free variables (Q symmetric: column
  // access Q[i][j] over i is coalesced across j)
  double rdmax = 0.0, comp = 0.0, nf = 0.0, xmax = 0.0;
  for (int j = t; j < np; j += kT) {
    xmax = fmax(xmax, fabs(x[j]));
    double qx = 0.0;
    for (int i = 0; i < np; ++i) qx += q.Q[(size_t)i * np + j] * x[i];
    double aty = 0.0;
    for (int i = 0; i < mp; ++i) aty += q.A[(size_t)i * np + j] * y[i];
    const double l = w.l[o + j], u = w.u[o + j];
    const bool fr = l < u;
    const double zl = w.zl[o + j], zu = w.zu[o + j];
    const double rd = fr ? qx + q.c[j] - aty - zl + zu : 0.0;
    w.rd[o + j] = rd;
    rdmax = fmax(rdmax, fabs(rd));
    if (fr) {
      comp += (x[j] - l) * zl + (u - x[j]) * zu;
      nf += 1.0;
    }
  }
  // rp = b - Ax (A' stored [np][mp]: coalesced across rows i)
  double rpmax = 0.0;
  for (int i = t; i < mp; i += kT) {
    double ax = 0.0;
    for (int j = 0; j < np; ++j) ax += q.AT[(size_t)j * mp + i] * x[j];
    const double rp = q.b[i] - ax;
    w.rp[oy + i] = rp;
    rpmax = fmax(rpmax, fabs(rp));
  }
  rdmax = block_max(rdmax, red);
  rpmax = block_max(rpmax, red);
  comp = block_sum(comp, red);
  nf = block_sum(nf, red);
  xmax = block_max(xmax, red);
  const double mu = comp / fmax(2.0 * nf, 1.0);
  // the primal tolerance scales with the rows' right-hand sides and the
  // iterate (slack columns of ranged rows carry the rows' activity while b
  // is 0: hs021), as oracle/qp_ipm.py
  const double tp = fmax(q.tp, kQpTolP * (1.0 + xmax));
  if (rpmax <= tp && rdmax <= q.td && mu <= kQpTolMu) {
    if (t == 0) {
      w.done[b] = 1;
      w.status[b] = 0;
    }
    return;
  }
  if (!assemble) return;
  // assemble: bit 0 K, bit 1 W (qp_potrf_ll builds its K tiles from Q and
  // qp_trsm_syrk_lds its W in LDS; the fallback kernels read these)
  // K = Q + diag(D), fixed rows/columns identity
  double *K = w.K + (size_t)b * np * np;
  for (size_t e = t; e < ((assemble & 1) ? (size_t)np * np : 0); e += kT) {
    const int i = (int)(e / np), j = (int)(e % np);
    const bool fi = w.l[o + i] < w.u[o + i], fj = w.l[o + j] < w.u[o + j];
    double v;
    if (!fi || !fj) {
      v = i == j ? 1.0 : 0.0;
    } else {
      v = q.Q[e];
      if (i == j) {
        const double sl = x[i] - w.l[o + i], su = w.u[o + i] - x[i];
        v += w.zl[o + i] / sl + w.zu[o + i] / su;
      }
    }
    K[e] = v;
  }
  // W = A' with the rows of fixed variables zeroed
  double *W = w.W + (size_t)b * np * mp;
  for (size_t e = t; e < ((assemble & 2) ? (size_t)np * mp : 0); e += kT) {
    const int j = (int)(e / mp);
    W[e] = w.l[o + j] < w.u[o + j] ? q.AT[e] : 0.0;
  }
}

// ---- blocked Cholesky K = L L' (lower), MFMA trailing update ---------------
__global__ __launch_bounds__(kT) void qp_potrf(QpWork w, int np) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (w.done[b]) return;
  double *K = w.K + (size_t)b * np * np;
  const int T = np / 16;
  double *D = sm;                 // [16][17] diagonal tile
  double *P = sm + 16 * 17;       // [T][16][16] panel (tiles kb..T-1 of column kb)
  for (int kb = 0; kb < T; ++kb) {
    const int c0 = kb * 16;
    // (1) factor the diagonal tile (wave 0)
    if (wave == 0) {
      for (int e = lane; e < 256; e += 64) D[(e >> 4) * 17 + (e & 15)] = K[(size_t)(c0 + (e >> 4)) * np + c0 + (e & 15)];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int c = 0; c < 16; ++c) {
        const double dd = sqrt(D[c * 17 + c]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) D[c * 17 + c] = dd;
        if (lane > c && lane < 16) D[lane * 17 + c] /= dd;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < 256; e += 64) {
          const int r = e >> 4, s = e & 15;
          if (s > c && r >= s) D[r * 17 + s] -= D[r * 17 + c] * D[s * 17 + c];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      for (int e = lane; e < 256; e += 64) {
        const int r = e >> 4, s = e & 15;
        const double v = s <= r ? D[r * 17 + s] : 0.0;
        P[e] = v;
        if (s <= r) K[(size_t)(c0 + r) * np + c0 + s] = v;
      }
    }
    __syncthreads();
    // (2) panel: rows below, X = A L_kk^-T by substitution (one row per thread)
    const int rows = np - c0 - 16;
    for (int r = t; r < rows; r += kT) {
      const int gr = c0 + 16 + r;
      double a[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = K[(size_t)gr * np + c0 + s];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        double v = a[s];
#pragma unroll
        for (int p = 0; p < s; ++p) v -= a[p] * D[s * 17 + p];
        a[s] = v / D[s * 17 + s];
      }
      const int ti = 1 + (r >> 4), rr = r & 15;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        P[ti * 256 + rr * 16 + s] = a[s];
        K[(size_t)gr * np + c0 + s] = a[s];
      }
    }
    __syncthreads();
    // (3) trailing update A_ij -= L_ik L_jk' for kb < j <= i < T on MFMA
    const int nt = T - kb - 1;
    const int npair = nt * (nt + 1) / 2;
    for (int pidx = wave; pidx < npair; pidx += 4) {
      // pair index -> (i, j), j <= i, row-major over the lower triangle
      int i = 0;
      while ((i + 1) * (i + 2) / 2 <= pidx) ++i;
      const int j = pidx - i * (i + 1) / 2;
      const int ti = i + 1, tj = j + 1;   // tile offsets inside the panel
      const int gi = (kb + ti) * 16, gj = (kb + tj) * 16;
      d4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[r] = K[(size_t)(gi + (lane >> 4) + 4 * r) * np + gj + (lane & 15)];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 4 * kk + (lane >> 4);
        const double av = -P[ti * 256 + (lane & 15) * 16 + k];   // A[row][k] = L_ik[row][k]
        const double bv = P[tj * 256 + (lane & 15) * 16 + k];    // B[k][col] = L_jk[col][k]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        K[(size_t)(gi + (lane >> 4) + 4 * r) * np + gj + (lane & 15)] = acc[r];
    }
    __syncthreads();
  }
}

// ---- left-looking blocked Cholesky, K assembled on the fly ------------------
// For column block j, every tile (i, j), i >= j, is K_ij - sum_k L_ik L_jk'
// accumulated on MFMA over all k at once (L_ik and L_jk streamed from
// HBM / L2, each 16x16 tile read as 16 rows of 128 contiguous bytes, four
// column blocks' loads in flight together; the LDS holds only the tiles of
// column block j: three workgroups fit a CU's LDS; at 5 waves per SIMD, 96
// VGPRs without spills, two run at once, which measured faster than three
// at 80 VGPRs with 9 spilled: 13.2 -> 11.6 ms per batch, profiles/r06aj),
// the diagonal tile is factored and the tiles
// below solved against it, and L_ij is written ONCE.  The right-looking
// kernel above read and wrote the whole trailing matrix for every column
// block (~9 MB per node at n = 304); this one reads ~2.3 MB of L and writes
// its lower triangle.  K_ij itself is never stored: Q (shared by the batch,
// L2-resident) plus the node's barrier diagonal, identity on fixed
// variables, as qp_prep assembles it.
constexpr int kPT = 512;   // 8 waves

size_t potrf_ll_lds(int np) {
  const int T = np / 16;
  return sizeof(double) * (16 * 17 + (size_t)T * 256 + 2 * (size_t)np);
}

__global__ __launch_bounds__(kPT, 5) void qp_potrf_ll(DevQP q, QpWork w) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (w.done[b]) return;
  const int np = q.np, T = np / 16;
  const size_t o = (size_t)b * np;
  double *K = w.K + (size_t)b * np * np;
  double *D = sm;                       // [16][17] diagonal tile
  double *P = D + 16 * 17;              // [T][16][16] tiles j..T-1 of column block j
  double *dg = P + (size_t)T * 256;     // [np] barrier diagonal zl/sl + zu/su
  double *fr = dg + np;                 // [np] 1 free, 0 fixed
  for (int j = t; j < np; j += kPT) {
    const double l = w.l[o + j], u = w.u[o + j], x = w.x[o + j];
    const bool f = l < u;
    fr[j] = f ? 1.0 : 0.0;
    dg[j] = f ? w.zl[o + j] / (x - l) + w.zu[o + j] / (u - x) : 0.0;
  }
  __syncthreads();
  const int row = lane & 15, kq = lane >> 4;
  for (int jb = 0; jb < T; ++jb) {
    const int c0 = jb * 16;
    // (1) tiles i >= jb: acc = K_ij - sum_{k < jb} L_ik L_jk'
    for (int i = jb + wave; i < T; i += kPT / 64) {
      const int gi = i * 16;
      d4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = gi + kq + 4 * r, gc = c0 + row;
        double v;
        if (fr[gr] == 0.0 || fr[gc] == 0.0) v = gr == gc ? 1.0 : 0.0;
        else v = gr == gc ? q.Q[(size_t)gr * np + gc] + dg[gr] : q.Q[(size_t)gr * np + gc];
        acc[r] = v;
      }
      // lane (row, kq) holds k = 16 kb + 4 kq + kk of A = L_ik and B = L_jk'
      const double *ap = K + (size_t)(gi + row) * np + 4 * kq;
      const double *bp = K + (size_t)(c0 + row) * np + 4 * kq;   // L_jk rows (L2 hits)
      // four column blocks' loads in flight before their 16 MFMAs (one
      // dependent HBM round trip per four blocks instead of per block)
      int kb = 0;
      for (; kb + 4 <= jb; kb += 4) {
        double4 a[4], bb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = *reinterpret_cast<const double4 *>(ap + (kb + u) * 16);
          bb[u] = *reinterpret_cast<const double4 *>(bp + (kb + u) * 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[u].x, bb[u].x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[u].y, bb[u].y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[u].z, bb[u].z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[u].w, bb[u].w, acc, 0, 0, 0);
        }
      }
      for (; kb < jb; ++kb) {
        const double4 a = *reinterpret_cast<const double4 *>(ap + kb * 16);
        const double4 bq = *reinterpret_cast<const double4 *>(bp + kb * 16);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.x, bq.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.y, bq.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.z, bq.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.w, bq.w, acc, 0, 0, 0);
      }
      double *pt = P + (size_t)(i - jb) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) pt[(kq + 4 * r) * 16 + row] = acc[r];
    }
    __syncthreads();
    // (2) factor the diagonal tile (wave 0)
    if (wave == 0) {
      for (int e = lane; e < 256; e += 64) D[(e >> 4) * 17 + (e & 15)] = P[e];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int c = 0; c < 16; ++c) {
        const double dd = sqrt(D[c * 17 + c]);
        const double rinv = 1.0 / dd;   // column 16 of the tile keeps 1 / L_cc
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          D[c * 17 + c] = dd;
          D[c * 17 + 16] = rinv;
        }
        if (lane > c && lane < 16) D[lane * 17 + c] *= rinv;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < 256; e += 64) {
          const int r = e >> 4, s2 = e & 15;
          if (s2 > c && r >= s2) D[r * 17 + s2] -= D[r * 17 + c] * D[s2 * 17 + c];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      for (int e = lane; e < 256; e += 64) {
        const int r = e >> 4, s2 = e & 15;
        if (s2 <= r) K[(size_t)(c0 + r) * np + c0 + s2] = D[r * 17 + s2];
      }
    }
    __syncthreads();
    // (3) the tiles below: X = P L_jj^-T, one row per thread, written once
    const int rows = np - c0 - 16;
#pragma unroll 1
    for (int r = t; r < rows; r += kPT) {
      const int gr = c0 + 16 + r;
      const double *pr = P + 256 + (size_t)(r >> 4) * 256 + (r & 15) * 16;
      double a[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) a[s2] = pr[s2];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        double v = a[s2];
        const double *dr = D + s2 * 17;   // re-read per row (LDS broadcast)
#pragma unroll
        for (int p2 = 0; p2 < s2; ++p2) v -= a[p2] * dr[p2];
        a[s2] = v * dr[16];   // 1 / L_ss (no division on the row's chain)
        // keep the tile's loads in their row: hoisting all 136 of them
        // (the compiler's choice) costs 250 VGPRs and spills at 8 waves
        asm volatile("" ::: "memory");
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) K[(size_t)gr * np + c0 + s2] = a[s2];
    }
    __syncthreads();
  }
}

// ---- W = L^-1 A' (blocked forward substitution) and M = W'W, MFMA ---------
__global__ __launch_bounds__(kT) void qp_trsm_syrk(QpWork w, int np, int mp) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (w.done[b]) return;
  const double *K = w.K + (size_t)b * np * np;
  double *W = w.W + (size_t)b * np * mp;
  double *M = w.M + (size_t)b * mp * mp;
  const int T = np / 16, CB = mp / 16;
  double *D = sm;              // [16][17]
  double *Wk = sm + 16 * 17;   // [16][mp]
  for (int kb = 0; kb < T; ++kb) {
    const int r0 = kb * 16;
    for (int e = t; e < 256; e += kT) D[(e >> 4) * 17 + (e & 15)] = K[(size_t)(r0 + (e >> 4)) * np + r0 + (e & 15)];
    __syncthreads();
    // solve the diagonal block rows: one column of W per thread
    for (int cidx = t; cidx < mp; cidx += kT) {
      double v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = W[(size_t)(r0 + r) * mp + cidx];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        double s = v[r];
#pragma unroll
        for (int p = 0; p < r; ++p) s -= D[r * 17 + p] * v[p];
        v[r] = s / D[r * 17 + r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        W[(size_t)(r0 + r) * mp + cidx] = v[r];
        Wk[r * mp + cidx] = v[r];
      }
    }
    __syncthreads();
    // W_i -= L_ik W_k for row tiles i > kb, column tiles cb (MFMA)
    const int ntiles = (T - kb - 1) * CB;
    for (int tix = wave; tix < ntiles; tix += 4) {
      const int i = kb + 1 + tix / CB, cb = tix % CB;
      d4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[r] = W[(size_t)(i * 16 + (lane >> 4) + 4 * r) * mp + cb * 16 + (lane & 15)];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 4 * kk + (lane >> 4);
        const double av = -K[(size_t)(i * 16 + (lane & 15)) * np + r0 + k];
        const double bv = Wk[k * mp + cb * 16 + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        W[(size_t)(i * 16 + (lane >> 4) + 4 * r) * mp + cb * 16 + (lane & 15)] = acc[r];
    }
    __syncthreads();
  }
  // W' copy for the step kernel's W dy (coalesced writes along j)
  double *WT = w.WT + (size_t)b * np * mp;
  for (size_t e = t; e < (size_t)np * mp; e += kT) {
    const int i = (int)(e / np), j = (int)(e % np);
    WT[e] = W[(size_t)j * mp + i];
  }
  // M = W'W: CB x CB output tiles, summed over the T row tiles of W
  for (int tix = wave; tix < CB * CB; tix += 4) {
    const int ib = tix / CB, jb = tix % CB;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int kb = 0; kb < T; ++kb) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = kb * 16 + 4 * kk + (lane >> 4);
        const double av = W[(size_t)k * mp + ib * 16 + (lane & 15)];   // A[i][k] = W[k][i]
        const double bv = W[(size_t)k * mp + jb * 16 + (lane & 15)];   // B[k][j] = W[k][j]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      M[(size_t)(ib * 16 + (lane >> 4) + 4 * r) * mp + jb * 16 + (lane & 15)] = acc[r];
  }
}

// ---- W = L^-1 A' and M = W'W with W resident in LDS -------------------------
// The whole W (np x mp, row stride mp + 1) lives in LDS (156 KB at n = 304,
// m = 61): assembled from A' there, solved block row by block row (diagonal
// block by substitution, the rows below on MFMA with L_ik streamed from HBM
// as 128-B row pieces), then written out once as W and W', and M = W'W
// taken from LDS on MFMA.  qp_trsm_syrk above read and wrote W's trailing
// rows in HBM for every block row.
size_t trsm_lds_bytes(int np, int mp) {
  return sizeof(double) * ((size_t)np * (mp + 1) + 16 * 17);
}

__global__ __launch_bounds__(kPT) void qp_trsm_syrk_lds(DevQP q, QpWork w) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (w.done[b]) return;
  const int np = q.np, mp = q.mp, ld = mp + 1, T = np / 16, CB = mp / 16;
  const size_t o = (size_t)b * np;
  const double *K = w.K + (size_t)b * np * np;
  double *Ws = sm;                 // [np][ld]
  double *D = Ws + (size_t)np * ld; // [16][17]
  for (int e = t; e < np * mp; e += kPT) {
    const int j = e / mp, i = e - j * mp;
    Ws[j * ld + i] = w.l[o + j] < w.u[o + j] ? q.AT[e] : 0.0;
  }
  const int row = lane & 15, kq = lane >> 4;
  for (int kb = 0; kb < T; ++kb) {
    const int r0 = kb * 16;
    for (int e = t; e < 256; e += kPT) {
      const double v = K[(size_t)(r0 + (e >> 4)) * np + r0 + (e & 15)];
      D[(e >> 4) * 17 + (e & 15)] = v;
      if ((e >> 4) == (e & 15)) D[(e >> 4) * 17 + 16] = 1.0 / v;
    }
    __syncthreads();
    // the diagonal block rows: one column per thread
    for (int cidx = t; cidx < mp; cidx += kPT) {
      double v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = Ws[(r0 + r) * ld + cidx];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        double s2 = v[r];
#pragma unroll
        for (int p2 = 0; p2 < r; ++p2) s2 -= D[r * 17 + p2] * v[p2];
        v[r] = s2 * D[r * 17 + 16];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) Ws[(r0 + r) * ld + cidx] = v[r];
    }
    __syncthreads();
    // W_i -= L_ik W_k for row tiles i > kb (MFMA; lane (row, kq) holds
    // k = 4 kq + kk of both operands)
    // a wave owns a row tile i and all CB column tiles of it: L_ik is loaded
    // once (and the next row tile's L prefetched) for CB x 4 MFMAs
    const int nrow = T - kb - 1;
    double4 an = make_double4(0.0, 0.0, 0.0, 0.0);
    if (wave < nrow)
      an = *reinterpret_cast<const double4 *>(K + (size_t)((kb + 1 + wave) * 16 + row) * np + r0 + 4 * kq);
    for (int ir = wave; ir < nrow; ir += kPT / 64) {
      const int i = kb + 1 + ir;
      const double4 a = an;
      if (ir + kPT / 64 < nrow)
        an = *reinterpret_cast<const double4 *>(K + (size_t)((i + kPT / 64) * 16 + row) * np + r0 + 4 * kq);
      for (int cb = 0; cb < CB; ++cb) {
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Ws[(i * 16 + kq + 4 * r) * ld + cb * 16 + row];
        const double *bp = Ws + (r0 + 4 * kq) * ld + cb * 16 + row;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.x, bp[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.y, bp[ld], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.z, bp[2 * ld], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.w, bp[3 * ld], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Ws[(i * 16 + kq + 4 * r) * ld + cb * 16 + row] = acc[r];
      }
    }
    __syncthreads();
  }
  // W (step: W'v, coalesced over i) and W' (step: W dy, coalesced over j)
  double *W = w.W + (size_t)b * np * mp;
  double *WT = w.WT + (size_t)b * np * mp;
  for (int e = t; e < np * mp; e += kPT) {
    const int j = e / mp, i = e - j * mp;
    W[e] = Ws[j * ld + i];
  }
  for (int e = t; e < np * mp; e += kPT) {
    const int i = e / np, j = e - i * np;
    WT[e] = Ws[j * ld + i];
  }
  // M = W'W: CB x CB tiles summed over np (A[i][k] = W[k][i], B[k][j] = W[k][j])
  double *M = w.M + (size_t)b * mp * mp;
  for (int tix = wave; tix < CB * CB; tix += kPT / 64) {
    const int ib = tix / CB, jb = tix % CB;
    d4 acc = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < np; k0 += 16) {
      const double *ap = Ws + (k0 + 4 * kq) * ld + ib * 16 + row;
      const double *bp = Ws + (k0 + 4 * kq) * ld + jb * 16 + row;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[0], bp[0], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[ld], bp[ld], acc1, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[2 * ld], bp[2 * ld], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ap[3 * ld], bp[3 * ld], acc1, 0, 0, 0);
    }
    acc += acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      M[(size_t)(ib * 16 + kq + 4 * r) * mp + jb * 16 + row] = acc[r];
  }
}

// ---- per-node Newton steps ---------------------------------------------------
// LDS of the step kernel: only what crosses threads (the triangular solves'
// vectors, the Schur factor and the solve pipeline's tiles); the per-column
// state (x, bounds, duals, residual, steps) lives in registers, J columns
// per thread (StepReg), so three workgroups share a CU.
struct StepSm {
  double *v, *dx;  // v: L^-1 r, then v + W dy in place; dx: the right-hand side, then the step
  double *tt, *dy; // dy aliases tt (wave 0 reads tt into registers, writes dy)
  double *Lm;     // lower triangle of [mp][mp], packed by rows (lt(i, j), j <= i)
  double *pre;    // [2][12][17] partial row sums (double-buffered)
  double *dt;     // [2][16][17] diagonal tiles of L
  double *xt;     // [2][16][17] the tiles between consecutive diagonal tiles
  double *red;    // [kT] (aliases pre: never live at the same time)
};
// packed lower-triangle index: the Schur factor of the m real rows takes
// m (m + 1) / 2 doubles of LDS instead of mp (mp + 1).  With the step's
// vectors aliased (the right-hand side in dx, v + W dy in place, dy over
// tt) a step workgroup takes 32.5 KB, so five fit a CU (two before).
// The padded rows of M are zero, so their dy is 0 and the real rows'
// factor and solves are the same operations as with the padding.
__device__ __forceinline__ int lt(int i, int j) { return i * (i + 1) / 2 + j; }

template <int J>
struct StepReg {   // column j = threadIdx.x + k * kT, k < J
  double x[J], l[J], u[J], zl[J], zu[J], rd[J], dzl[J], dzu[J], rl[J], ru[J];
  __device__ __forceinline__ bool fr(int k) const { return l[k] < u[k]; }
};

// The triangular solves with L, pipelined over 16-row blocks.  Block ib's
// row sums split into the columns solved before the previous block (a GEMV
// waves 1-3 compute while wave 0 is still substituting the previous block,
// 12 partial sums per row) and the previous block's 16 columns (the tile
// between the two diagonal tiles, prefetched into LDS by the same waves);
// wave 0 adds the two parts, then substitutes the diagonal tile (staged
// the same way) with v_readlane broadcasts.  One workgroup barrier per
// block; nothing from HBM is on wave 0's critical path.  pre / dt / xt are
// double-buffered [12|16][17] LDS tiles (StepSm::pre, dt, xt).
__device__ void fwd_L(const double *K, int np, const double *r, double *v, const StepSm &s) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int T = np / 16;
  if (wave > 0)
    for (int e = t - 64; e < 256; e += kT - 64) {
      const double v = K[(size_t)(e >> 4) * np + (e & 15)];
      s.dt[(e >> 4) * 17 + (e & 15)] = v;
      if ((e >> 4) == (e & 15)) s.dt[(e >> 4) * 17 + 16] = 1.0 / v;   // 1 / L_cc
    }
  __syncthreads();
  for (int ib = 0; ib < T; ++ib) {
    const int cur = ib & 1, nxt = cur ^ 1;
    const int r0 = ib * 16;
    if (wave == 0) {
      const int i = lane & 15, q = lane >> 4;
      double acc = 0.0;
      if (ib > 0) {
        const double *pre = s.pre + cur * 204, *xt = s.xt + cur * 272;
        for (int k = q; k < 28; k += 4)
          acc += k < 12 ? pre[k * 17 + i] : xt[i * 17 + (k - 12)] * v[r0 - 16 + (k - 12)];
      }
      acc += __shfl_xor(acc, 16, 64);
      acc += __shfl_xor(acc, 32, 64);
      const double *dt = s.dt + cur * 272;
      double val = lane < 16 ? r[r0 + lane] - acc : 0.0;
      double mine = 0.0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const double vc = rld(val, c) * dt[c * 17 + 16];   // v_readlane broadcast
        if (lane == c) mine = vc;
        if (lane > c && lane < 16) val -= dt[lane * 17 + c] * vc;
      }
      if (lane < 16) v[r0 + lane] = mine;
    } else if (ib + 1 < T) {
      const int tt = t - 64, rr = tt & 15, pq = tt >> 4, r1 = r0 + 16;
      double a = 0.0;
      for (int c = pq; c < r0; c += 12) a += K[(size_t)(r1 + rr) * np + c] * v[c];
      s.pre[nxt * 204 + pq * 17 + rr] = a;
      for (int e = tt; e < 256; e += kT - 64) {
        const int ei = e >> 4, ej = e & 15;
        const double dv = K[(size_t)(r1 + ei) * np + r1 + ej];
        s.dt[nxt * 272 + ei * 17 + ej] = dv;
        if (ei == ej) s.dt[nxt * 272 + ei * 17 + 16] = 1.0 / dv;
        s.xt[nxt * 272 + ei * 17 + ej] = K[(size_t)(r1 + ei) * np + r0 + ej];
      }
    }
    __syncthreads();
  }
}

// x = L^-T s (from the last row block up; the same pipeline over columns of L)
__device__ void bwd_LT(const double *K, int np, const double *sv, double *xo, const StepSm &s) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int T = np / 16;
  if (wave > 0) {
    const int d0 = (T - 1) * 16;
    for (int e = t - 64; e < 256; e += kT - 64) {
      const double v = K[(size_t)(d0 + (e >> 4)) * np + d0 + (e & 15)];
      s.dt[(e >> 4) * 17 + (e & 15)] = v;
      if ((e >> 4) == (e & 15)) s.dt[(e >> 4) * 17 + 16] = 1.0 / v;
    }
  }
  __syncthreads();
  for (int n = 0; n < T; ++n) {
    const int ib = T - 1 - n;
    const int cur = n & 1, nxt = cur ^ 1;
    const int r0 = ib * 16;
    if (wave == 0) {
      const int i = lane & 15, q = lane >> 4;
      double acc = 0.0;
      if (n > 0) {
        const double *pre = s.pre + cur * 204, *xt = s.xt + cur * 272;
        for (int k = q; k < 28; k += 4)
          acc += k < 12 ? pre[k * 17 + i] : xt[(k - 12) * 17 + i] * xo[r0 + 16 + (k - 12)];
      }
      acc += __shfl_xor(acc, 16, 64);
      acc += __shfl_xor(acc, 32, 64);
      const double *dt = s.dt + cur * 272;
      double val = lane < 16 ? sv[r0 + lane] - acc : 0.0;
      double mine = 0.0;
#pragma unroll
      for (int c = 15; c >= 0; --c) {
        const double xc = rld(val, c) * dt[c * 17 + 16];
        if (lane == c) mine = xc;
        if (lane < c) val -= dt[c * 17 + lane] * xc;
      }
      if (lane < 16) xo[r0 + lane] = mine;
    } else if (ib > 0) {
      // block ib - 1: rows k >= r0 + 16 of columns r0-16+rr (solved), the
      // tile rows [r0, r0+16) for the combine, its diagonal tile
      const int tt = t - 64, rr = tt & 15, pq = tt >> 4, c1 = r0 - 16;
      double a = 0.0;
      for (int k = r0 + 16 + pq; k < np; k += 12) a += K[(size_t)k * np + c1 + rr] * xo[k];
      s.pre[nxt * 204 + pq * 17 + rr] = a;
      for (int e = tt; e < 256; e += kT - 64) {
        const int ei = e >> 4, ej = e & 15;
        const double dv = K[(size_t)(c1 + ei) * np + c1 + ej];
        s.dt[nxt * 272 + ei * 17 + ej] = dv;
        if (ei == ej) s.dt[nxt * 272 + ei * 17 + 16] = 1.0 / dv;
        s.xt[nxt * 272 + ei * 17 + ej] = K[(size_t)(r0 + ei) * np + c1 + ej];
      }
    }
    __syncthreads();
  }
}

// (dx, dy) for right-hand side r1: v = L^-1 r1, Lm Lm' dy = rp - W'v,
// dx = L^-T (v + W dy), dx = 0 on fixed variables
template <int J>
__device__ void kkt_solve(const double *K, const double *W, const double *WT, const double *rp,
                          int np, int mp, int mr, const StepSm &s, const StepReg<J> &g,
                          const double *r1) {
  const int t = threadIdx.x;
  fwd_L(K, np, r1, s.v, s);
  // tt = rp - W'v (4 partial sums per column, coalesced over the column)
  {
    const int i = t & 63, pp = t >> 6;
    double acc = 0.0;
    if (i < mp)
      for (int j = pp; j < np; j += 4) acc += W[(size_t)j * mp + i] * s.v[j];
    s.red[t] = acc;
    __syncthreads();
    if (t < mp) s.tt[t] = rp[t] - (((s.red[t] + s.red[t + 64]) + s.red[t + 128]) + s.red[t + 192]);
    __syncthreads();
  }
  // dy = Lm^-T Lm^-1 tt (wave 0: lane t holds tt[t] in a register, the
  // pivot value broadcast by v_readlane; same operations in the same order
  // as the column sweeps through LDS they replace)
  if (t < 64) {
    double val = t < mr ? s.tt[t] : 0.0;
    for (int k = 0; k < mr; ++k) {
      const double zk = rld(val, k) / s.Lm[lt(k, k)];
      if (t == k) val = zk;
      else if (t > k && t < mr) val -= s.Lm[lt(t, k)] * zk;
    }
    for (int k = mr - 1; k >= 0; --k) {
      const double zk = rld(val, k) / s.Lm[lt(k, k)];
      if (t == k) val = zk;
      else if (t < k) val -= s.Lm[lt(k, t)] * zk;
    }
    if (t < mp) s.dy[t] = val;
  }
  __syncthreads();
  // v += W dy  (W' [mp][np] copy: coalesced across j; each j by one thread)
  for (int j = t; j < np; j += kT) {
    double acc = 0.0;
    for (int i = 0; i < mp; ++i) acc += WT[(size_t)i * np + j] * s.dy[i];
    s.v[j] = s.v[j] + acc;
  }
  __syncthreads();
  bwd_LT(K, np, s.v, s.dx, s);
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j < np && !g.fr(k)) s.dx[j] = 0.0;
  }
  __syncthreads();
}

template <int J>
__device__ double max_step(const StepSm &s, const StepReg<J> &g, int np, int which) {
  // which: 0 primal (sl with dx, su with -dx), 1 dual (zl with dzl, zu with dzu)
  double a = 1.0;
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = threadIdx.x + k * kT;
    if (j >= np || !g.fr(k)) continue;
    if (which == 0) {
      const double sl = g.x[k] - g.l[k], su = g.u[k] - g.x[k], d = s.dx[j];
      if (d < 0) a = fmin(a, -sl / d);
      if (-d < 0) a = fmin(a, -su / -d);
    } else {
      if (g.dzl[k] < 0) a = fmin(a, -g.zl[k] / g.dzl[k]);
      if (g.dzu[k] < 0) a = fmin(a, -g.zu[k] / g.dzu[k]);
    }
  }
  return block_min(a, s.red);
}

template <int J>
__global__ __launch_bounds__(kT) void qp_step(DevQP q, QpWork w) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x;
  if (w.done[b]) return;
  const int np = q.np, mp = q.mp, mr = q.m;
  StepSm s;
  double *p = sm;
  s.v = p; p += np; s.dx = p; p += np;
  s.tt = p; s.dy = p; p += mp;
  s.Lm = p; p += mr * (mr + 1) / 2; s.pre = p; p += 2 * 204; s.dt = p; p += 2 * 272;
  s.xt = p; p += 2 * 272;
  s.red = s.pre;   // kT = 256 <= 408 doubles
  // the right-hand side in dx: fwd_L consumes it before bwd_LT writes the
  // step there, and the corrector's right-hand side reads the predictor's
  // dx[j] in the same thread that overwrites it
  double *r1 = s.dx;
  const size_t o = (size_t)b * np, oy = (size_t)b * mp;
  const double *K = w.K + (size_t)b * np * np;
  const double *W = w.W + (size_t)b * np * mp;
  const double *WT = w.WT + (size_t)b * np * mp;
  const double *rp = w.rp + oy;
  StepReg<J> g;
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    const bool in = j < np;
    g.x[k] = in ? w.x[o + j] : 0.0;
    g.l[k] = in ? w.l[o + j] : 0.0;
    g.u[k] = in ? w.u[o + j] : 0.0;   // padding: l = u, a fixed column
    g.zl[k] = in ? w.zl[o + j] : 0.0;
    g.zu[k] = in ? w.zu[o + j] : 0.0;
    g.rd[k] = in ? w.rd[o + j] : 0.0;
  }
  // Lm = chol(M + reg I)
  const double *M = w.M + (size_t)b * mp * mp;
  double dmax = 0.0;
  for (int e = t; e < mp * mp; e += kT) {
    const int i = e / mp, j = e % mp;
    if (i < mr && j <= i) s.Lm[lt(i, j)] = M[e];
    if (i == j) dmax = fmax(dmax, M[e]);
  }
  dmax = block_max(dmax, s.red);
  for (int i = t; i < mr; i += kT) s.Lm[lt(i, i)] += kQpReg * (1.0 + dmax);
  __syncthreads();
  for (int k = 0; k < mr; ++k) {
    if (t == 0) s.Lm[lt(k, k)] = sqrt(s.Lm[lt(k, k)]);
    __syncthreads();
    const double dk = s.Lm[lt(k, k)];
    for (int i = k + 1 + t; i < mr; i += kT) s.Lm[lt(i, k)] /= dk;
    __syncthreads();
    const int nt = mr - k - 1;
    for (int e = t; e < nt * nt; e += kT) {
      const int i = k + 1 + e / nt, j = k + 1 + e % nt;
      if (j <= i) s.Lm[lt(i, j)] -= s.Lm[lt(i, k)] * s.Lm[lt(j, k)];
    }
    __syncthreads();
  }
  // mu
  double comp = 0.0, nf = 0.0;
#pragma unroll
  for (int k = 0; k < J; ++k)
    if (t + k * kT < np && g.fr(k)) {
      comp += (g.x[k] - g.l[k]) * g.zl[k] + (g.u[k] - g.x[k]) * g.zu[k];
      nf += 1.0;
    }
  comp = block_sum(comp, s.red);
  nf = block_sum(nf, s.red);
  const double mu = comp / fmax(2.0 * nf, 1.0);
  // predictor
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j < np) r1[j] = g.fr(k) ? -g.rd[k] - g.zl[k] + g.zu[k] : 0.0;
  }
  __syncthreads();
  kkt_solve<J>(K, W, WT, rp, np, mp, mr, s, g, r1);
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j >= np) continue;
    const bool fr = g.fr(k);
    const double sl = g.x[k] - g.l[k], su = g.u[k] - g.x[k];
    g.dzl[k] = fr ? -g.zl[k] - (g.zl[k] / sl) * s.dx[j] : 0.0;
    g.dzu[k] = fr ? -g.zu[k] + (g.zu[k] / su) * s.dx[j] : 0.0;
  }
  const double ap0 = max_step<J>(s, g, np, 0), ad0 = max_step<J>(s, g, np, 1);
  double ca = 0.0;
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j < np && g.fr(k)) {
      const double sl = g.x[k] - g.l[k], su = g.u[k] - g.x[k];
      ca += (sl + ap0 * s.dx[j]) * (g.zl[k] + ad0 * g.dzl[k]) +
            (su - ap0 * s.dx[j]) * (g.zu[k] + ad0 * g.dzu[k]);
    }
  }
  ca = block_sum(ca, s.red);
  const double mu_aff = ca / fmax(2.0 * nf, 1.0);
  const double ratio = mu > 0 ? mu_aff / mu : 0.0;
  const double sigma = mu > 0 ? ratio * ratio * ratio : 0.0;
  // corrector (r1 = s2 is rewritten: every read of the predictor's s2 ended
  // inside kkt_solve, before its closing barrier)
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j >= np) continue;
    const bool fr = g.fr(k);
    const double sl = g.x[k] - g.l[k], su = g.u[k] - g.x[k];
    const double rl = sigma * mu - sl * g.zl[k] - s.dx[j] * g.dzl[k];
    const double ru = sigma * mu - su * g.zu[k] + s.dx[j] * g.dzu[k];
    g.rl[k] = rl;
    g.ru[k] = ru;
    r1[j] = fr ? -g.rd[k] + rl / sl - ru / su : 0.0;
  }
  __syncthreads();
  kkt_solve<J>(K, W, WT, rp, np, mp, mr, s, g, r1);
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j >= np) continue;
    const bool fr = g.fr(k);
    const double sl = g.x[k] - g.l[k], su = g.u[k] - g.x[k];
    g.dzl[k] = fr ? (g.rl[k] - g.zl[k] * s.dx[j]) / sl : 0.0;
    g.dzu[k] = fr ? (g.ru[k] + g.zu[k] * s.dx[j]) / su : 0.0;
  }
  double ap = kQpStep * max_step<J>(s, g, np, 0), ad = kQpStep * max_step<J>(s, g, np, 1);
  ap = fmin(ap, 1.0);
  ad = fmin(ad, 1.0);
#pragma unroll
  for (int k = 0; k < J; ++k) {
    const int j = t + k * kT;
    if (j >= np) continue;
    w.x[o + j] = g.x[k] + ap * s.dx[j];
    w.zl[o + j] = g.zl[k] + ad * g.dzl[k];
    w.zu[o + j] = g.zu[k] + ad * g.dzu[k];
  }
  for (int i = t; i < mp; i += kT) w.y[oy + i] = w.y[oy + i] + ad * s.dy[i];
  if (t == 0) w.iters[b] += 1;
}

// ---- objective --------------------------------------------------------------
__global__ __launch_bounds__(kT) void qp_final(DevQP q, QpWork w) {
  __shared__ double red[kT];
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x;
  const int np = q.np;
  const size_t o = (size_t)b * np;
  double *x = sm;
  for (int j = t; j < np; j += kT) x[j] = w.x[o + j];
  __syncthreads();
  double f = 0.0;
  for (int j = t; j < np; j += kT) {
    double qx = 0.0;
    for (int i = 0; i < np; ++i) qx += q.Q[(size_t)i * np + j] * x[i];
    f += 0.5 * x[j] * qx + q.c[j] * x[j];
  }
  f = block_sum(f, red);
  const int st = w.status[b];
  if (t == 0) w.obj[b] = (st == 12 || st == 2) ? INFINITY : f + q.k;
}

}  // namespace

size_t qp_step_lds(int np, int mp, int m) {
  return sizeof(double) * ((size_t)2 * np + mp + (size_t)m * (m + 1) / 2 + 2 * 204 + 4 * 272);
}

hipError_t launch_qp_init(const DevQP &q, const QpWork &w, hipStream_t s) {
  hipLaunchKernelGGL(qp_init, dim3(w.B), dim3(kT), 0, s, q, w);
  return hipGetLastError();
}

hipError_t launch_qp_iteration(const DevQP &q, const QpWork &w, hipStream_t s, hipEvent_t *ev) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipSuccess;
    for (const void *f : {(const void *)qp_step<2>, (const void *)qp_step<4>,
                          (const void *)qp_step<8>})
      if (e == hipSuccess)
        e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void *)qp_potrf,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void *)qp_potrf_ll,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void *)qp_trsm_syrk_lds,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const size_t lds_prep = sizeof(double) * (size_t)(q.np + q.mp);
  const size_t lds_potrf = sizeof(double) * (16 * 17 + (size_t)(q.np / 16) * 256);
  const size_t lds_trsm = sizeof(double) * (16 * 17 + (size_t)16 * q.mp);
  // left-looking factorization while its row panel fits the LDS (n <= ~580)
  static const bool rl = getenv("MGPU_QP_RIGHT_LOOKING") != nullptr;   // A/B switch
  const bool ll = !rl && potrf_ll_lds(q.np) <= 160 * 1024;
  // W resident in LDS when it fits (n * (m + 1) <= ~20 000)
  const bool wl = ll && trsm_lds_bytes(q.np, q.mp) <= 160 * 1024;
  hipLaunchKernelGGL(qp_prep, dim3(w.B), dim3(kT), lds_prep, s, q, w, (ll ? 0 : 1) | (wl ? 0 : 2));
  if (ev) (void)hipEventRecord(ev[0], s);
  if (ll)
    hipLaunchKernelGGL(qp_potrf_ll, dim3(w.B), dim3(kPT), potrf_ll_lds(q.np), s, q, w);
  else
    hipLaunchKernelGGL(qp_potrf, dim3(w.B), dim3(kT), lds_potrf, s, w, q.np);
  if (ev) (void)hipEventRecord(ev[1], s);
  if (wl)
    hipLaunchKernelGGL(qp_trsm_syrk_lds, dim3(w.B), dim3(kPT), trsm_lds_bytes(q.np, q.mp), s, q,
                       w);
  else
    hipLaunchKernelGGL(qp_trsm_syrk, dim3(w.B), dim3(kT), lds_trsm, s, w, q.np, q.mp);
  if (ev) (void)hipEventRecord(ev[2], s);
  // the step's per-column registers: J columns per thread
  const size_t lstep = qp_step_lds(q.np, q.mp, q.m);
  if (q.np <= 2 * kT)
    hipLaunchKernelGGL(qp_step<2>, dim3(w.B), dim3(kT), lstep, s, q, w);
  else if (q.np <= 4 * kT)
    hipLaunchKernelGGL(qp_step<4>, dim3(w.B), dim3(kT), lstep, s, q, w);
  else if (q.np <= 8 * kT)
    hipLaunchKernelGGL(qp_step<8>, dim3(w.B), dim3(kT), lstep, s, q, w);
  else
    return hipErrorInvalidValue;   // n > 2048: mgpu_load_qp refuses it
  if (ev) (void)hipEventRecord(ev[3], s);
  return hipGetLastError();
}

hipError_t launch_qp_iteration_check(const DevQP &q, const QpWork &w, hipStream_t s) {
  hipLaunchKernelGGL(qp_prep, dim3(w.B), dim3(kT), sizeof(double) * (size_t)(q.np + q.mp), s, q,
                     w, 0);
  return hipGetLastError();
}

hipError_t launch_qp_final(const DevQP &q, const QpWork &w, hipStream_t s) {
  hipLaunchKernelGGL(qp_final, dim3(w.B), dim3(kT), sizeof(double) * q.np, s, q, w);
  return hipGetLastError();
}

}  // namespace mgpu
