// K5 — batched QP relaxation solve with an MFMA KKT block, gfx950
// (QPDRelaxer / BqpdEngine, src/interfaces/
// BqpdEngine.cpp:449-534).
//
//   min 1/2 x'Qx + c'x + k   s.t.  A x = b,  l <= x <= u   (node box)
//
// Mehrotra predictor-corrector interior point, one node per workgroup.  The
// Newton system is the KKT block [Q + D, A'; A, 0] (D = Z_l/S_l + Z_u/S_u),
// reduced through its Schur complement:
//   K = Q + D = L L'        qp_potrf   blocked right-looking Cholesky:
//                                       16x16 tiles, trailing updates on
//                                       v_mfma_f64_16x16x4_f64
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
  double rdmax = 0.0, comp = 0.0, nf = 0.0;
  for (int j = t; j < np; j += kT) {
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
  const double mu = comp / fmax(2.0 * nf, 1.0);
  if (rpmax <= q.tp && rdmax <= q.td && mu <= kQpTolMu) {
    if (t == 0) {
      w.done[b] = 1;
      w.status[b] = 0;
    }
    return;
  }
  if (!assemble) return;
  // K = Q + diag(D), fixed rows/columns identity
  double *K = w.K + (size_t)b * np * np;
  for (size_t e = t; e < (size_t)np * np; e += kT) {
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
  for (size_t e = t; e < (size_t)np * mp; e += kT) {
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

// ---- per-node Newton steps ---------------------------------------------------
struct StepSm {
  double *x, *l, *u, *zl, *zu, *rd, *v, *dx, *s2, *dzl, *dzu, *rl, *ru;
  double *y, *rp, *tt, *dy;
  double *Lm;     // [mp][mp+1]
  double *part;   // [16][17] partial sums
  double *dt;     // [16][17] diagonal tile of L
  double *red;    // [kT]
};

// v = L^-1 r, blocked by 16 rows: a GEMV of the block's rows against the
// solved part (256 threads, 16 partial sums per row), then the diagonal
// tile (staged in LDS) by a 16-lane substitution with v_readlane
// broadcasts.  dt: [16][17] LDS tile.
__device__ void fwd_L(const double *K, int np, const double *r, double *v, double *part,
                      double *dt) {
  const int t = threadIdx.x, rr = t & 15, pp = t >> 4;
  const int T = np / 16;
  for (int ib = 0; ib < T; ++ib) {
    const int r0 = ib * 16;
    double acc = 0.0;
    for (int c = pp; c < r0; c += 16) acc += K[(size_t)(r0 + rr) * np + c] * v[c];
    part[pp * 17 + rr] = acc;
    dt[(t >> 4) * 17 + (t & 15)] = K[(size_t)(r0 + (t >> 4)) * np + r0 + (t & 15)];
    __syncthreads();
    if (t < 64) {
      double val = 0.0;
      if (t < 16) {
        double sum = 0.0;
        for (int q2 = 0; q2 < 16; ++q2) sum += part[q2 * 17 + t];
        val = r[r0 + t] - sum;
      }
      double mine = 0.0;
      for (int c = 0; c < 16; ++c) {
        const double vc = __shfl(val, c, 64) / dt[c * 17 + c];
        if (t == c) mine = vc;
        if (t > c && t < 16) val -= dt[t * 17 + c] * vc;
      }
      if (t < 16) v[r0 + t] = mine;
    }
    __syncthreads();
  }
}

// x = L^-T s (blocked, from the last row block up; same scheme)
__device__ void bwd_LT(const double *K, int np, const double *s, double *xo, double *part,
                       double *dt) {
  const int t = threadIdx.x, rr = t & 15, pp = t >> 4;
  const int T = np / 16;
  for (int ib = T - 1; ib >= 0; --ib) {
    const int r0 = ib * 16;
    double acc = 0.0;
    for (int k = r0 + 16 + pp; k < np; k += 16) acc += K[(size_t)k * np + r0 + rr] * xo[k];
    part[pp * 17 + rr] = acc;
    dt[(t >> 4) * 17 + (t & 15)] = K[(size_t)(r0 + (t >> 4)) * np + r0 + (t & 15)];
    __syncthreads();
    if (t < 64) {
      double val = 0.0;
      if (t < 16) {
        double sum = 0.0;
        for (int q2 = 0; q2 < 16; ++q2) sum += part[q2 * 17 + t];
        val = s[r0 + t] - sum;
      }
      double mine = 0.0;
      for (int c = 15; c >= 0; --c) {
        const double xc = __shfl(val, c, 64) / dt[c * 17 + c];
        if (t == c) mine = xc;
        if (t < c) val -= dt[c * 17 + t] * xc;
      }
      if (t < 16) xo[r0 + t] = mine;
    }
    __syncthreads();
  }
}

// (dx, dy) for right-hand side r1: v = L^-1 r1, Lm Lm' dy = rp - W'v,
// dx = L^-T (v + W dy), dx = 0 on fixed variables
__device__ void kkt_solve(const double *K, const double *W, const double *WT, int np, int mp,
                          const StepSm &s, const double *r1) {
  const int t = threadIdx.x;
  fwd_L(K, np, r1, s.v, s.part, s.dt);
  // tt = rp - W'v (4 partial sums per column, coalesced over the column)
  {
    const int i = t & 63, pp = t >> 6;
    double acc = 0.0;
    if (i < mp)
      for (int j = pp; j < np; j += 4) acc += W[(size_t)j * mp + i] * s.v[j];
    s.red[t] = acc;
    __syncthreads();
    if (t < mp) s.tt[t] = s.rp[t] - (((s.red[t] + s.red[t + 64]) + s.red[t + 128]) + s.red[t + 192]);
    __syncthreads();
  }
  // dy = Lm^-T Lm^-1 tt (wave 0, column sweeps in LDS)
  if (t < 64) {
    const int mpad = mp + 1;
    for (int k = 0; k < mp; ++k) {
      const double zk = s.tt[k] / s.Lm[k * mpad + k];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (t == k) s.tt[k] = zk;
      if (t > k && t < mp) s.tt[t] -= s.Lm[t * mpad + k] * zk;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    for (int k = mp - 1; k >= 0; --k) {
      const double zk = s.tt[k] / s.Lm[k * mpad + k];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (t == k) s.dy[k] = zk;
      if (t < k) s.tt[t] -= s.Lm[k * mpad + t] * zk;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
  // s2 = v + W dy  (W' [mp][np] copy: coalesced across j)
  for (int j = t; j < np; j += kT) {
    double acc = 0.0;
    for (int i = 0; i < mp; ++i) acc += WT[(size_t)i * np + j] * s.dy[i];
    s.s2[j] = s.v[j] + acc;
  }
  __syncthreads();
  bwd_LT(K, np, s.s2, s.dx, s.part, s.dt);
  for (int j = t; j < np; j += kT)
    if (!(s.l[j] < s.u[j])) s.dx[j] = 0.0;
  __syncthreads();
}

__device__ double max_step(const StepSm &s, int np, int which) {
  // which: 0 primal (sl with dx, su with -dx), 1 dual (zl with dzl, zu with dzu)
  double a = 1.0;
  for (int j = threadIdx.x; j < np; j += kT) {
    if (!(s.l[j] < s.u[j])) continue;
    if (which == 0) {
      const double sl = s.x[j] - s.l[j], su = s.u[j] - s.x[j], d = s.dx[j];
      if (d < 0) a = fmin(a, -sl / d);
      if (-d < 0) a = fmin(a, -su / -d);
    } else {
      if (s.dzl[j] < 0) a = fmin(a, -s.zl[j] / s.dzl[j]);
      if (s.dzu[j] < 0) a = fmin(a, -s.zu[j] / s.dzu[j]);
    }
  }
  return block_min(a, s.red);
}

__global__ __launch_bounds__(kT) void qp_step(DevQP q, QpWork w) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, t = threadIdx.x;
  if (w.done[b]) return;
  const int np = q.np, mp = q.mp, mpad = mp + 1;
  StepSm s;
  double *p = sm;
  s.x = p; p += np; s.l = p; p += np; s.u = p; p += np; s.zl = p; p += np; s.zu = p; p += np;
  s.rd = p; p += np; s.v = p; p += np; s.dx = p; p += np; s.s2 = p; p += np;
  s.dzl = p; p += np; s.dzu = p; p += np; s.rl = p; p += np; s.ru = p; p += np;
  s.y = p; p += mp; s.rp = p; p += mp; s.tt = p; p += mp; s.dy = p; p += mp;
  s.Lm = p; p += mp * mpad; s.part = p; p += 16 * 17; s.dt = p; p += 16 * 17;
  s.red = p; p += kT;
  double *r1 = s.s2;  // reuse: r1 is consumed by fwd_L before s2 is written
  const size_t o = (size_t)b * np, oy = (size_t)b * mp;
  const double *K = w.K + (size_t)b * np * np;
  const double *W = w.W + (size_t)b * np * mp;
  const double *WT = w.WT + (size_t)b * np * mp;
  for (int j = t; j < np; j += kT) {
    s.x[j] = w.x[o + j];
    s.l[j] = w.l[o + j];
    s.u[j] = w.u[o + j];
    s.zl[j] = w.zl[o + j];
    s.zu[j] = w.zu[o + j];
    s.rd[j] = w.rd[o + j];
  }
  for (int i = t; i < mp; i += kT) {
    s.y[i] = w.y[oy + i];
    s.rp[i] = w.rp[oy + i];
  }
  // Lm = chol(M + reg I)
  const double *M = w.M + (size_t)b * mp * mp;
  double dmax = 0.0;
  for (int e = t; e < mp * mp; e += kT) {
    const int i = e / mp, j = e % mp;
    s.Lm[i * mpad + j] = M[e];
    if (i == j) dmax = fmax(dmax, M[e]);
  }
  dmax = block_max(dmax, s.red);
  for (int i = t; i < mp; i += kT) s.Lm[i * mpad + i] += kQpReg * (1.0 + dmax);
  __syncthreads();
  for (int k = 0; k < mp; ++k) {
    if (t == 0) s.Lm[k * mpad + k] = sqrt(s.Lm[k * mpad + k]);
    __syncthreads();
    const double dk = s.Lm[k * mpad + k];
    for (int i = k + 1 + t; i < mp; i += kT) s.Lm[i * mpad + k] /= dk;
    __syncthreads();
    const int nt = mp - k - 1;
    for (int e = t; e < nt * nt; e += kT) {
      const int i = k + 1 + e / nt, j = k + 1 + e % nt;
      if (j <= i) s.Lm[i * mpad + j] -= s.Lm[i * mpad + k] * s.Lm[j * mpad + k];
    }
    __syncthreads();
  }
  // mu
  double comp = 0.0, nf = 0.0;
  for (int j = t; j < np; j += kT)
    if (s.l[j] < s.u[j]) {
      comp += (s.x[j] - s.l[j]) * s.zl[j] + (s.u[j] - s.x[j]) * s.zu[j];
      nf += 1.0;
    }
  comp = block_sum(comp, s.red);
  nf = block_sum(nf, s.red);
  const double mu = comp / fmax(2.0 * nf, 1.0);
  // predictor
  for (int j = t; j < np; j += kT)
    r1[j] = s.l[j] < s.u[j] ? -s.rd[j] - s.zl[j] + s.zu[j] : 0.0;
  __syncthreads();
  kkt_solve(K, W, WT, np, mp, s, r1);
  for (int j = t; j < np; j += kT) {
    const bool fr = s.l[j] < s.u[j];
    const double sl = s.x[j] - s.l[j], su = s.u[j] - s.x[j];
    s.dzl[j] = fr ? -s.zl[j] - (s.zl[j] / sl) * s.dx[j] : 0.0;
    s.dzu[j] = fr ? -s.zu[j] + (s.zu[j] / su) * s.dx[j] : 0.0;
  }
  __syncthreads();
  const double ap0 = max_step(s, np, 0), ad0 = max_step(s, np, 1);
  double ca = 0.0;
  for (int j = t; j < np; j += kT)
    if (s.l[j] < s.u[j]) {
      const double sl = s.x[j] - s.l[j], su = s.u[j] - s.x[j];
      ca += (sl + ap0 * s.dx[j]) * (s.zl[j] + ad0 * s.dzl[j]) +
            (su - ap0 * s.dx[j]) * (s.zu[j] + ad0 * s.dzu[j]);
    }
  ca = block_sum(ca, s.red);
  const double mu_aff = ca / fmax(2.0 * nf, 1.0);
  const double ratio = mu > 0 ? mu_aff / mu : 0.0;
  const double sigma = mu > 0 ? ratio * ratio * ratio : 0.0;
  // corrector
  for (int j = t; j < np; j += kT) {
    const bool fr = s.l[j] < s.u[j];
    const double sl = s.x[j] - s.l[j], su = s.u[j] - s.x[j];
    const double rl = sigma * mu - sl * s.zl[j] - s.dx[j] * s.dzl[j];
    const double ru = sigma * mu - su * s.zu[j] + s.dx[j] * s.dzu[j];
    s.rl[j] = rl;
    s.ru[j] = ru;
    r1[j] = fr ? -s.rd[j] + rl / sl - ru / su : 0.0;
  }
  __syncthreads();
  kkt_solve(K, W, WT, np, mp, s, r1);
  for (int j = t; j < np; j += kT) {
    const bool fr = s.l[j] < s.u[j];
    const double sl = s.x[j] - s.l[j], su = s.u[j] - s.x[j];
    s.dzl[j] = fr ? (s.rl[j] - s.zl[j] * s.dx[j]) / sl : 0.0;
    s.dzu[j] = fr ? (s.ru[j] + s.zu[j] * s.dx[j]) / su : 0.0;
  }
  __syncthreads();
  double ap = kQpStep * max_step(s, np, 0), ad = kQpStep * max_step(s, np, 1);
  ap = fmin(ap, 1.0);
  ad = fmin(ad, 1.0);
  for (int j = t; j < np; j += kT) {
    w.x[o + j] = s.x[j] + ap * s.dx[j];
    w.zl[o + j] = s.zl[j] + ad * s.dzl[j];
    w.zu[o + j] = s.zu[j] + ad * s.dzu[j];
  }
  for (int i = t; i < mp; i += kT) w.y[oy + i] = s.y[i] + ad * s.dy[i];
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

size_t qp_step_lds(int np, int mp) {
  return sizeof(double) * ((size_t)13 * np + 4 * mp + (size_t)mp * (mp + 1) + 2 * 16 * 17 + kT);
}

hipError_t launch_qp_init(const DevQP &q, const QpWork &w, hipStream_t s) {
  hipLaunchKernelGGL(qp_init, dim3(w.B), dim3(kT), 0, s, q, w);
  return hipGetLastError();
}

hipError_t launch_qp_iteration(const DevQP &q, const QpWork &w, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void *)qp_step,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void *)qp_potrf,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const size_t lds_prep = sizeof(double) * (size_t)(q.np + q.mp);
  const size_t lds_potrf = sizeof(double) * (16 * 17 + (size_t)(q.np / 16) * 256);
  const size_t lds_trsm = sizeof(double) * (16 * 17 + (size_t)16 * q.mp);
  hipLaunchKernelGGL(qp_prep, dim3(w.B), dim3(kT), lds_prep, s, q, w, 1);
  hipLaunchKernelGGL(qp_potrf, dim3(w.B), dim3(kT), lds_potrf, s, w, q.np);
  hipLaunchKernelGGL(qp_trsm_syrk, dim3(w.B), dim3(kT), lds_trsm, s, w, q.np, q.mp);
  hipLaunchKernelGGL(qp_step, dim3(w.B), dim3(kT), qp_step_lds(q.np, q.mp), s, q, w);
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
