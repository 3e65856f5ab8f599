/*
 * ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY.
 *
 * Bounded dual simplex with an explicit dense basis inverse: the CPU
 * restatement of what OsiLPEngine::solve asks Clp for
 * (src/interfaces/OsiLPEngine.cpp:571-652: resolve() = dual simplex from the
 * loaded warm basis, OsiDoDualInResolve hint :579-583, iteration limit
 * :561-569, status map :592-627).  Clp 1.17.9 itself is not vendored and
 * cannot be built here; this file restates the published
 * algorithm (textbook bounded dual simplex with Dantzig pricing, Harris
 * two-pass ratio test and artificial bounds for free columns), the same
 * algorithm the HIP kernel K3 runs.  Objective/status parity is pinned
 * against scipy's HiGHS and the AMPLOsiUT known answers
 * (src/testing/AMPLOsiUT.cpp:46-120).
 *
 * Problem: min c'x  s.t.  rlo <= A x <= rhi,  lb <= x <= ub.
 * Internally [A  -I] z = 0 with z = (x, r), r the row activities, so the
 * slack basis is B = -I.  Columns n..n+m-1 are the logicals.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define P_TOL 1e-7      /* primal feasibility (Clp default primal tolerance) */
#define D_TOL 1e-7      /* dual feasibility   (Clp default dual tolerance)   */
#define PIV_TOL 1e-9    /* smallest acceptable |alpha_rq| in the ratio test  */
#define ART_BOUND 1e7   /* first artificial box for free / half-free columns */
#define INF_B 1e30
/* pivots after which a solve switches to Bland's rule (anti-cycling; the GPU
 * kernels K3 / K3L use the same constant, kStallPivots in mgpu_internal.h) */
#define STALL_PIVOTS 128

enum { ST_LB = 0, ST_UB = 1, ST_FREE = 2, ST_BASIC = 3 };

typedef struct {
  const orc_lp *P;
  int N;               /* n + m */
  const double *lb, *ub;  /* structural node box */
  double *blo, *bhi;   /* working bounds of all N columns (may be artificial) */
  unsigned char *art;  /* 1 if the current bound of column j is artificial */
  double *z, *d;       /* values and reduced costs of all N columns */
  double *binv;        /* m x m row-major */
  int *head;           /* basic column of each row */
  signed char *st;
  double *rho, *alpha_r, *alpha_q, *w;
  /* product-form mode (K3P, repo:minotaur_amd/csrc/lp_pfi.hip): B^{-1} =
   * E_{k-1} ... E_0 B0^{-1} with B0^{-1} the shared warm-start inverse
   * (row-major, never modified) and at most pfi eta columns */
  int pfi, neta;
  const double *binv0;
  double *eta;         /* pfi x m: eta column t */
  int *prow;           /* pivot row of eta t */
  int *pq;             /* entering column of eta t (path warm starts) */
  double *u;           /* m: BTRAN work vector */
} lpw;

/* Basis warm start of the batched tree's warm mode 2 (bnb.cpp): the node's
 * basis is its parent's optimal basis, given as the parent's column statuses
 * st[N] and the k basic columns that are not basic in the shared root basis
 * B0 (path[0..k), ascending column index).  They replace, one after the
 * other, the root's basic columns that are nonbasic in st, each at the free
 * row with the largest |alpha| (lowest row on ties): a column replacement
 * with partial pivoting, one eta column each, exactly as a pivot makes it.
 * The reduced costs are recomputed from the basis.  A replacement whose
 * largest |alpha| is below COLREP_TOL falls back to the root basis.  k <= 0:
 * the root basis as is.  Out: the node's own final basis in the same form
 * (k_out = 0: children restart from the root).  ORC_PATH_PIVOTS (tuning A/B
 * only): the earlier form, the node's pivot path from the root basis. */
static int g_path_pivots = 0;
void orc_set_path_pivots(int on) { g_path_pivots = on; }
#define COLREP_TOL 1e-9
typedef struct {
  int k;
  const unsigned *path;
  const signed char *st;
  int inherit;         /* longest path handed to children */
  int *k_out;
  unsigned *path_out;
  signed char *st_out;
} orc_path;

static double bnd_lo(const orc_lp *P, const double *lb, int j) {
  return j < P->n ? lb[j] : P->rlo[j - P->n];
}
static double bnd_hi(const orc_lp *P, const double *ub, int j) {
  return j < P->n ? ub[j] : P->rhi[j - P->n];
}

/* alpha_r[j] = rho' a_j for column j of [A -I]. */
static double col_dot(const orc_lp *P, const double *v, int j) {
  if (j >= P->n) return -v[j - P->n];
  double s = 0.0;
  for (int k = P->colptr[j]; k < P->colptr[j + 1]; ++k) s += P->cval[k] * v[P->rowidx[k]];
  return s;
}

/* ---- product form (K3P): every loop below is the kernel's, in its order */

/* out <- E_{k-1} ... E_0 out.  E_t is the identity except column p = prow[t]
 * (= eta t): out_p' = eta_p out_p, out_i' = out_i + eta_i out_p. */
static void pfi_apply_etas(const lpw *W, double *out) {
  int m = W->P->m;
  for (int t = 0; t < W->neta; ++t) {
    const double *e = W->eta + (size_t) t * m;
    int p = W->prow[t];
    double vp = out[p];
    if (vp == 0.0) continue;
    for (int i = 0; i < m; ++i) out[i] = i == p ? e[i] * vp : out[i] + e[i] * vp;
  }
}

/* u' e_t as the product-form kernels sum it (wave.h wave_sum_sym): lane i
 * holds u_i e_i (K3PW: plus row i + 64's product); the 64 lanes are summed
 * by the symmetric DPP butterfly — pairs (i, i^1), (i, i^2), the half-row
 * mirror (i, i^7), the row mirror (i, i^15) — and the four 16-lane rows as
 * (r0 + r1) + (r2 + r3).  Every step adds a lane to its partner, so the
 * association is fixed and the same in every lane. */
static double eta_dot(int m, const double *u, const double *e) {
  double a[64], b[64];
  for (int i = 0; i < 64; ++i) {
    a[i] = i < m ? u[i] * e[i] : 0.0;
    if (m > 64) a[i] = a[i] + (i + 64 < m ? u[i + 64] * e[i + 64] : 0.0);
  }
  for (int i = 0; i < 64; ++i) b[i] = a[i] + a[i ^ 1];
  for (int i = 0; i < 64; ++i) a[i] = b[i] + b[i ^ 2];
  for (int i = 0; i < 64; ++i) b[i] = a[i] + a[i ^ 7];
  for (int i = 0; i < 64; ++i) a[i] = b[i] + b[i ^ 15];
  return (a[0] + a[16]) + (a[32] + a[48]);
}

/* rho = e_r' B^{-1}: u = e_r' E_{k-1} ... E_0 (each E_t' only rewrites
 * component prow[t] with u' e_t, eta_dot's order), then rho = u' B0^{-1}
 * over the nonzeros of u in ascending row order. */
static void pfi_btran(const lpw *W, int r, double *rho) {
  int m = W->P->m;
  double *u = W->u;
  for (int i = 0; i < m; ++i) u[i] = 0.0;
  u[r] = 1.0;
  for (int t = W->neta - 1; t >= 0; --t)
    u[W->prow[t]] = eta_dot(m, u, W->eta + (size_t) t * m);
  for (int k = 0; k < m; ++k) rho[k] = 0.0;
  for (int i = 0; i < m; ++i) {
    if (u[i] == 0.0) continue;
    for (int k = 0; k < m; ++k) rho[k] += u[i] * W->binv0[(size_t) i * m + k];
  }
}

/* out = B^{-1} a_j */
static void ftran_col(const lpw *W, int j, double *out) {
  const orc_lp *P = W->P;
  int m = P->m;
  if (W->pfi) {
    if (j >= P->n) {
      int i0 = j - P->n;
      for (int i = 0; i < m; ++i) out[i] = -W->binv0[(size_t) i * m + i0];
    } else {
      for (int i = 0; i < m; ++i) out[i] = 0.0;
      for (int k = P->colptr[j]; k < P->colptr[j + 1]; ++k) {
        int r = P->rowidx[k];
        double a = P->cval[k];
        for (int i = 0; i < m; ++i) out[i] += W->binv0[(size_t) i * m + r] * a;
      }
    }
    pfi_apply_etas(W, out);
    return;
  }
  if (j >= P->n) {
    int i0 = j - P->n;
    for (int i = 0; i < m; ++i) out[i] = -W->binv[i * m + i0];
    return;
  }
  for (int i = 0; i < m; ++i) out[i] = 0.0;
  for (int k = P->colptr[j]; k < P->colptr[j + 1]; ++k) {
    int r = P->rowidx[k];
    double a = P->cval[k];
    for (int i = 0; i < m; ++i) out[i] += W->binv[i * m + r] * a;
  }
}

/* Artificial bounds of a column whose true bound is infinite: a box of
 * half-width art_bound anchored at the finite side (or at 0). */
static double art_lo(double tlo_, double thi_, double art_bound) {
  (void) tlo_;
  return (thi_ < INF_B ? thi_ : 0.0) - art_bound;
}
static double art_hi(double tlo_, double thi_, double art_bound) {
  (void) thi_;
  return (tlo_ > -INF_B ? tlo_ : 0.0) + art_bound;
}

/* Choose the status of a nonbasic column from its reduced cost so the basis
 * is dual feasible; use an artificial bound when the needed side is
 * infinite. */
static void place_nonbasic(lpw *W, int j, double art_bound) {
  double lo = W->blo[j], hi = W->bhi[j], dj = W->d[j];
  int lo_f = lo > -INF_B, hi_f = hi < INF_B;
  if (lo_f && hi_f && lo == hi) { W->st[j] = ST_LB; W->z[j] = lo; return; }
  if (dj > D_TOL) {
    if (!lo_f) { W->blo[j] = art_lo(lo, hi, art_bound); W->art[j] |= 1; }
    W->st[j] = ST_LB; W->z[j] = W->blo[j];
  } else if (dj < -D_TOL) {
    if (!hi_f) { W->bhi[j] = art_hi(lo, hi, art_bound); W->art[j] |= 2; }
    W->st[j] = ST_UB; W->z[j] = W->bhi[j];
  } else {
    if (lo_f) { W->st[j] = ST_LB; W->z[j] = lo; }
    else if (hi_f) { W->st[j] = ST_UB; W->z[j] = hi; }
    else { W->st[j] = ST_FREE; W->z[j] = 0.0; }
  }
}

/* Widen every artificial bound to the new half-width (nonbasic columns keep
 * their status and move with their bound). */
static void grow_art(lpw *W, double art_bound) {
  for (int j = 0; j < W->N; ++j) {
    if (!W->art[j] || W->st[j] == ST_BASIC) continue;
    double tl = bnd_lo(W->P, W->lb, j), th = bnd_hi(W->P, W->ub, j);
    if (W->art[j] & 1) W->blo[j] = art_lo(tl, th, art_bound);
    if (W->art[j] & 2) W->bhi[j] = art_hi(tl, th, art_bound);
    if (W->st[j] == ST_LB) W->z[j] = W->blo[j];
    if (W->st[j] == ST_UB) W->z[j] = W->bhi[j];
  }
}

static void compute_duals(lpw *W) {
  const orc_lp *P = W->P;
  int m = P->m, N = W->N;
  /* y = c_B' B^{-1}; reuse rho as y */
  double *y = W->rho;
  /* product form: only called before the first pivot, where B^{-1} = B0^{-1} */
  const double *bi = W->pfi ? W->binv0 : W->binv;
  for (int k = 0; k < m; ++k) y[k] = 0.0;
  for (int i = 0; i < m; ++i) {
    int h = W->head[i];
    double cb = h < P->n ? P->c[h] : 0.0;
    if (cb != 0.0)
      for (int k = 0; k < m; ++k) y[k] += cb * bi[i * m + k];
  }
  for (int j = 0; j < N; ++j) {
    if (W->st[j] == ST_BASIC) { W->d[j] = 0.0; continue; }
    double cj = j < P->n ? P->c[j] : 0.0;
    W->d[j] = cj - col_dot(P, y, j);
  }
}

static void compute_primals(lpw *W) {
  const orc_lp *P = W->P;
  int m = P->m, N = W->N;
  double *w = W->w;
  for (int i = 0; i < m; ++i) w[i] = 0.0;
  for (int j = 0; j < N; ++j) {
    if (W->st[j] == ST_BASIC) continue;
    double zj = W->z[j];
    if (zj == 0.0) continue;
    if (j >= P->n) {
      w[j - P->n] -= zj;
    } else {
      for (int k = P->colptr[j]; k < P->colptr[j + 1]; ++k) w[P->rowidx[k]] += P->cval[k] * zj;
    }
  }
  if (W->pfi) {
    double *s = W->alpha_q;   /* free outside a pivot */
    for (int i = 0; i < m; ++i) {
      s[i] = 0.0;
      for (int k = 0; k < m; ++k) s[i] += W->binv0[(size_t) i * m + k] * w[k];
    }
    pfi_apply_etas(W, s);
    for (int i = 0; i < m; ++i) W->z[W->head[i]] = -s[i];
    return;
  }
  for (int i = 0; i < m; ++i) {
    double s = 0.0;
    for (int k = 0; k < m; ++k) s += W->binv[i * m + k] * w[k];
    W->z[W->head[i]] = -s;
  }
}

/* Gauss-Jordan inverse of the basis matrix (used when no inverse is
 * supplied with a warm basis).  Returns 0 if singular. */
static int invert_basis(lpw *W) {
  const orc_lp *P = W->P;
  int m = P->m;
  double *Bm = (double *) calloc((size_t) m * m, sizeof(double));
  double *I = W->binv;
  for (int i = 0; i < m; ++i) {
    int h = W->head[i];
    if (h >= P->n) {
      Bm[(h - P->n) * m + i] = -1.0;
    } else {
      for (int k = P->colptr[h]; k < P->colptr[h + 1]; ++k) Bm[P->rowidx[k] * m + i] = P->cval[k];
    }
  }
  for (int i = 0; i < m * m; ++i) I[i] = 0.0;
  for (int i = 0; i < m; ++i) I[i * m + i] = 1.0;
  for (int c = 0; c < m; ++c) {
    int piv = -1;
    double best = 0.0;
    for (int r = c; r < m; ++r)
      if (fabs(Bm[r * m + c]) > best) { best = fabs(Bm[r * m + c]); piv = r; }
    if (piv < 0 || best < 1e-12) { free(Bm); return 0; }
    if (piv != c) {
      for (int k = 0; k < m; ++k) {
        double t = Bm[c * m + k]; Bm[c * m + k] = Bm[piv * m + k]; Bm[piv * m + k] = t;
        t = I[c * m + k]; I[c * m + k] = I[piv * m + k]; I[piv * m + k] = t;
      }
    }
    double inv = 1.0 / Bm[c * m + c];
    for (int k = 0; k < m; ++k) { Bm[c * m + k] *= inv; I[c * m + k] *= inv; }
    for (int r = 0; r < m; ++r) {
      if (r == c) continue;
      double f = Bm[r * m + c];
      if (f == 0.0) continue;
      for (int k = 0; k < m; ++k) { Bm[r * m + k] -= f * Bm[c * m + k]; I[r * m + k] -= f * I[c * m + k]; }
    }
  }
  free(Bm);
  /* rows of B^{-1} are indexed by basis position: B^{-1} = (B)^-1 where
   * column i of B is the column of head[i]; I now holds B^{-1} with row i
   * <-> basis position i. */
  return 1;
}

/*
 * Solve one LP.  ws_head/ws_st/ws_binv: warm start in/out (NULL = slack
 * basis).  Returns an EngineStatus numeric (Types.h:152-166).
 */
/*
 * pfi > 0: product-form mode of K3P (only with a supplied warm-start inverse,
 * which becomes B0^{-1}): pivots append eta columns instead of updating a
 * dense inverse, and a solve that needs more than pfi pivots stops with
 * status -1 (the caller re-solves it densely, as the GPU does).  No
 * warm-start or dual output in this mode.
 */
/* y' = c_B' E_{k-1} ... E_0 B0^{-1} (pfi_btran's loops from u = c_B), then
 * d_j = c_j - y' a_j: the reduced costs of a path warm start. */
static void pfi_compute_duals(lpw *W) {
  const orc_lp *P = W->P;
  int m = P->m, N = W->N;
  double *u = W->u, *y = W->rho;
  for (int i = 0; i < m; ++i) u[i] = W->head[i] < P->n ? P->c[W->head[i]] : 0.0;
  for (int t = W->neta - 1; t >= 0; --t)
    u[W->prow[t]] = eta_dot(m, u, W->eta + (size_t) t * m);
  for (int k = 0; k < m; ++k) y[k] = 0.0;
  for (int i = 0; i < m; ++i) {
    if (u[i] == 0.0) continue;
    for (int k = 0; k < m; ++k) y[k] += u[i] * W->binv0[(size_t) i * m + k];
  }
  for (int j = 0; j < N; ++j) {
    if (W->st[j] == ST_BASIC) { W->d[j] = 0.0; continue; }
    double cj = j < P->n ? P->c[j] : 0.0;
    W->d[j] = cj - col_dot(P, y, j);
  }
}

/* The basis warm start's column replacement (see orc_path): returns 0, with
 * the root basis restored, when a replacement has no usable pivot. */
static int colrep_basis(lpw *W, const orc_path *path) {
  int m = W->P->m;
  int *h0 = (int *) malloc(sizeof(int) * (size_t) m);
  unsigned char *fr = (unsigned char *) malloc((size_t) m);
  int ok = 1;
  memcpy(h0, W->head, sizeof(int) * (size_t) m);
  for (int i = 0; i < m; ++i) fr[i] = path->st[W->head[i]] != ST_BASIC;
  for (int t = 0; t < path->k; ++t) {
    int q = (int) (path->path[t] & 0xFFFFu), r = -1;
    double best = 0.0;
    ftran_col(W, q, W->alpha_q);
    for (int i = 0; i < m; ++i)
      if (fr[i] && fabs(W->alpha_q[i]) > best) { best = fabs(W->alpha_q[i]); r = i; }
    if (r < 0 || best < COLREP_TOL) { ok = 0; break; }
    double inv = 1.0 / W->alpha_q[r];
    double *e = W->eta + (size_t) W->neta * m;
    for (int i = 0; i < m; ++i) e[i] = i == r ? inv : -W->alpha_q[i] * inv;
    W->pq[W->neta] = q;
    W->prow[W->neta++] = r;
    W->head[r] = q;
    fr[r] = 0;
  }
  if (!ok) {
    W->neta = 0;
    memcpy(W->head, h0, sizeof(int) * (size_t) m);
  }
  free(h0);
  free(fr);
  return ok;
}

/* K3P's reinversion when the eta file is full (lp_pfi.hip, the same rule):
 * the current basis as column replacements on B0 -- its basic columns
 * outside B0 in ascending order, from B0's head, exactly as a basis warm
 * start (colrep_basis) -- when that difference kb leaves an eighth of the
 * file free (kb <= pfi - max(1, pfi / 8)) and pivots + (pfi - kb) < 64 (the
 * product form never reaches the 64-pivot refresh).  Returns 1 when the etas
 * were rebuilt; 0 with the state untouched when the rule declines; -1 after
 * a failed replacement (no usable pivot) with the SHARED basis in place
 * (B0's head, the shared statuses and reduced costs): the dense
 * continuation then restarts from it, the pivots so far counted. */
static int reinvert(lpw *W, const int *hroot, const unsigned char *rootb,
                    const signed char *ws_st, const double *ws_d, int iters) {
  int m = W->P->m, N = W->N, kb = 0;
  int room = W->pfi / 8 > 1 ? W->pfi / 8 : 1;
  for (int j = 0; j < N; ++j) kb += W->st[j] == ST_BASIC && !rootb[j];
  if (kb > W->pfi - room || iters + (W->pfi - kb) >= 64) return 0;
  unsigned *cols = (unsigned *) malloc(sizeof(unsigned) * (size_t) (kb + 1));
  signed char *stc = (signed char *) malloc((size_t) N);
  for (int j = 0, t = 0; j < N; ++j) {
    stc[j] = W->st[j];
    if (W->st[j] == ST_BASIC && !rootb[j]) cols[t++] = (unsigned) j;
  }
  orc_path tp;
  memset(&tp, 0, sizeof tp);
  tp.k = kb;
  tp.path = cols;
  tp.st = stc;
  memcpy(W->head, hroot, sizeof(int) * (size_t) m);
  W->neta = 0;
  int ok = colrep_basis(W, &tp) ? 1 : -1;
  if (ok < 0) {   /* the shared basis (colrep_basis restored B0's head) */
    for (int j = 0; j < N; ++j) W->st[j] = ws_st[j] == ST_BASIC ? ST_LB : ws_st[j];
    for (int i = 0; i < m; ++i) W->st[W->head[i]] = ST_BASIC;
    for (int j = 0; j < N; ++j) W->d[j] = W->st[j] == ST_BASIC ? 0.0 : ws_d[j];
  }
  free(cols);
  free(stc);
  return ok;
}

static int dual_simplex_impl(const orc_lp *P, const double *lb, const double *ub,
                             int *ws_head, signed char *ws_st, double *ws_binv, double *ws_d,
                             int have_ws, int have_binv, int iter_limit, double *obj_out,
                             double *x_out, double *y_out, int *iters_out, int pfi,
                             int iter_base, const orc_path *path)
{
  int n = P->n, m = P->m, N = n + m;
  lpw W;
  int status = 12, iters = 0, fresh = 1;
  double art_bound = ART_BOUND;
  unsigned char *rootb = 0;   /* basis warm start output: basic in B0 */
  int *hroot = 0;             /* product form: B0's head */
  memset(&W, 0, sizeof W);
  W.P = P; W.N = N; W.lb = lb; W.ub = ub;
  if (pfi > 0 && have_ws && have_binv) {
    W.pfi = pfi;
    W.binv0 = ws_binv;
    W.eta = (double *) malloc(sizeof(double) * (size_t) pfi * m + 8);
    W.prow = (int *) malloc(sizeof(int) * (size_t) pfi + 4);
    W.pq = (int *) malloc(sizeof(int) * (size_t) pfi + 4);
    W.u = (double *) malloc(sizeof(double) * (size_t) m + 8);
  }
  W.blo = (double *) malloc(sizeof(double) * N);
  W.bhi = (double *) malloc(sizeof(double) * N);
  W.art = (unsigned char *) calloc((size_t) N, 1);
  W.z = (double *) calloc((size_t) N, sizeof(double));
  W.d = (double *) calloc((size_t) N, sizeof(double));
  W.binv = (double *) malloc(sizeof(double) * (size_t) m * m + 8);
  W.head = (int *) malloc(sizeof(int) * (size_t) m + 4);
  W.st = (signed char *) malloc((size_t) N);
  W.rho = (double *) malloc(sizeof(double) * (size_t) m + 8);
  W.w = (double *) malloc(sizeof(double) * (size_t) m + 8);
  W.alpha_r = (double *) malloc(sizeof(double) * (size_t) N);
  W.alpha_q = (double *) malloc(sizeof(double) * (size_t) m + 8);

  for (int j = 0; j < N; ++j) {
    W.blo[j] = bnd_lo(P, lb, j);
    W.bhi[j] = bnd_hi(P, ub, j);
    if (W.blo[j] < -INF_B) W.blo[j] = -INFINITY;
    if (W.bhi[j] > INF_B) W.bhi[j] = INFINITY;
  }
  /* quick primal-infeasibility check of the box itself */
  for (int j = 0; j < N; ++j) {
    if (W.blo[j] > W.bhi[j] + P_TOL) { status = 2; goto done; }
  }
  if (have_ws) {
    memcpy(W.head, ws_head, sizeof(int) * (size_t) m);
    for (int j = 0; j < N; ++j) W.st[j] = ST_LB;
    for (int i = 0; i < m; ++i) W.st[W.head[i]] = ST_BASIC;
    for (int j = 0; j < N; ++j) if (W.st[j] != ST_BASIC) W.st[j] = ws_st[j] == ST_BASIC ? ST_LB : ws_st[j];
    if (have_binv) {
      memcpy(W.binv, ws_binv, sizeof(double) * (size_t) m * m);
    } else if (!invert_basis(&W)) {
      have_ws = 0;
    }
  }
  if (!have_ws) {
    for (int i = 0; i < m; ++i) W.head[i] = n + i;
    for (int j = 0; j < N; ++j) W.st[j] = ST_LB;
    for (int i = 0; i < m; ++i) W.st[n + i] = ST_BASIC;
    for (int i = 0; i < m * m; ++i) W.binv[i] = 0.0;
    for (int i = 0; i < m; ++i) W.binv[i * m + i] = -1.0;
  }
  if ((path && path->k_out) || W.pfi) {
    rootb = (unsigned char *) calloc((size_t) N, 1);
    for (int i = 0; i < m; ++i) rootb[W.head[i]] = 1;
  }
  if (W.pfi) {   /* the shared basis's head, for a reinversion */
    hroot = (int *) malloc(sizeof(int) * (size_t) m + 4);
    memcpy(hroot, W.head, sizeof(int) * (size_t) m);
  }
  if (path && path->k > 0 && W.pfi && g_path_pivots) {
    /* pivot path: replay each pivot on the root basis (FTRAN of its entering
     * column through B0^{-1} and the etas so far) */
    for (int t = 0; t < path->k; ++t) {
      int q = (int) (path->path[t] & 0xFFFFu), r = (int) (path->path[t] >> 16);
      ftran_col(&W, q, W.alpha_q);
      double inv = 1.0 / W.alpha_q[r];
      double *e = W.eta + (size_t) W.neta * m;
      for (int i = 0; i < m; ++i) e[i] = i == r ? inv : -W.alpha_q[i] * inv;
      W.pq[W.neta] = q;
      W.prow[W.neta++] = r;
      W.head[r] = q;
    }
    for (int j = 0; j < N; ++j) W.st[j] = path->st[j];
    pfi_compute_duals(&W);
  } else if (path && path->k > 0 && W.pfi && path->k <= W.pfi && colrep_basis(&W, path)) {
    /* (a difference larger than the eta file: the shared basis, as K3P) */
    for (int j = 0; j < N; ++j) W.st[j] = path->st[j];
    pfi_compute_duals(&W);
  } else if (have_ws && have_binv == 1 && ws_d) {
    /* reduced costs depend only on the basis: reuse the parent's
     * (have_binv == 2: the inverse is given but ws_d, an output only, is for
     * another objective -- rebuilt below, as mgpu_lp_solve1 with ws_d = 0) */
    for (int j = 0; j < N; ++j) W.d[j] = W.st[j] == ST_BASIC ? 0.0 : ws_d[j];
  } else {
    compute_duals(&W);
  }
  /* nonbasic placement: keep the warm status when dual feasible */
  for (int j = 0; j < N; ++j) {
    if (W.st[j] == ST_BASIC) continue;
    double lo = W.blo[j], hi = W.bhi[j], dj = W.d[j];
    int keep = 0;
    if (have_ws) {
      if (W.st[j] == ST_LB && lo > -INF_B && dj >= -D_TOL) { W.z[j] = lo; keep = 1; }
      else if (W.st[j] == ST_UB && hi < INF_B && dj <= D_TOL) { W.z[j] = hi; keep = 1; }
      else if (lo == hi && lo > -INF_B) { W.st[j] = ST_LB; W.z[j] = lo; keep = 1; }
    }
    if (!keep) place_nonbasic(&W, j, art_bound);
  }
  compute_primals(&W);

  for (;;) {
    /* anti-cycling: past STALL_PIVOTS pivots of the solve (counted across
     * the product-form / dense split) Bland's rule replaces Dantzig pricing
     * and the Harris ratio test */
    const int bland = iter_base + iters >= STALL_PIVOTS;
    /* ---- pricing: most infeasible basic row (Dantzig); Bland: the
     * infeasible row whose basic column has the lowest index ---- */
    int r = -1;
    double best = 0.0, delta = 0.0;
    for (int i = 0; i < m; ++i) {
      int h = W.head[i];
      double v = W.z[h], inf = 0.0;
      if (v < W.blo[h] - P_TOL) inf = v - W.blo[h];
      else if (v > W.bhi[h] + P_TOL) inf = v - W.bhi[h];
      if (bland) {
        if (inf != 0.0 && (r < 0 || h < W.head[r])) { best = fabs(inf); r = i; delta = inf; }
      } else if (fabs(inf) > best) {
        best = fabs(inf); r = i; delta = inf;
      }
    }
    if (r < 0 && !fresh && !W.pfi) {
      /* confirm against freshly recomputed primal values (the product form,
       * K3P / K3PW: at most pfi etas since the recompute at the solve's
       * start, so its maintained values are declared final) */
      compute_primals(&W);
      fresh = 1;
      continue;
    }
    if (r < 0) {
      /* optimal for the (possibly artificially boxed) LP */
      int grow = 0;
      for (int j = 0; j < N; ++j) {
        if (W.st[j] == ST_BASIC || !W.art[j]) continue;
        if ((W.st[j] == ST_LB && (W.art[j] & 1)) || (W.st[j] == ST_UB && (W.art[j] & 2))) grow = 1;
      }
      if (!grow) { status = 0; break; }
      if (art_bound >= 1e13) { status = 4; break; }   /* ProvenUnbounded */
      art_bound *= 1e3;
      grow_art(&W, art_bound);
      compute_primals(&W);
      fresh = 1;
      continue;
    }
    if (iters >= iter_limit) { status = 6; break; }   /* EngineIterationLimit */
    int to_dense = 0;
    if (W.pfi && W.neta >= W.pfi && ws_d && m <= 64) {
      /* K3P's reinversion: the eta file rebuilt from B0, primal values
       * recomputed, reduced costs kept (-1: failed, the shared basis in
       * place for the dense continuation) */
      const int re = reinvert(&W, hroot, rootb, ws_st, ws_d, iters);
      if (re > 0) {
        compute_primals(&W);
        fresh = 1;
        continue;
      }
      to_dense = re < 0;
    }
    if (W.pfi && (W.neta >= W.pfi || to_dense)) {
      /* eta file full: the dense solve continues from this basis with its
       * explicit inverse E_{k-1}...E_0 B0^{-1}, column by column */
      for (int c = 0; c < m; ++c) {
        for (int i = 0; i < m; ++i) W.alpha_q[i] = W.binv0[(size_t) i * m + c];
        pfi_apply_etas(&W, W.alpha_q);
        for (int i = 0; i < m; ++i) W.binv[(size_t) i * m + c] = W.alpha_q[i];
      }
      status = -1;
      break;
    }
    /* ---- row r of B^{-1}, pivot row ---- */
    if (W.pfi) pfi_btran(&W, r, W.rho);
    else for (int k = 0; k < m; ++k) W.rho[k] = W.binv[r * m + k];
    double sigma = delta > 0 ? 1.0 : -1.0;
    /* ---- Harris two-pass ratio test ---- */
    double tmax = INFINITY;
    for (int j = 0; j < N; ++j) {
      W.alpha_r[j] = 0.0;
      if (W.st[j] == ST_BASIC) continue;
      if (W.blo[j] == W.bhi[j]) continue;             /* fixed: never enters */
      double a = col_dot(P, W.rho, j);
      W.alpha_r[j] = a;
      double at = sigma * a;
      double dj = W.d[j];
      if (W.st[j] == ST_LB && at > PIV_TOL) {
        double t = (fmax(dj, 0.0) + D_TOL) / at;
        if (t < tmax) tmax = t;
      } else if (W.st[j] == ST_UB && at < -PIV_TOL) {
        double t = (fmin(dj, 0.0) - D_TOL) / at;
        if (t < tmax) tmax = t;
      } else if (W.st[j] == ST_FREE && fabs(at) > PIV_TOL) {
        double t = D_TOL / fabs(at);
        if (t < tmax) tmax = t;
      }
    }
    if (tmax == INFINITY) {                             /* dual unbounded */
      int boxed = 0;
      for (int j = 0; j < N; ++j) if (W.st[j] != ST_BASIC && W.art[j]) boxed = 1;
      if (!boxed || art_bound >= 1e13) { status = 2; break; }
      art_bound *= 1e3;          /* the artificial box may be what is infeasible */
      grow_art(&W, art_bound);
      compute_primals(&W);
      fresh = 1;
      continue;
    }
    int q = -1;
    double qa = 0.0, tb = INFINITY;
    for (int j = 0; j < N; ++j) {
      if (W.st[j] == ST_BASIC || W.blo[j] == W.bhi[j]) continue;
      double at = sigma * W.alpha_r[j], dj = W.d[j], t;
      if (W.st[j] == ST_LB && at > PIV_TOL) t = fmax(dj, 0.0) / at;
      else if (W.st[j] == ST_UB && at < -PIV_TOL) t = fmin(dj, 0.0) / at;
      else if (W.st[j] == ST_FREE && fabs(at) > PIV_TOL) t = 0.0;
      else continue;
      if (bland) {   /* the exact minimum ratio, lowest column on ties */
        if (t < tb) { tb = t; q = j; }
      } else if (t <= tmax && fabs(at) > qa) {
        qa = fabs(at); q = j;
      }
    }
    if (q < 0) { status = 2; break; }
    /* ---- column q, steps ---- */
    ftran_col(&W, q, W.alpha_q);
    double arq = W.alpha_q[r];
    double theta_d = W.d[q] / W.alpha_r[q];
    /* keep the step sign consistent with the leaving direction */
    if (sigma * theta_d < 0) theta_d = 0.0;
    double theta_p = delta / arq;
    int p = W.head[r];
    /* duals */
    for (int j = 0; j < N; ++j) {
      if (W.st[j] == ST_BASIC) continue;
      W.d[j] -= theta_d * W.alpha_r[j];
    }
    W.d[q] = 0.0;
    W.d[p] = -theta_d;
    /* primals */
    for (int i = 0; i < m; ++i) W.z[W.head[i]] -= theta_p * W.alpha_q[i];
    double zq = W.z[q] + theta_p;
    /* leaving variable to its violated bound */
    if (delta < 0) { W.st[p] = ST_LB; W.z[p] = W.blo[p]; }
    else { W.st[p] = ST_UB; W.z[p] = W.bhi[p]; }
    /* basis */
    W.head[r] = q;
    W.st[q] = ST_BASIC;
    W.z[q] = zq;
    if (W.art[q]) {   /* basic columns keep their true (infinite) bounds */
      W.blo[q] = bnd_lo(P, lb, q) < -INF_B ? -INFINITY : bnd_lo(P, lb, q);
      W.bhi[q] = bnd_hi(P, ub, q) > INF_B ? INFINITY : bnd_hi(P, ub, q);
      W.art[q] = 0;
    }
    if (W.pfi) {
      /* eta column of this pivot: -alpha_q / alpha_rq, 1 / alpha_rq at r */
      double inv = 1.0 / arq;
      double *e = W.eta + (size_t) W.neta * m;
      for (int i = 0; i < m; ++i) e[i] = i == r ? inv : -W.alpha_q[i] * inv;
      W.pq[W.neta] = q;
      W.prow[W.neta++] = r;
    } else {
      double inv = 1.0 / arq;
      double *br = W.binv + (size_t) r * m;
      for (int k = 0; k < m; ++k) br[k] *= inv;
      for (int i = 0; i < m; ++i) {
        if (i == r) continue;
        double f = W.alpha_q[i];
        if (f == 0.0) continue;
        double *bi = W.binv + (size_t) i * m;
        for (int k = 0; k < m; ++k) bi[k] -= f * br[k];
      }
    }
    ++iters;
    fresh = 0;
    /* periodic refresh of primal values against drift */
    if (iters % 64 == 0) { compute_primals(&W); fresh = 1; }
  }
done:
  if (status == -1 && ws_head) {   /* product form: continuation state */
    memcpy(ws_head, W.head, sizeof(int) * (size_t) m);
    for (int j = 0; j < N; ++j) ws_st[j] = W.st[j];
    memcpy(ws_binv, W.binv, sizeof(double) * (size_t) m * m);
    if (ws_d) memcpy(ws_d, W.d, sizeof(double) * (size_t) N);
  }
  /* warm start out: the maintained reduced costs (reduced costs of fixed
   * nonbasic columns are not maintained: they can never enter) */
  if (ws_head && !W.pfi && (status == 0 || status == 6)) {
    memcpy(ws_head, W.head, sizeof(int) * (size_t) m);
    if (ws_st) for (int j = 0; j < N; ++j) ws_st[j] = W.st[j];
    if (ws_binv) memcpy(ws_binv, W.binv, sizeof(double) * (size_t) m * m);
    if (ws_d) memcpy(ws_d, W.d, sizeof(double) * (size_t) N);
  }
  if (status == 0 || status == 6) {
    double obj = 0.0;
    for (int j = 0; j < n; ++j) obj += P->c[j] * W.z[j];
    if (obj_out) *obj_out = obj;
    if (x_out) for (int j = 0; j < n; ++j) x_out[j] = W.z[j];
    if (y_out && !W.pfi) {
      compute_duals(&W);
      for (int i = 0; i < m; ++i) y_out[i] = W.rho[i];
    }
  } else if (obj_out) {
    *obj_out = status == 2 ? INFINITY : -INFINITY;
  }
  if (iters_out) *iters_out = iters;
  if (path && path->k_out && g_path_pivots) {
    /* the node's final path for its children: optimal in the product form
     * with a path no longer than `inherit`, else the root (k_out 0) */
    int ko = (W.pfi && status == 0 && W.neta > 0 && W.neta <= path->inherit) ? W.neta : 0;
    *path->k_out = ko;
    for (int t = 0; t < ko; ++t) path->path_out[t] = (unsigned) W.pq[t] | ((unsigned) W.prow[t] << 16);
    if (ko) for (int j = 0; j < N; ++j) path->st_out[j] = W.st[j];
  } else if (path && path->k_out) {
    /* the node's final basis for its children: optimal in the product form
     * and at most `inherit` basic columns outside B0, else the root (k_out 0) */
    int ko = 0;
    if (W.pfi && status == 0)
      for (int j = 0; j < N; ++j) ko += W.st[j] == ST_BASIC && !rootb[j];
    if (ko > path->inherit) ko = 0;
    *path->k_out = ko;
    for (int j = 0, t = 0; ko && j < N; ++j)
      if (W.st[j] == ST_BASIC && !rootb[j]) path->path_out[t++] = (unsigned) j;
    if (ko) for (int j = 0; j < N; ++j) path->st_out[j] = W.st[j];
  }
  free(rootb);
  free(hroot);
  free(W.blo); free(W.bhi); free(W.art); free(W.z); free(W.d); free(W.binv);
  free(W.head); free(W.st); free(W.rho); free(W.w); free(W.alpha_r); free(W.alpha_q);
  free(W.eta); free(W.prow); free(W.pq); free(W.u);
  return status;
}

int orc_dual_simplex(const orc_lp *P, const double *lb, const double *ub,
                     int *ws_head, signed char *ws_st, double *ws_binv, double *ws_d,
                     int have_ws, int have_binv, int iter_limit, double *obj_out,
                     double *x_out, double *y_out, int *iters_out)
{
  return dual_simplex_impl(P, lb, ub, ws_head, ws_st, ws_binv, ws_d, have_ws, have_binv,
                           iter_limit, obj_out, x_out, y_out, iters_out, 0, 0, 0);
}

/* What the GPU runs for one LP of a batch that shares its warm start: K3P
 * (product form, at most pfi etas: a path warm start's replayed pivots plus
 * the solve's own); an LP that fills the eta file is continued by the dense
 * K3 from K3P's basis, status and reduced costs with the explicit inverse
 * (iteration counts add up; the continuation's iteration limit and Bland
 * switch count the pivots already made).  ws_* are read-only here. */
static int solve_shared(const orc_lp *P, const double *lb, const double *ub, const int *ws_head,
                        const signed char *ws_st, const double *ws_binv, const double *ws_d,
                        int have_ws, int have_binv, int iter_limit, double *obj, double *x,
                        int *iters, int pfi, int *h, signed char *s, double *bi, double *dd,
                        const orc_path *path)
{
  int n = P->n, m = P->m, st;
  if (have_ws) {
    memcpy(h, ws_head, sizeof(int) * (size_t) m);
    memcpy(s, ws_st, (size_t) (n + m));
    if (ws_binv) memcpy(bi, ws_binv, sizeof(double) * (size_t) m * m);
    if (ws_d) memcpy(dd, ws_d, sizeof(double) * (size_t) (n + m));
  }
  if (!(pfi > 0 && have_ws && have_binv))
    return dual_simplex_impl(P, lb, ub, h, s, bi, ws_d ? dd : 0, have_ws, have_binv, iter_limit,
                             obj, x, 0, iters, 0, 0, 0);
  st = dual_simplex_impl(P, lb, ub, h, s, bi, ws_d ? dd : 0, 1, 1, iter_limit, obj, x, 0, iters,
                         pfi, 0, path);
  if (st == -1) {
    int it1 = *iters, it2 = 0;
    st = dual_simplex_impl(P, lb, ub, h, s, bi, ws_d ? dd : 0, 1, 1, iter_limit - it1, obj, x,
                           0, &it2, 0, it1, 0);
    *iters = it1 + it2;
  }
  return st;
}

/* Batch entry for ctypes: one LP per node box, optional shared warm start
 * (head/st/binv of e.g. the root optimum), OpenMP over nodes. */
#ifdef _OPENMP
#include <omp.h>
#endif
int orc_dual_simplex_batch(int n, int m, const int *colptr, const int *rowidx,
                           const double *cval, const double *c, const double *rlo,
                           const double *rhi, int B, const double *lb, const double *ub,
                           const int *ws_head, const signed char *ws_st,
                           const double *ws_binv, const double *ws_d, int iter_limit, int *status,
                           double *obj, double *x, int *iters, int nthreads, int pfi)
{
  orc_lp P;
  P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cval; P.c = c;
  P.rlo = rlo; P.rhi = rhi;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    int *h = (int *) malloc(sizeof(int) * (size_t) (m + 1));
    signed char *s = (signed char *) malloc((size_t) (n + m + 1));
    double *bi = (double *) malloc(sizeof(double) * (size_t) m * m + 8);
    double *dd = (double *) malloc(sizeof(double) * (size_t) (n + m) + 8);
#pragma omp for schedule(dynamic, 16)
    for (int b = 0; b < B; ++b) {
      int have = ws_head != 0;
      status[b] = solve_shared(&P, lb + (size_t) b * n, ub + (size_t) b * n, ws_head, ws_st,
                               ws_binv, ws_d, have, have && ws_binv != 0,
                               iter_limit, obj + b, x ? x + (size_t) b * n : 0, iters + b, pfi,
                               h, s, bi, dd, 0);
    }
    free(h); free(s); free(bi); free(dd);
  }
  return 0;
}

/* Path warm starts (the batched tree's warm mode 2): node b starts from the
 * shared root basis after its path of k_in[b] pivots (path_in[b][0..k),
 * stride MGPU path cap 32) with statuses st_in[b][n+m]; k_in[b] <= 0: the
 * root basis, statuses and reduced costs.  Out: status / objective / own
 * pivots and the node's final path for its children (k_out[b] = 0: restart
 * from the root). */
int orc_dual_simplex_path_batch(int n, int m, const int *colptr, const int *rowidx,
                                const double *cval, const double *c, const double *rlo,
                                const double *rhi, int B, const double *lb, const double *ub,
                                const int *ws_head, const signed char *ws_st,
                                const double *ws_binv, const double *ws_d, const int *k_in,
                                const unsigned *path_in, const signed char *st_in, int iter_limit,
                                int *status, double *obj, double *x, int *iters, int *k_out,
                                unsigned *path_out, signed char *st_out, int pfi, int inherit,
                                int nthreads)
{
  orc_lp P;
  P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cval; P.c = c;
  P.rlo = rlo; P.rhi = rhi;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    int *h = (int *) malloc(sizeof(int) * (size_t) (m + 1));
    signed char *s = (signed char *) malloc((size_t) (n + m + 1));
    double *bi = (double *) malloc(sizeof(double) * (size_t) m * m + 8);
    double *dd = (double *) malloc(sizeof(double) * (size_t) (n + m) + 8);
#pragma omp for schedule(dynamic, 16)
    for (int b = 0; b < B; ++b) {
      orc_path pa;
      pa.k = k_in[b];
      pa.path = path_in + (size_t) b * ORC_PATH_MAX;
      pa.st = st_in + (size_t) b * (n + m);
      pa.inherit = inherit;
      pa.k_out = k_out + b;
      pa.path_out = path_out + (size_t) b * ORC_PATH_MAX;
      pa.st_out = st_out + (size_t) b * (n + m);
      k_out[b] = 0;
      status[b] = solve_shared(&P, lb + (size_t) b * n, ub + (size_t) b * n, ws_head, ws_st,
                               ws_binv, ws_d, 1, 1, iter_limit, obj + b,
                               x ? x + (size_t) b * n : 0, iters + b, pfi, h, s, bi, dd, &pa);
    }
    free(h); free(s); free(bi); free(dd);
  }
  return 0;
}

/* Root solve that also returns the optimal warm start (head, st, binv). */
int orc_dual_simplex_root(int n, int m, const int *colptr, const int *rowidx,
                          const double *cval, const double *c, const double *rlo,
                          const double *rhi, const double *lb, const double *ub,
                          int iter_limit, int *head, signed char *st, double *binv,
                          double *dred, double *obj, double *x, double *y, int *iters)
{
  orc_lp P;
  P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cval; P.c = c;
  P.rlo = rlo; P.rhi = rhi;
  return orc_dual_simplex(&P, lb, ub, head, st, binv, dred, 0, 0, iter_limit, obj, x, y,
                          iters);
}

/* Bound LPs (QuadHandler::getBndByLP_, QuadHandler.cpp:2080-2109, inside
 * tightenLP_ :2218-2297): LP b minimises sign[b] * x[col[b]] over the same
 * box, warm-started from one basis (head/st/binv row-major); the reduced
 * costs of each objective are rebuilt from that basis (compute_duals). */
int orc_lp_bound_batch(int n, int m, const int *colptr, const int *rowidx, const double *cval,
                       const double *rlo, const double *rhi, const double *lb, const double *ub,
                       int B, const int *col, const double *sign, const int *ws_head,
                       const signed char *ws_st, const double *ws_binv, int iter_limit,
                       int *status, double *obj, double *x, int *iters, int nthreads, int pfi)
{
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    int *h = (int *) malloc(sizeof(int) * (size_t) (m + 1));
    signed char *s = (signed char *) malloc((size_t) (n + m + 1));
    double *bi = (double *) malloc(sizeof(double) * (size_t) m * m + 8);
    double *c = (double *) calloc((size_t) n + 1, sizeof(double));
    double *dd = (double *) malloc(sizeof(double) * (size_t) (n + m) + 8);
    orc_lp P;
    P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cval; P.c = c;
    P.rlo = rlo; P.rhi = rhi;
#pragma omp for schedule(dynamic, 4)
    for (int b = 0; b < B; ++b) {
      const int have = ws_head != 0;
      c[col[b]] = sign[b];
      status[b] = solve_shared(&P, lb, ub, ws_head, ws_st, ws_binv, 0, have, have, iter_limit,
                               obj + b, x ? x + (size_t) b * n : 0, iters + b, pfi, h, s, bi,
                               dd, 0);
      c[col[b]] = 0.0;
    }
    free(h); free(s); free(bi); free(c); free(dd);
  }
  return 0;
}

/* Per-node warm starts in and out (the batched tree's parent warm starts,
 * NodeIncRelaxer.cpp:146-150): node b starts from ws_*[b] (head [m], st
 * [n+m], binv [m][m] row-major, d [n+m]) and leaves its final basis in
 * wo_*[b]; dense explicit-inverse arithmetic (the K3 / K3L restatement). */
int orc_dual_simplex_nodes(int n, int m, const int *colptr, const int *rowidx,
                           const double *cval, const double *c, const double *rlo,
                           const double *rhi, int B, const double *lb, const double *ub,
                           const int *ws_head, const signed char *ws_st, const double *ws_binv,
                           const double *ws_d, int iter_limit, int *status, double *obj,
                           double *x, int *iters, int *wo_head, signed char *wo_st,
                           double *wo_binv, double *wo_d, int nthreads)
{
  orc_lp P;
  P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cval; P.c = c;
  P.rlo = rlo; P.rhi = rhi;
  if (nthreads < 1) nthreads = 1;
  const size_t N = (size_t) (n + m), mm = (size_t) m * m;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 8)
  for (int b = 0; b < B; ++b) {
    /* ws_head NULL: slack basis; ws_d NULL: reduced costs rebuilt for c */
    int have = ws_head != 0;
    status[b] = solve_shared(&P, lb + (size_t) b * n, ub + (size_t) b * n,
                             have ? ws_head + (size_t) b * m : 0,
                             have ? ws_st + (size_t) b * N : 0,
                             have ? ws_binv + (size_t) b * mm : 0,
                             have && ws_d ? ws_d + (size_t) b * N : 0, have, have, iter_limit,
                             obj + b,
                             x ? x + (size_t) b * n : 0, iters + b, 0, wo_head + (size_t) b * m,
                             wo_st + (size_t) b * N, wo_binv + (size_t) b * mm,
                             wo_d + (size_t) b * N, 0);
  }
  return 0;
}

/* Per-node rows (mgpu_lp_solve_rows, the glob path: QuadHandler::upSqCon_ /
 * upBilCon_ rewrite rows at every node, QuadHandler.cpp:3322-3419, and
 * OsiLPEngine::changeConstraint loads them, OsiLPEngine.cpp:206-243): node b
 * solves the loaded LP with matrix entries csc_pos[k] (CSC order) set to
 * vals[b][coef_src[k]] (|v| <= 1e-9 -> 0, LinearFunction::addTerm) and the
 * bounds of rows row[q] from vals[b][lo_src[q]] / vals[b][hi_src[q]] (-1 =
 * loaded), from the warm basis head/st (shared when ws_shared, else per node)
 * with the inverse rebuilt for the node's matrix (invert_basis, singular ->
 * slack basis) and compute_duals; dense arithmetic (K3R + K3). */
/* K3R's column-replacement refactor (m <= 64): the node's basis differs
 * from the warm (root) basis only in the basic structural columns whose
 * rewritten entries changed; starting from the root inverse binv0
 * (row-major), each such basis position i (ascending) takes its node column
 * a' by one product-form update: alpha = B^-1 a' (ftran_col's order), row i
 * / alpha_i, row r -= alpha_r row i (the dual simplex's update).  Returns 0
 * when some |alpha_i| < 1e-12 (the caller refactors from scratch). */
static int colrep_refactor(int n, int m, const int *colptr, const int *rowidx,
                           const double *cval0, const double *cv, const int *head,
                           const double *binv0, double *bi, double *alpha)
{
  memcpy(bi, binv0, sizeof(double) * (size_t) m * m);
  for (int i = 0; i < m; ++i) {
    int h = head[i], changed = 0;
    if (h >= n) continue;
    for (int k = colptr[h]; k < colptr[h + 1]; ++k)
      if (cv[k] != cval0[k]) { changed = 1; break; }
    if (!changed) continue;
    for (int r = 0; r < m; ++r) alpha[r] = 0.0;
    for (int k = colptr[h]; k < colptr[h + 1]; ++k) {
      int r = rowidx[k];
      double a = cv[k];
      for (int ii = 0; ii < m; ++ii) alpha[ii] += bi[(size_t) ii * m + r] * a;
    }
    if (fabs(alpha[i]) < 1e-12) return 0;
    double inv = 1.0 / alpha[i];
    double *br = bi + (size_t) i * m;
    for (int k = 0; k < m; ++k) br[k] *= inv;
    for (int ii = 0; ii < m; ++ii) {
      if (ii == i) continue;
      double f = alpha[ii];
      if (f == 0.0) continue;
      double *bj = bi + (size_t) ii * m;
      for (int k = 0; k < m; ++k) bj[k] -= f * br[k];
    }
  }
  return 1;
}

int orc_dual_simplex_rows(int n, int m, const int *colptr, const int *rowidx,
                          const double *cval, const double *c, const double *rlo,
                          const double *rhi, int B, const double *lb, const double *ub,
                          const double *vals, int stride, int ncoef, const int *csc_pos,
                          const int *coef_src, int nrow, const int *row, const int *lo_src,
                          const int *hi_src, const int *ws_head, const signed char *ws_st,
                          int ws_shared, int iter_limit, int *status, double *obj, double *x,
                          int *iters, int nthreads, const double *ws_binv0, int *head_out,
                          signed char *st_out)
{
  const int nnz = colptr[n];
  const size_t N = (size_t) (n + m);
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    double *cv = (double *) malloc(sizeof(double) * (size_t) (nnz + 1));
    double *lo = (double *) malloc(sizeof(double) * (size_t) (m + 1));
    double *hi = (double *) malloc(sizeof(double) * (size_t) (m + 1));
    int *h = (int *) malloc(sizeof(int) * (size_t) (m + 1));
    signed char *s = (signed char *) malloc(N + 1);
    double *bi = (double *) malloc(sizeof(double) * (size_t) m * m + 8);
    double *al = (double *) malloc(sizeof(double) * (size_t) (m + 1));
    orc_lp P;
    P.n = n; P.m = m; P.colptr = colptr; P.rowidx = rowidx; P.cval = cv; P.c = c;
    P.rlo = lo; P.rhi = hi;
#pragma omp for schedule(dynamic, 8)
    for (int b = 0; b < B; ++b) {
      const double *rec = vals + (size_t) b * stride;
      memcpy(cv, cval, sizeof(double) * (size_t) nnz);
      memcpy(lo, rlo, sizeof(double) * (size_t) m);
      memcpy(hi, rhi, sizeof(double) * (size_t) m);
      for (int k = 0; k < ncoef; ++k) {
        double v = rec[coef_src[k]];
        cv[csc_pos[k]] = fabs(v) <= 1e-9 ? 0.0 : v;
      }
      for (int q = 0; q < nrow; ++q) {
        if (lo_src[q] >= 0) lo[row[q]] = rec[lo_src[q]];
        if (hi_src[q] >= 0) hi[row[q]] = rec[hi_src[q]];
      }
      const int have = ws_head != 0;
      const size_t wb = ws_shared ? 0 : (size_t) b;
      /* the root inverse given (shared warm start, m <= 64): the basis by
       * column replacement, reduced costs rebuilt (have_binv 2); else the
       * Gauss-Jordan refactor of invert_basis */
      int hb = 0;
      if (have && ws_binv0 && ws_shared &&
          colrep_refactor(n, m, colptr, rowidx, cval, cv, ws_head, ws_binv0, bi, al))
        hb = 2;
      if (hb) {
        memcpy(h, ws_head, sizeof(int) * (size_t) m);
        memcpy(s, ws_st, N);
      }
      status[b] = hb ? dual_simplex_impl(&P, lb + (size_t) b * n, ub + (size_t) b * n, h, s, bi,
                                         0, 1, 2, iter_limit, obj + b,
                                         x ? x + (size_t) b * n : 0, 0, iters + b, 0, 0, 0)
                     : solve_shared(&P, lb + (size_t) b * n, ub + (size_t) b * n,
                                    have ? ws_head + wb * m : 0, have ? ws_st + wb * N : 0, 0, 0,
                                    have, 0, iter_limit, obj + b, x ? x + (size_t) b * n : 0,
                                    iters + b, 0, h, s, bi, 0, 0);
      /* the final basis (the glob tree's parent-basis warm starts) */
      if (head_out) memcpy(head_out + (size_t) b * m, h, sizeof(int) * (size_t) m);
      if (st_out) memcpy(st_out + (size_t) b * N, s, N);
    }
    free(cv); free(lo); free(hi); free(h); free(s); free(bi); free(al);
  }
  return 0;
}
