/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of Minotaur's quadratic node FBBT,
 * QuadHandler::presolveNode (/root/reference/src/base/QuadHandler.cpp:
 * 1204-1269) and everything it calls, with the interval primitives of
 * Operations.cpp:100-246.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product path never does.
 *
 * Parity pin: checked bit-for-bit (bounds, verdicts, mod logs, secant /
 * McCormick row state) against the reference itself, oracle/_ref/
 * libref_fbbt.so (oracle/ref/ref_quad.cpp), through tests/golden/quad_*.npz.
 *
 * Problem layout (orc_qspec, shared with the reference driver): variables
 * 0..nv0-1 are the original problem's, the rest are the aux y's of
 * y = x^2 (squares, ascending x: the LinSqrMap order, QuadHandler.h:54) and
 * y = x0*x1 (bilinears, ascending (x0, x1): CompareLinBil, LinBil.cpp:51-62).
 * The original quadratic constraints (tightenQuad_) are term lists in
 * ascending variable order (VariableGroup / CompareVariablePair,
 * Types.cpp:30-66).  Compiled with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* QuadHandler.cpp:60-67 */
#define A_TOL 1e-6
#define B_TOL 1e-8
#define R_TOL 1e-7
/* LinearFunction.cpp:22, :89-95: |a| <= 1e-9 is not stored in a row */
#define LF_TOL 1e-9
/* safety cap on the unbounded propagation loop (QuadHandler.cpp:1215) */
#define PROP_CAP 100000

static double smin(double a, double b) { return (b < a) ? b : a; } /* std::min */
static double smax(double a, double b) { return (a < b) ? b : a; } /* std::max */

/* Operations.cpp:122-177 BoundsOnProduct */
void orc_bounds_on_product(int zxiz, double l0, double u0, double l1, double u1, double *lb,
                           double *ub)
{
  double p;
  if (fabs(l1) <= 1e-10 && fabs(u1) <= 1e-10) {
    p = l1; l1 = l0; l0 = p;
    p = u1; u1 = u0; u0 = p;
  }
  if (fabs(l0) <= 1e-10 && fabs(u0) <= 1e-10) {
    if (zxiz) {
      *lb = 0.0;
      *ub = 0.0;
    } else {
      *lb = l1 == -INFINITY ? -INFINITY : 0.0;
      *ub = u1 == INFINITY ? INFINITY : 0.0;
    }
  } else if ((l1 == -INFINITY && u1 == INFINITY) || (l0 == -INFINITY && u0 == INFINITY)) {
    *lb = -INFINITY;
    *ub = INFINITY;
  } else {
    double lo, hi;
    p = l0 * l1;
    if (isnan(p)) p = -INFINITY;
    lo = p;
    hi = p;
    p = u0 * l1;
    if (isnan(p)) p = INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    p = u0 * u1;
    if (isnan(p)) p = -INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    p = l0 * u1;
    if (isnan(p)) p = INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    *lb = lo;
    *ub = hi;
  }
}

/* Operations.cpp:180-210 BoundsOnRecip */
void orc_bounds_on_recip(double l0, double u0, double *lb, double *ub)
{
  if (fabs(u0) < 1e-10 && fabs(l0) < 1e-10) {
    *lb = -INFINITY;
    *ub = INFINITY;
  } else if (l0 < -1e-10 && u0 > 1e-10) {
    *lb = -INFINITY;
    *ub = INFINITY;
  } else if (fabs(u0) < 1e-10 && l0 < 0) {
    *lb = -INFINITY;
    *ub = 1.0 / l0;
  } else if (fabs(l0) < 1e-10 && u0 < 0) {
    *lb = 1.0 / u0;
    *ub = INFINITY;
  } else {
    *lb = 1.0 / u0;
    *ub = 1.0 / l0;
  }
}

/* Operations.cpp:100-106 BoundsOnDiv */
void orc_bounds_on_div(double l0, double u0, double l1, double u1, double *lb, double *ub)
{
  double tl, tu;
  orc_bounds_on_recip(l1, u1, &tl, &tu);
  orc_bounds_on_product(0, l0, u0, tl, tu, lb, ub);
}

/* Operations.cpp:213-227 BoundsOnSquare */
void orc_bounds_on_square(double l1, double u1, double *lb, double *ub)
{
  if (u1 < 0.) {
    *lb = u1 * u1;
    *ub = l1 * l1;
  } else if (l1 > 0.) {
    *lb = l1 * l1;
    *ub = u1 * u1;
  } else {
    *lb = 0.;
    *ub = smax(l1 * l1, u1 * u1);
  }
}

typedef struct {
  const orc_qspec *S;
  double *lb, *ub;
  int nmods, mod_cap;
  int *mod_kind, *mod_idx;
  double *mod_v1, *mod_v2;
  unsigned char *isq; /* tightenQuad_'s accumulated qvars (by index) */
  double *fl, *fu;    /* fwdLb / fwdUb */
} qnode;

static void qpush(qnode *s, int kind, int idx, double v1, double v2)
{
  if (s->mod_kind && s->nmods < s->mod_cap) {
    s->mod_kind[s->nmods] = kind;
    s->mod_idx[s->nmods] = idx;
    s->mod_v1[s->nmods] = v1;
    s->mod_v2[s->nmods] = v2;
  }
  s->nmods++;
}

/* QuadHandler::updatePBounds_ (relaxation form), QuadHandler.cpp:3248-3320.
 * Returns -1 when the new bounds cross the old ones by more than bTol. */
static int update_pbounds(qnode *s, int v, double lb, double ub, int *changed)
{
  const int t = s->S->vtype[v];
  const double L = s->lb[v], U = s->ub[v];
  if (t == 0 || t == 1 || t == 2 || t == 3) { /* Binary, Integer, ImplBin, ImplInt */
    ub = floor(ub);
    lb = ceil(lb);
  }
  if (lb > U + B_TOL || ub < L - B_TOL) return -1;
  if (lb > L + B_TOL && ub < U - B_TOL && (L == -INFINITY || lb > L + R_TOL * fabs(L)) &&
      (U == INFINITY || ub < U - R_TOL * fabs(U))) {
    *changed = 1;
    s->lb[v] = lb;
    s->ub[v] = ub;
    qpush(s, 2, v, lb, ub); /* VarBoundMod2 */
  } else if (lb > L + B_TOL && (L == -INFINITY || lb > L + R_TOL * fabs(L))) {
    *changed = 1;
    s->lb[v] = lb;
    qpush(s, 0, v, lb, 0.0);
  } else if (ub < U - B_TOL && (U == INFINITY || ub < U - R_TOL * fabs(U))) {
    *changed = 1;
    s->ub[v] = ub;
    qpush(s, 1, v, ub, 0.0);
  }
  return 0;
}

/* propSqrBnds_ (relaxation form), QuadHandler.cpp:1361-1395 */
static int prop_sqr(qnode *s, int x, int y, int *changed)
{
  double lb, ub;
  orc_bounds_on_square(s->lb[x], s->ub[x], &lb, &ub);
  if (update_pbounds(s, y, lb, ub, changed) < 0) return 1;
  if (s->ub[y] > B_TOL) {
    ub = sqrt(s->ub[y]);
    lb = -ub;
    if (s->lb[x] > -sqrt(s->lb[y]) + B_TOL) lb = sqrt(s->lb[y]);
    if (update_pbounds(s, x, lb, ub, changed) < 0) return 1;
  } else if (s->ub[y] < -B_TOL) {
    return 1;
  } else {
    if (update_pbounds(s, x, 0.0, 0.0, changed) < 0) return 1;
  }
  return 0;
}

/* propBilBnds_ (relaxation form), QuadHandler.cpp:1271-1301 */
static int prop_bil(qnode *s, int x0, int x1, int y, int *changed)
{
  double lb, ub;
  orc_bounds_on_product(1, s->lb[x0], s->ub[x0], s->lb[x1], s->ub[x1], &lb, &ub);
  if (update_pbounds(s, y, lb, ub, changed) < 0) return 1;
  orc_bounds_on_div(s->lb[y], s->ub[y], s->lb[x0], s->ub[x0], &lb, &ub);
  if (update_pbounds(s, x1, lb, ub, changed) < 0) return 1;
  orc_bounds_on_div(s->lb[y], s->ub[y], s->lb[x1], s->ub[x1], &lb, &ub);
  if (update_pbounds(s, x0, lb, ub, changed) < 0) return 1;
  return 0;
}

/* calcUpperUnivar_, QuadHandler.cpp:1707-1720: max of a x^2 + b x on [lx, ux] */
static double calc_upper_univar(double a, double b, double lx, double ux)
{
  double u = smax(lx * (a * lx + b), ux * (a * ux + b));
  const double sh = b / 2.0, t = sh / (-a);
  if (t > lx) {
    const double r = (-2.0 * a) * ux;
    if (r > b) u = smax(u, sh * t);
  }
  return u;
}

/* getTermBnds_(v, coef), QuadHandler.cpp:1723-1733 */
static void term_bnds_lin(const qnode *s, int v, double c, double *lb, double *ub)
{
  const double L = s->lb[v], U = s->ub[v];
  if (c > 0) {
    *lb = L > -INFINITY ? c * L : -INFINITY;
    *ub = U < INFINITY ? c * U : INFINITY;
  } else {
    *lb = U < INFINITY ? c * U : -INFINITY;
    *ub = L > -INFINITY ? c * L : INFINITY;
  }
}

/* getTermBnds_(v1, v2, coef), QuadHandler.cpp:1735-1751 */
static void term_bnds_quad(const qnode *s, int v1, int v2, double c, double *lb, double *ub)
{
  double ql, qu;
  if (v1 == v2) orc_bounds_on_square(s->lb[v1], s->ub[v1], &ql, &qu);
  else orc_bounds_on_product(1, s->lb[v1], s->ub[v1], s->lb[v2], s->ub[v2], &ql, &qu);
  if (c > 0) {
    *lb = ql > -INFINITY ? c * ql : -INFINITY;
    *ub = qu < INFINITY ? c * qu : INFINITY;
  } else {
    *lb = qu < INFINITY ? c * qu : -INFINITY;
    *ub = ql > -INFINITY ? c * ql : INFINITY;
  }
}

/* getTermBnds_(v, a, b), QuadHandler.cpp:1753-1771: bounds of a v^2 + b v */
static void term_bnds_univar(const qnode *s, int v, double a, double b, double *lb, double *ub)
{
  const double lx = s->lb[v], ux = s->ub[v];
  if (lx > -A_TOL) {
    *ub = calc_upper_univar(a, b, lx, ux);
    *lb = -calc_upper_univar(-a, -b, lx, ux);
  } else if (ux < A_TOL) {
    *ub = calc_upper_univar(a, -b, -ux, -lx);
    *lb = -calc_upper_univar(-a, b, -ux, -lx);
  } else {
    *ub = calc_upper_univar(a, b, 0.0, ux);
    *ub = smax(*ub, calc_upper_univar(a, -b, 0.0, -lx));
    *lb = -calc_upper_univar(-a, -b, 0.0, ux);
    *lb = smin(*lb, -calc_upper_univar(-a, b, 0.0, -lx));
  }
}

/* calcVarBnd_(rel, v, coef, lb, ub), QuadHandler.cpp:1786-1797 */
static int calc_var_bnd_lin(qnode *s, int v, double c, double lb, double ub, int *ch)
{
  const double vlb = c > 0 ? lb / c : ub / c;
  const double vub = c > 0 ? ub / c : lb / c;
  return update_pbounds(s, v, vlb, vub, ch) < 0;
}

/* calcVarBnd_(rel, v1, v2, coef, lb, ub), QuadHandler.cpp:1841-1881.  The
 * square branch starts vlb from -ub (the function argument), as :1852 does. */
static int calc_var_bnd_quad(qnode *s, int v1, int v2, double c, double lb, double ub, int *ch)
{
  double qlb = c > 0 ? lb / c : ub / c;
  const double qub = c > 0 ? ub / c : lb / c;
  double vlb, vub;
  if (v1 == v2) {
    if (qub > B_TOL) {
      vub = sqrt(qub);
      vlb = -ub;
      qlb = qlb >= 0 ? qlb : 0;
      if (s->lb[v1] > -sqrt(qlb) + B_TOL) vlb = sqrt(qlb);
      if (update_pbounds(s, v1, vlb, vub, ch) < 0) return 1;
    } else if (qub < -B_TOL) {
      return 1;
    } else {
      if (update_pbounds(s, v1, 0.0, 0.0, ch) < 0) return 1;
    }
    return 0;
  }
  orc_bounds_on_div(qlb, qub, s->lb[v1], s->ub[v1], &vlb, &vub);
  if (update_pbounds(s, v2, vlb, vub, ch) < 0) return 1;
  orc_bounds_on_div(qlb, qub, s->lb[v2], s->ub[v2], &vlb, &vub);
  if (update_pbounds(s, v1, vlb, vub, ch) < 0) return 1;
  return 0;
}

/* calcVarBnd_(rel, v, a, b, ly, uy), QuadHandler.cpp:1968-2078: x with
 * ly <= a x^2 + b x <= uy. */
static int calc_var_bnd_univar(qnode *s, int v, double a, double b, double ly, double uy, int *ch)
{
  const double lx = s->lb[v], ux = s->ub[v];
  double lb = -INFINITY, ub = INFINITY, delta, lb2, ub2;
  if (fabs(a) <= A_TOL) {
    lb = ly / b;
    ub = uy / b;
  } else if (a > A_TOL) { /* convex */
    if (uy < INFINITY) {
      delta = b * b + 4.0 * a * uy;
      if (delta < -A_TOL) {
        return 1;
      } else if (fabs(delta) <= A_TOL) {
        lb = -b / (2.0 * a);
        ub = lb;
      } else {
        lb = (-b - sqrt(delta)) / (2.0 * a);
        ub = (-b + sqrt(delta)) / (2.0 * a);
        delta = b * b + 4.0 * a * ly;
        if (delta > A_TOL) {
          lb2 = (-b - sqrt(delta)) / (2.0 * a);
          ub2 = (-b + sqrt(delta)) / (2.0 * a);
          if (lx > lb2 + B_TOL) lb = ub2;
          if (ux < ub2 - B_TOL) ub = lb2;
        }
      }
    } else {
      delta = b * b + 4.0 * a * ly;
      if (delta > A_TOL) {
        lb2 = (-b - sqrt(delta)) / (2.0 * a);
        ub2 = (-b + sqrt(delta)) / (2.0 * a);
        if (lx > lb2 + B_TOL && lx < ub2 - B_TOL) lb = ub2;
        if (ux > lb2 + B_TOL && ux < ub2 - B_TOL) ub = lb2;
      }
    }
  } else { /* concave */
    if (ly > -INFINITY) {
      delta = b * b + 4.0 * a * ly;
      if (delta < -A_TOL) {
        return 1;
      } else if (fabs(delta) <= A_TOL) {
        lb = -b / (2.0 * a);
        ub = lb;
      } else {
        lb = (-b + sqrt(delta)) / (2.0 * a);
        ub = (-b - sqrt(delta)) / (2.0 * a);
        delta = b * b + 4.0 * a * uy;
        if (delta > A_TOL) {
          lb2 = (-b + sqrt(delta)) / (2.0 * a);
          ub2 = (-b - sqrt(delta)) / (2.0 * a);
          if (lx > lb2 + B_TOL) lb = ub2;
          if (ux < ub2 - B_TOL) ub = lb2;
        }
      }
    } else {
      delta = b * b + 4.0 * a * uy;
      if (delta > A_TOL) {
        lb2 = (-b - sqrt(delta)) / (2.0 * a);
        ub2 = (-b + sqrt(delta)) / (2.0 * a);
        if (lx > lb2 + B_TOL && lx < ub2 - B_TOL) lb = ub2;
        if (ux > lb2 + B_TOL && ux < ub2 - B_TOL) ub = lb2;
      }
    }
  }
  return update_pbounds(s, v, lb, ub, ch) < 0;
}

/* getSumExcept1_, QuadHandler.cpp:2111-2146 (lower: which = 0) */
static double sum_except1(const double *f, int nf, int cur, int upper, double bound, unsigned ninf)
{
  if (ninf == 0) return bound - f[cur];
  if (ninf == 1) {
    if (upper ? f[cur] >= INFINITY : f[cur] <= -INFINITY) {
      double sum = 0.0;
      for (int i = 0; i < nf; ++i)
        if (i != cur) sum += f[i];
      return sum;
    }
    return upper ? INFINITY : -INFINITY;
  }
  return upper ? INFINITY : -INFINITY;
}

/* Linear weight of v in the term list of constraint c (0 if absent):
 * LinearFunction::getWeight / hasVar. */
static int lin_weight(const orc_qspec *S, int c, int v, double *w)
{
  for (int k = S->lptr[c]; k < S->lptr[c + 1]; ++k)
    if (S->lvar[k] == v) {
      *w = S->lval[k];
      return 1;
    }
  *w = 0.0;
  return 0;
}

/* Function type Quadratic: some square term (Function.cpp:41-64). */
static int has_square(const orc_qspec *S, int c)
{
  for (int k = S->qptr[c]; k < S->qptr[c + 1]; ++k)
    if (S->qv1[k] == S->qv2[k]) return 1;
  return 0;
}

/* getQfLfBnds_(rel, ...), QuadHandler.cpp:2361-2427.  Fills fl/fu with the
 * term bounds (quadratic terms, then the linear terms that are not in the
 * accumulated qvars); returns 0 when qvars is still empty. */
static int qf_lf_bnds(qnode *s, int c, double *il, double *iu, int *nf, unsigned *cil,
                      unsigned *ciu, int *any_qv)
{
  const orc_qspec *S = s->S;
  double lb = 0, ub = 0, w;
  int k0 = 0;
  for (int k = S->qptr[c]; k < S->qptr[c + 1]; ++k) {
    const int v1 = S->qv1[k], v2 = S->qv2[k];
    if (v1 == v2 && lin_weight(S, c, v1, &w)) {
      s->isq[v1] = 1;
      *any_qv = 1;
      term_bnds_univar(s, v1, S->qval[k], w, &lb, &ub);
    } else {
      term_bnds_quad(s, v1, v2, S->qval[k], &lb, &ub);
    }
    if (lb <= -INFINITY) ++*cil;
    if (ub >= INFINITY) ++*ciu;
    *il += lb;
    *iu += ub;
    s->fl[k0] = lb;
    s->fu[k0] = ub;
    ++k0;
  }
  if (!*any_qv) {
    *nf = 0;
    return 0;
  }
  for (int k = S->lptr[c]; k < S->lptr[c + 1]; ++k) {
    const int v = S->lvar[k];
    if (s->isq[v]) continue;
    term_bnds_lin(s, v, S->lval[k], &lb, &ub);
    if (lb <= -INFINITY) ++*cil;
    if (ub >= INFINITY) ++*ciu;
    *il += lb;
    *iu += ub;
    s->fl[k0] = lb;
    s->fu[k0] = ub;
    ++k0;
  }
  *nf = k0;
  return 1;
}

/* Backward pass of tightenQuad_ for one function (QuadHandler.cpp:2713-2790
 * objective / :2818-2915 constraints): every term against the stale forward
 * sums. */
static int backward(qnode *s, int c, double clb, double cub, double il, double iu, int nf,
                    unsigned cil, unsigned ciu)
{
  const orc_qspec *S = s->S;
  int ch = 0, i = 0;
  double w;
  for (int k = S->qptr[c]; k < S->qptr[c + 1]; ++k, ++i) {
    const int v1 = S->qv1[k], v2 = S->qv2[k];
    const double lb = clb - sum_except1(s->fu, nf, i, 1, iu, ciu);
    const double ub = cub - sum_except1(s->fl, nf, i, 0, il, cil);
    if (v1 == v2 && lin_weight(S, c, v1, &w)) {
      if (calc_var_bnd_univar(s, v1, S->qval[k], w, lb, ub, &ch)) return 1;
    } else {
      if (calc_var_bnd_quad(s, v1, v2, S->qval[k], lb, ub, &ch)) return 1;
    }
  }
  for (int k = S->lptr[c]; k < S->lptr[c + 1]; ++k) {
    const int v = S->lvar[k];
    if (s->isq[v]) continue;
    const double lb = clb - sum_except1(s->fu, nf, i, 1, iu, ciu);
    const double ub = cub - sum_except1(s->fl, nf, i, 0, il, cil);
    if (calc_var_bnd_lin(s, v, S->lval[k], lb, ub, &ch)) return 1;
    ++i;
  }
  return 0;
}

/* tightenQuad_(rel, bestSol, ...), QuadHandler.cpp:2683-2924 */
static int tighten_quad(qnode *s, double best)
{
  const orc_qspec *S = s->S;
  int any_qv = 0, nf;
  unsigned cil = 0, ciu = 0;
  double cub = best - S->obj_const, clb = -INFINITY;
  memset(s->isq, 0, (size_t)S->nv);
  if (cub < INFINITY) {
    const int c = S->ncon;
    double il = 0.0, iu = 0.0;
    if (S->has_obj && has_square(S, c) && S->lptr[c + 1] > S->lptr[c]) {
      if (qf_lf_bnds(s, c, &il, &iu, &nf, &cil, &ciu, &any_qv)) {
        clb = clb > il ? clb : il;
        cub = cub < iu ? cub : iu;
        if (backward(s, c, clb, cub, il, iu, nf, cil, ciu)) return 1;
      }
    }
  }
  for (int c = 0; c < S->ncon; ++c) {
    double il = 0.0, iu = 0.0;
    cil = 0;
    ciu = 0;
    if (!has_square(S, c) || S->lptr[c + 1] == S->lptr[c]) continue;
    if (!qf_lf_bnds(s, c, &il, &iu, &nf, &cil, &ciu, &any_qv)) continue;
    clb = S->clb[c];
    cub = S->cub[c];
    if (il > cub + A_TOL || iu < clb - A_TOL) return 1;
    clb = clb > il ? clb : il;
    cub = cub < iu ? cub : iu;
    if (backward(s, c, clb, cub, il, iu, nf, cil, ciu)) return 1;
  }
  return 0;
}

static double lf_keep(double a) { return fabs(a) > LF_TOL ? a : 0.0; }

/* upSqCon_, QuadHandler.cpp:3396-3419, with getNewSqLf_ :772-803.  Row
 * state [a_x, rhs] of  y + a_x x <= rhs. */
static void up_sq_con(qnode *s, int k, double *row)
{
  const orc_qspec *S = s->S;
  const double eps = A_TOL / 10.0;
  const int x = S->sq_x[k];
  const double lb = s->lb[x], ub = s->ub[x], ax = row[0];
  if ((lb * lb + ax * lb < row[1] - eps) || (ub * ub + ax * ub < row[1] - eps)) {
    row[1] = -ub * lb;
    row[0] = fabs(ub + lb) > 1e-5 ? lf_keep(-1. * (ub + lb)) : 0.0;
    qpush(s, 3, k, row[1], 0.0);
  }
}

/* upBilCon_, QuadHandler.cpp:3322-3394, with getNewBilLf_ :702-770.  Row
 * state [a0, a1, rhs] x 4 of  -+y + a0 x0 + a1 x1 <= rhs. */
static void up_bil_con(qnode *s, int k, double *row)
{
  const orc_qspec *S = s->S;
  const double eps = A_TOL / 10.0;
  const int x0 = S->bil_x0[k], x1 = S->bil_x1[k];
  const double l0 = s->lb[x0], u0 = s->ub[x0], l1 = s->lb[x1], u1 = s->ub[x1];
  const int rbase = S->nsq + 4 * k;
  double *r;
  /* y >= l1 x0 + l0 x1 - l0 l1 */
  r = row;
  if (r[0] * l0 + r[1] * l1 - l0 * l1 < r[2] - eps || r[0] * l0 + r[1] * u1 - l0 * u1 < r[2] - eps ||
      r[0] * u0 + r[1] * l1 - u0 * l1 < r[2] - eps) {
    r[0] = lf_keep(l1);
    r[1] = lf_keep(l0);
    r[2] = l0 * l1;
    qpush(s, 3, rbase + 0, r[2], 0.0);
  }
  /* y >= u1 x0 + u0 x1 - u0 u1 */
  r = row + 3;
  if (r[0] * l0 + r[1] * u1 - l0 * u1 < r[2] - eps || r[0] * u0 + r[1] * l1 - u0 * l1 < r[2] - eps ||
      r[0] * u0 + r[1] * u1 - u0 * u1 < r[2] - eps) {
    r[0] = lf_keep(u1);
    r[1] = lf_keep(u0);
    r[2] = u0 * u1;
    qpush(s, 3, rbase + 1, r[2], 0.0);
  }
  /* y <= u1 x0 + l0 x1 - l0 u1 */
  r = row + 6;
  if (r[0] * l0 + r[1] * l1 + l0 * l1 < r[2] - eps || r[0] * l0 + r[1] * u1 + l0 * u1 < r[2] - eps ||
      r[0] * u0 + r[1] * u1 + u0 * u1 < r[2] - eps) {
    r[0] = lf_keep(-1.0 * u1);
    r[1] = lf_keep(-1.0 * l0);
    r[2] = -l0 * u1;
    qpush(s, 3, rbase + 2, r[2], 0.0);
  }
  /* y <= l1 x0 + u0 x1 - u0 l1 */
  r = row + 9;
  if (r[0] * l0 + r[1] * l1 + l0 * l1 < r[2] - eps || r[0] * u0 + r[1] * l1 + u0 * l1 < r[2] - eps ||
      r[0] * u0 + r[1] * u1 + u0 * u1 < r[2] - eps) {
    r[0] = lf_keep(-1.0 * l1);
    r[1] = lf_keep(-1.0 * u0);
    r[2] = -u0 * l1;
    qpush(s, 3, rbase + 3, r[2], 0.0);
  }
}

/* Row state of QuadHandler::relax_ (QuadHandler.cpp:1549-1592) at bounds
 * lb/ub: rows[2 nsq + 12 nbil]. */
void orc_quad_rows(const orc_qspec *S, const double *lb, const double *ub, double *rows)
{
  int o = 0;
  for (int k = 0; k < S->nsq; ++k, o += 2) {
    const double l = lb[S->sq_x[k]], u = ub[S->sq_x[k]];
    rows[o + 1] = -u * l;
    rows[o] = fabs(u + l) > 1e-5 ? lf_keep(-1. * (u + l)) : 0.0;
  }
  for (int k = 0; k < S->nbil; ++k, o += 12) {
    const double l0 = lb[S->bil_x0[k]], u0 = ub[S->bil_x0[k]];
    const double l1 = lb[S->bil_x1[k]], u1 = ub[S->bil_x1[k]];
    double *r = rows + o;
    r[0] = lf_keep(l1);        r[1] = lf_keep(l0);        r[2] = l0 * l1;
    r[3] = lf_keep(u1);        r[4] = lf_keep(u0);        r[5] = u0 * u1;
    r[6] = lf_keep(-1.0 * u1); r[7] = lf_keep(-1.0 * l0); r[8] = -l0 * u1;
    r[9] = lf_keep(-1.0 * l1); r[10] = lf_keep(-1.0 * u0); r[11] = -u0 * l1;
  }
}

/* upSqCon_ / upBilCon_ over every square, then every bilinear, on the row
 * state rows[R] with box lb/ub: QuadHandler::postSolveRootNode's rewrite
 * after OBBT moved a bound (QuadHandler.cpp:1527-1533). */
void orc_quad_update_rows(const orc_qspec *S, double *lb, double *ub, double *rows)
{
  qnode s = {S, lb, ub, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < S->nsq; ++k) up_sq_con(&s, k, rows + 2 * k);
  for (int k = 0; k < S->nbil; ++k) up_bil_con(&s, k, rows + 2 * S->nsq + 12 * k);
}

/* QuadHandler::presolveNode, QuadHandler.cpp:1204-1269, on one node box
 * (lb/ub updated in place, rows = row state updated in place).  Returns 1
 * when the node is infeasible, -1 when the propagation loop hit PROP_CAP. */
int orc_quad_fbbt_node(const orc_qspec *S, double *lb, double *ub, double best, int qt,
                       double *rows, int mod_cap, int *mod_kind, int *mod_idx, double *mod_v1,
                       double *mod_v2, int *nmods_out, unsigned char *isq, double *fl,
                       double *fu)
{
  qnode s = {S, lb, ub, 0, mod_cap, mod_kind, mod_idx, mod_v1, mod_v2, isq, fl, fu};
  int changed = 1, ret = 0, iters = 0;
  while (changed) {
    int lch = 0;
    changed = 0;
    if (++iters > PROP_CAP) {
      ret = -1;
      goto done;
    }
    for (int k = 0; k < S->nsq; ++k) {
      if (prop_sqr(&s, S->sq_x[k], S->sq_y[k], &lch)) {
        ret = 1;
        goto done;
      }
    }
    for (int k = 0; k < S->nbil; ++k) {
      if (prop_bil(&s, S->bil_x0[k], S->bil_x1[k], S->bil_y[k], &lch)) {
        ret = 1;
        goto done;
      }
    }
    changed = lch;
  }
  if (qt && tighten_quad(&s, best)) {
    ret = 1;
    goto done;
  }
  for (int k = 0; k < S->nsq; ++k) up_sq_con(&s, k, rows + 2 * k);
  for (int k = 0; k < S->nbil; ++k) up_bil_con(&s, k, rows + 2 * S->nsq + 12 * k);
done:
  *nmods_out = s.nmods;
  return ret;
}

/* Longest forward-term list of any tightenQuad_ function (scratch size). */
int orc_quad_max_terms(const orc_qspec *S)
{
  int mx = 0;
  const int nc = S->ncon + (S->has_obj ? 1 : 0);
  for (int c = 0; c < nc; ++c) {
    const int t = (S->qptr[c + 1] - S->qptr[c]) + (S->lptr[c + 1] - S->lptr[c]);
    if (t > mx) mx = t;
  }
  return mx;
}

int orc_quad_fbbt_batch(const orc_qspec *S, int B, const double *lb_in, const double *ub_in,
                        double best, int qt, const double *rows_in, long rows_stride,
                        double *lb_out, double *ub_out, int *infeas, int *nmods,
                        double *rows_out, int mod_cap, int *mod_kind, int *mod_idx,
                        double *mod_v1, double *mod_v2)
{
  const int nv = S->nv, R = 2 * S->nsq + 12 * S->nbil;
  const int mt = orc_quad_max_terms(S) + 1;
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(| : bad)
  for (int b = 0; b < B; ++b) {
    unsigned char *isq = (unsigned char *)malloc((size_t)nv + 1);
    double *fl = (double *)malloc(sizeof(double) * (size_t)mt);
    double *fu = (double *)malloc(sizeof(double) * (size_t)mt);
    double *lb = lb_out + (size_t)b * nv, *ub = ub_out + (size_t)b * nv;
    double *rows = rows_out + (size_t)b * R;
    memcpy(lb, lb_in + (size_t)b * nv, sizeof(double) * nv);
    memcpy(ub, ub_in + (size_t)b * nv, sizeof(double) * nv);
    memcpy(rows, rows_in + (size_t)b * rows_stride, sizeof(double) * R);
    const size_t mo = (size_t)b * (mod_cap > 0 ? mod_cap : 0);
    const int r = orc_quad_fbbt_node(S, lb, ub, best, qt, rows, mod_cap,
                                     mod_kind ? mod_kind + mo : NULL, mod_idx ? mod_idx + mo : NULL,
                                     mod_v1 ? mod_v1 + mo : NULL, mod_v2 ? mod_v2 + mo : NULL,
                                     &nmods[b], isq, fl, fu);
    infeas[b] = r > 0 ? 1 : 0;
    if (r < 0) bad = 1;
    free(isq);
    free(fl);
    free(fu);
  }
  return bad ? -1 : 0;
}
