/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of Minotaur's node FBBT for linear rows:
 * LinearHandler::presolveNode -> simplePresolve in node mode
 * (apply_to_prob == false), /root/reference/src/base/LinearHandler.cpp.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this; the product path (minotaur_amd/) never does.
 *
 * Parity pin: checked bit-for-bit against the reference itself
 * (oracle/_ref/libref_fbbt.so, built from /root/reference/src/base by
 * oracle/Makefile) through the golden vectors in tests/golden/.
 *
 * Every function names the reference lines it restates.  Compiled with
 * -ffp-contract=off so no multiply-add is fused (the reference x86-64 build
 * has no FMA: no -march in CMakeLists.txt:36-39,184-190).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

/* LinearHandler.cpp:56-58 (constructor): intTol_, eTol_, infty_. */
#define INT_TOL 1e-6
#define E_TOL 1e-8
#define INFTY 1e20

/* Types.h:83-89 VariableType numerics. */
#define VT_BINARY 0
#define VT_INTEGER 1

typedef struct {
  const orc_lin_problem *P;
  double *lb, *ub;
  unsigned char *flag;     /* per-row BFlag (Constraint::setBFlag) */
  int nmods, mod_cap;
  int *mod_var, *mod_lu;
  double *mod_val;
  unsigned nintmods;
} node_state;

static int is_int_type(int t) { return t == VT_BINARY || t == VT_INTEGER; }

/* VarBoundMod pushed into the ModQ (apply_to_prob == false branch). */
static void push_mod(node_state *s, int j, int lu, double v)
{
  if (s->mod_var && s->nmods < s->mod_cap) {
    s->mod_var[s->nmods] = j;
    s->mod_lu[s->nmods] = lu;
    s->mod_val[s->nmods] = v;
  }
  s->nmods++;
}

/* LinearHandler::changeBFlag_, LinearHandler.cpp:1229-1234. */
static void change_bflag(node_state *s, int j)
{
  const orc_lin_problem *P = s->P;
  for (int k = P->colptr[j]; k < P->colptr[j + 1]; ++k) {
    s->flag[P->rowidx[k]] = 1;
  }
}

/* LinearHandler::getLfBnds_, LinearHandler.cpp:1237-1258. */
static void lf_bnds(const node_state *s, int nt, const int *idx,
                    const double *a, double *lo, double *up)
{
  double l = 0, u = 0;
  for (int t = 0; t < nt; ++t) {
    double c = a[t], vl = s->lb[idx[t]], vu = s->ub[idx[t]];
    if (c > 0) {
      l += c * vl;
      u += c * vu;
    } else {
      l += c * vu;
      u += c * vl;
    }
  }
  *lo = l;
  *up = u;
}

/* LinearHandler::getSingLfBnds_, LinearHandler.cpp:1261-1319. */
static void sing_lf_bnds(const node_state *s, int nt, const int *idx,
                         const double *a, double *lo, double *up)
{
  double l = 0, u = 0;
  int lo_sing = 0, up_sing = 0, lo_fin = 1, up_fin = 1;
  for (int t = 0; t < nt; ++t) {
    double c = a[t], vl = s->lb[idx[t]], vu = s->ub[idx[t]];
    if (c > E_TOL) {
      if (vu < INFTY && up_fin) {
        u += c * vu;
      } else if (up_sing) {
        up_sing = 0; u = INFINITY; up_fin = 0;
      } else {
        up_sing = 1;
      }
      if (vl > -INFTY && lo_fin) {
        l += c * vl;
      } else if (lo_sing) {
        lo_sing = 0; l = -INFINITY; lo_fin = 0;
      } else {
        lo_sing = 1;
      }
    } else if (c < -E_TOL) {
      if (vu < INFTY && lo_fin) {
        l += c * vu;
      } else if (lo_sing) {
        lo_sing = 0; l = -INFINITY; lo_fin = 0;
      } else {
        lo_sing = 1;
      }
      if (vl > -INFTY && up_fin) {
        u += c * vl;
      } else if (up_sing) {
        up_sing = 0; u = INFINITY; up_fin = 0;
      } else {
        up_sing = 1;
      }
    }
  }
  *lo = l;
  *up = u;
}

/* LinearHandler::updateLfBoundsFromLb_, LinearHandler.cpp:1048-1134. */
static void upd_from_lb(node_state *s, int nt, const int *idx, const double *a,
                        double lb, double uu, int is_sing, int *changed,
                        int count_int)
{
  for (int t = 0; t < nt; ++t) {
    int j = idx[t];
    double c = a[t], vlb = s->lb[j], vub = s->ub[j];
    if (c > E_TOL && (!is_sing || vub >= INFTY)) {
      if (vub >= INFTY) vub = 0.;
      double nlb = (lb - uu) / c + vub;
      if (nlb > vlb + E_TOL) {
        if (nlb > s->ub[j] - E_TOL) nlb = s->ub[j];
        change_bflag(s, j);
        s->lb[j] = nlb;
        push_mod(s, j, 0, nlb);
        if (count_int && is_int_type(s->P->vtype[j])) s->nintmods++;
        *changed = 1;
      }
    } else if (c < -E_TOL && (!is_sing || vlb <= -INFTY)) {
      if (vlb <= -INFTY) vlb = 0.;
      double nub = (lb - uu) / c + vlb;
      if (nub < vub - E_TOL) {
        if (nub < s->lb[j] + E_TOL) nub = s->lb[j];
        change_bflag(s, j);
        s->ub[j] = nub;
        push_mod(s, j, 1, nub);
        if (count_int && is_int_type(s->P->vtype[j])) s->nintmods++;
        *changed = 1;
      }
    }
  }
}

/* LinearHandler::updateLfBoundsFromUb_, LinearHandler.cpp:1137-1226. */
static void upd_from_ub(node_state *s, int nt, const int *idx, const double *a,
                        double ub, double ll, int is_sing, int *changed,
                        int count_int)
{
  for (int t = 0; t < nt; ++t) {
    int j = idx[t];
    double c = a[t], vlb = s->lb[j], vub = s->ub[j];
    if (c > E_TOL && (!is_sing || vlb <= -INFTY)) {
      if (vlb <= -INFTY) vlb = 0.;
      double nub = (ub - ll) / c + vlb;
      if (nub < vub - E_TOL) {
        if (nub < s->lb[j] + E_TOL) nub = s->lb[j];
        change_bflag(s, j);
        s->ub[j] = nub;
        push_mod(s, j, 1, nub);
        if (count_int && is_int_type(s->P->vtype[j])) s->nintmods++;
        *changed = 1;
      }
    } else if (c < -E_TOL && (!is_sing || vub >= INFTY)) {
      if (vub >= INFTY) vub = 0.;
      double nlb = (ub - ll) / c + vub;
      if (nlb > vlb + E_TOL) {
        if (nlb > s->ub[j] - E_TOL) nlb = s->ub[j];
        change_bflag(s, j);
        s->lb[j] = nlb;
        push_mod(s, j, 0, nlb);
        if (count_int && is_int_type(s->P->vtype[j])) s->nintmods++;
        *changed = 1;
      }
    }
  }
}

/* LinearHandler::linBndTighten_, LinearHandler.cpp:952-1045 (node mode). */
static int lin_bnd_tighten(node_state *s, int i, int *changed)
{
  const orc_lin_problem *P = s->P;
  int nt = P->rowptr[i + 1] - P->rowptr[i];
  const int *idx = P->colidx + P->rowptr[i];
  const double *a = P->val + P->rowptr[i];
  double lb = P->rlo[i], ub = P->rhi[i];
  double ll, uu, sing_ll = -INFINITY, sing_uu = INFINITY;

  *changed = 0;
  lf_bnds(s, nt, idx, a, &ll, &uu);
  if (ll < -INFTY || uu > INFTY) sing_lf_bnds(s, nt, idx, a, &sing_ll, &sing_uu);
  if (ll > ub + E_TOL) return 1;
  if (uu < lb - E_TOL) return 1;
  if (lb > -INFTY) {
    if (uu < INFTY) {
      upd_from_lb(s, nt, idx, a, lb, uu, 0, changed, 1);
    } else if (sing_uu < INFTY) {
      upd_from_lb(s, nt, idx, a, lb, sing_uu, 1, changed, 1);
    }
  }
  if (*changed) {
    lf_bnds(s, nt, idx, a, &ll, &uu);
    if (ll < -INFTY || uu > INFTY) sing_lf_bnds(s, nt, idx, a, &sing_ll, &sing_uu);
  }
  if (ub < INFTY) {
    if (ll > -INFTY) {
      upd_from_ub(s, nt, idx, a, ub, ll, 0, changed, 1);
    } else if (sing_ll > -INFTY) {
      upd_from_ub(s, nt, idx, a, ub, sing_ll, 1, changed, 1);
    }
  }
  return 0;
}

/* Diagnostics (tools/fbbt_sweep_stats.py; single-threaded use): per sweep
 * index, how many nodes ran it and how many rows they tightened. */
static int g_stats_on;
static long g_stats[2][16];
static unsigned g_sweep;
long *orc_fbbt_stats(int enable)
{
  g_stats_on = enable;
  if (enable) memset(g_stats, 0, sizeof g_stats);
  return &g_stats[0][0];
}

/* LinearHandler::varBndsFromCons_, LinearHandler.cpp:493-541 (node mode:
 * each flagged row is tightened once per sweep, :520-524). */
static int bnds_from_cons(node_state *s, int *changed)
{
  for (int i = 0; i < s->P->m; ++i) {
    if (s->flag[i]) {
      int tch;
      s->flag[i] = 0;
      if (g_stats_on && g_sweep < 16) g_stats[1][g_sweep]++;
      if (lin_bnd_tighten(s, i, &tch)) return 1;
      if (tch) *changed = 1;
    }
  }
  return 0;
}

/* LinearHandler::varBndsFromObj_, LinearHandler.cpp:544-597. */
static int bnds_from_obj(node_state *s, double ub, int *changed)
{
  const orc_lin_problem *P = s->P;
  int tch = 1;
  long guard = 0;
  if (P->nobj <= 0) return 0;
  while (tch) {
    double ll, uu, sing_ll = INFINITY, sing_uu = INFINITY;
    tch = 0;
    lf_bnds(s, P->nobj, P->objidx, P->objval, &ll, &uu);
    if (ll < -INFTY || uu > INFTY) {
      sing_lf_bnds(s, P->nobj, P->objidx, P->objval, &sing_ll, &sing_uu);
    }
    if (ll > ub + E_TOL) return 1;
    if (ll > -INFTY) {
      upd_from_ub(s, P->nobj, P->objidx, P->objval, ub, ll, 0, &tch, 0);
    } else if (sing_ll > -INFTY) {
      upd_from_ub(s, P->nobj, P->objidx, P->objval, ub, sing_ll, 1, &tch, 0);
    }
    if (tch) *changed = 1;
    if (++guard > ORC_OBJ_LOOP_CAP) break;  /* never reached on real data */
  }
  return 0;
}

/* LinearHandler::tightenInts_, LinearHandler.cpp:415-490 (node mode). */
static void tighten_ints(node_state *s, int *changed)
{
  const orc_lin_problem *P = s->P;
  for (int j = 0; j < P->n; ++j) {
    if (!is_int_type(P->vtype[j])) continue;
    double l = s->lb[j], u = s->ub[j];
    if (l > -INFTY && fabs(l - floor(l + 0.5)) > INT_TOL) {
      double v = ceil(l);
      change_bflag(s, j);
      s->lb[j] = v;
      push_mod(s, j, 0, v);
      *changed = 1;
    }
    if (u < INFTY && fabs(u - floor(u + 0.5)) > INT_TOL) {
      double v = floor(u);
      s->ub[j] = v;
      change_bflag(s, j);
      push_mod(s, j, 1, v);
      *changed = 1;
    }
  }
}

/* LinearHandler::checkBounds_, LinearHandler.cpp:328-359. */
static int check_bounds(const node_state *s)
{
  for (int j = 0; j < s->P->n; ++j) {
    if (s->lb[j] > s->ub[j] + E_TOL) return 1;
  }
  return s->P->cons_bad ? 1 : 0;
}

/* LinearHandler::presolveNode -> simplePresolve, LinearHandler.cpp:1592-1653.
 * The status returns of varBndsFromCons_/varBndsFromObj_ are ignored there
 * (:1630,:1636-1640): only checkBounds_ decides infeasibility. */
int orc_linear_fbbt_node(const orc_lin_problem *P, double *lb, double *ub,
                         int has_inc, double inc_ub, unsigned char *flag,
                         int mod_cap, int *mod_var, int *mod_lu,
                         double *mod_val, int *nmods_out)
{
  node_state s;
  int changed = 1, infeas = 0;
  unsigned iters = 1;
  const unsigned max_iters = 10, min_iters = 2;

  s.P = P; s.lb = lb; s.ub = ub; s.flag = flag;
  s.nmods = 0; s.mod_cap = mod_cap;
  s.mod_var = mod_var; s.mod_lu = mod_lu; s.mod_val = mod_val;
  s.nintmods = 0;
  memset(flag, 1, (size_t) P->m);

  while (changed && iters <= max_iters &&
         (iters <= min_iters || s.nintmods > 0) && !infeas) {
    s.nintmods = 0;
    changed = 0;
    g_sweep = iters - 1;
    if (g_stats_on && g_sweep < 16) g_stats[0][g_sweep]++;
    ++iters;
    (void) bnds_from_cons(&s, &changed);
    if (has_inc) (void) bnds_from_obj(&s, inc_ub, &changed);
    tighten_ints(&s, &changed);
    infeas = check_bounds(&s);
  }
  if (nmods_out) *nmods_out = s.nmods;
  return infeas;
}

int orc_linear_fbbt_batch(const orc_lin_problem *P, int B,
                          const double *lb_in, const double *ub_in,
                          double *lb_out, double *ub_out, int has_inc,
                          double inc_ub, int *infeas, int *nmods,
                          unsigned char *flag_scratch, int mod_cap,
                          int *mod_var, int *mod_lu, double *mod_val)
{
  size_t n = (size_t) P->n;
  for (int b = 0; b < B; ++b) {
    memcpy(lb_out + b * n, lb_in + b * n, n * sizeof(double));
    memcpy(ub_out + b * n, ub_in + b * n, n * sizeof(double));
    infeas[b] = orc_linear_fbbt_node(
        P, lb_out + b * n, ub_out + b * n, has_inc, inc_ub, flag_scratch,
        mod_cap, mod_var ? mod_var + (size_t) b * mod_cap : 0,
        mod_lu ? mod_lu + (size_t) b * mod_cap : 0,
        mod_val ? mod_val + (size_t) b * mod_cap : 0, nmods + b);
  }
  return 0;
}

/* Flat-argument entry for ctypes callers; OpenMP over nodes when
 * nthreads > 1 (the CPU baseline "port" leg times this). */
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>

int orc_linear_fbbt(int n, int m, const int *rowptr, const int *colidx,
                    const double *val, const double *rlo, const double *rhi,
                    const int *colptr, const int *rowidx, const int *vtype,
                    int nobj, const int *objidx, const double *objval,
                    int cons_bad, int B, const double *lb_in,
                    const double *ub_in, double *lb_out, double *ub_out,
                    int has_inc, double inc_ub, int *infeas, int *nmods,
                    int mod_cap, int *mod_var, int *mod_lu, double *mod_val,
                    int nthreads)
{
  orc_lin_problem P;
  P.n = n; P.m = m; P.rowptr = rowptr; P.colidx = colidx; P.val = val;
  P.rlo = rlo; P.rhi = rhi; P.colptr = colptr; P.rowidx = rowidx;
  P.vtype = vtype; P.nobj = nobj; P.objidx = objidx; P.objval = objval;
  P.cons_bad = cons_bad;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    unsigned char *flag = (unsigned char *) malloc((size_t) (m > 0 ? m : 1));
#pragma omp for schedule(static)
    for (int b = 0; b < B; ++b) {
      size_t o = (size_t) b * (size_t) n;
      memcpy(lb_out + o, lb_in + o, (size_t) n * sizeof(double));
      memcpy(ub_out + o, ub_in + o, (size_t) n * sizeof(double));
      infeas[b] = orc_linear_fbbt_node(
          &P, lb_out + o, ub_out + o, has_inc, inc_ub, flag, mod_cap,
          mod_var ? mod_var + (size_t) b * mod_cap : 0,
          mod_lu ? mod_lu + (size_t) b * mod_cap : 0,
          mod_val ? mod_val + (size_t) b * mod_cap : 0, nmods + b);
    }
    free(flag);
  }
  return 0;
}
