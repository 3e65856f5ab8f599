// Batched spatial branch-and-bound over the McCormick relaxation: the node
// loop of the reference's glob solver (Glob::createBab_, src/solvers/
// Glob.cpp:134-220: BranchAndBound + NodeIncRelaxer + PCBProcessor with
// IntVarHandler, LinearHandler, QuadHandler and, brancher=maxvio,
// MaxVioBrancher; BranchAndBound.cpp:424-514) for a QCQP after
// SimpleTransformer: one round pops the top B open nodes of an HBM stack and
// runs, all on the device,
//   lin  (mgpu_glob_config lin 1) LinearHandler::presolveNode: simplePresolve
//        in node mode over the node's relaxation rows (glob_linear);
//   K2   QuadHandler::presolveNode (QuadHandler.cpp:1204-1269): bound
//        propagation over the products and tightenQuad_, then the rewrite of
//        the node's secant / McCormick rows (upSqCon_ / upBilCon_,
//        :3322-3419) from its PARENT's row state (the incremental
//        relaxation: NodeIncRelaxer keeps the parent's rows, :94-175);
//   K3R + K3   the node's own LP with those rows (OsiLPEngine::
//        changeConstraint then solve, OsiLPEngine.cpp:206-243, 571-652),
//        warm-started from the root basis refactored for the node's matrix
//        (m > 64: K3L with the rows in HBM and the refactorisation inside);
//   decide     shouldPrune_, IntVarHandler + QuadHandler isFeasible, and
//        MaxVioBrancher over both handlers' candidates (glob_tree.hip),
//        spatial branching at the LP value on a continuous variable;
//   OBBT (mgpu_glob_config obbt 1, the root only) QuadHandler::
//        postSolveRootNode's bound LPs, chained on a bound-tightening
//        context of its own (bte_), then the root re-solved when its point
//        left the tightened relaxation (PCBProcessor.cpp:256-280);
//   children   two per branched node, each with the node's tightened box,
//        the branching bound and the node's rows.
// One small record comes back per round (counts, best feasible node).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <utility>
#include <vector>

#include "ctx.h"
#include "glob_internal.h"
#include "quad_state.h"

// Reference node order (mgpu_glob_config order 2): TreeManager's "bfs"
// NodeHeap (NodeHeap.cpp:24-47: bound within 1e-6, shallower first, then the
// larger node id on top), node ids as TreeManager assigns them (root 0,
// children in branch order, TreeManager.cpp:97-136), open nodes pruned at
// the top by the incumbent (TreeManager::getCandidate, :162-186) -- the
// batched linear tree's order 2 (bnb.cpp).
struct GHeap {
  double lb;
  int depth;
  long long id;
  int slot;
};
static bool gheap_greater(const GHeap &a, const GHeap &b) {
  if (a.lb > b.lb + 1e-6) return true;
  if (a.lb < b.lb - 1e-6) return false;
  if (a.depth < b.depth) return false;
  if (a.depth > b.depth) return true;
  return a.id < b.id;
}

struct GlobState {
  int nv = 0, R = 0, S = 0, T = 0, cap = 0, count = 0, maxb = 0;
  // mgpu_glob_config at init: order 0 stack / 2 reference heap; warm 0 the
  // root basis / 1 the parent's basis; qt 1 tightenQuad_ at every node / 0 at
  // the first presolveNode call only
  int order = 0, warm = 0, qt = 1, lin = 0, obbt = 0;
  mgpu_ctx *bte = nullptr;       // root OBBT's bound-tightening engine (bte_)
  // Glob's relstronger (mgpu_glob_brancher 1): per pool slot the branching
  // that made the node (updateAfterSolve), the pseudocosts, and the main
  // engine's last solution value (strongBranch_ reads it after a verdict of
  // the stronger mods)
  int brancher = 0;
  struct BrInfo {
    int var = -1, isint = 0;
    double act = 0.0, dd = 0.0, ud = 0.0, plb = 0.0;
  };
  std::vector<BrInfo> pinfo;
  std::vector<double> pc_up, pc_dn;
  std::vector<long long> tm_up, tm_dn;
  double last_val = 0.0;
  struct LpRec {
    int32_t status, iters;
    double value;
  };
  std::vector<LpRec> lp_log;     // relstronger: every main-engine solve in order
  DevBuf rs_head, rs_st;         // relstronger: the node's basis for its children
  std::vector<GHeap> heap;
  std::vector<int> free_slots;
  long long next_id = 1;
  int hw = 0;                    // reference order: pool high-water mark
  DevBuf pws_head, pws_st, pws_ok;                 // per pool slot: the parent's basis
  DevBuf gsel, cslots, glb, gub, grows, gtan, gdepth, ghead, gst, gok, skip_a;
  DevBuf wo_head, wo_st, wo_d, wo_binv;            // the round's optimal bases
  double inc = INFINITY;
  bool root_ws = false;
  std::vector<double> best_x;
  mgpu_glob_stats tot{};
  DevBuf plb, pub, prows, pnlb, pdepth, ptan;
  DevBuf wlb, wub, wrows, kinf, knm, st, obj, it, x, cand, dec, bvar, bval, bup, bint, pos,
      depth_in, out;
  DevBuf wvals, flag, skip2, st2, obj2, it2, x2, acc;   // the separation loop
  DevBuf ws_head, ws_st, ws_d, ws_binv, r_st, r_obj, r_it;
  DevBuf fvtype, fsq, fbil, flptr, flvar, flval, fqptr, fqv1, fqv2, fqval, fclb, fcub;
  // the linear presolve (lin 1): the relaxation's term table and its scratch
  int M = 0, nobj = 0, cons_bad = 0;
  std::vector<int32_t> h_rptr, h_tvar, h_tsrc, h_rhsrc, h_oidx;
  std::vector<double> h_tval, h_rlo, h_rhi, h_oval;
  DevBuf lrptr, ltvar, ltsrc, ltrow, lrhsrc, lcptr, lcterm, loidx, ltval, lrlo, lrhi, loval;
  DevBuf flb, fub, finf, fflag;
  void release() {
    for (DevBuf *b : {&plb, &pub, &prows, &pnlb, &pdepth, &ptan, &wlb, &wub, &wrows, &kinf,
                      &knm, &st, &obj, &it, &x, &cand, &dec, &bvar, &bval, &bup, &bint, &pos,
                      &depth_in, &out, &wvals, &flag, &skip2, &st2, &obj2, &it2, &x2, &acc,
                      &ws_head, &ws_st, &ws_d, &ws_binv, &r_st, &r_obj, &r_it, &fvtype, &fsq,
                      &fbil, &flptr, &flvar, &flval, &fqptr, &fqv1, &fqv2, &fqval, &fclb, &fcub,
                      &pws_head, &pws_st, &pws_ok, &gsel, &cslots, &glb, &gub, &grows, &gtan,
                      &gdepth, &ghead, &gst, &gok, &skip_a, &wo_head, &wo_st, &wo_d, &wo_binv,
                      &lrptr, &ltvar, &ltsrc, &ltrow, &lrhsrc, &lcptr, &lcterm, &loidx, &ltval,
                      &lrlo, &lrhi, &loval, &flb, &fub, &finf, &fflag, &rs_head, &rs_st})
      b->release();
    if (bte) mgpu_destroy(bte);
    bte = nullptr;
  }
};

void glob_state_free(mgpu_ctx *c) {
  if (c && c->glob) {
    c->glob->release();
    delete c->glob;
    c->glob = nullptr;
  }
}

namespace {

int ensure_glob_batch(mgpu_ctx *c, GlobState &s, int B) {
  if (B <= s.maxb) return MGPU_OK;
  const size_t nv = (size_t)s.nv, R = (size_t)(s.R > 0 ? s.R : 1);
  HIPCHK(c, s.wlb.ensure((size_t)B * nv * 8));
  HIPCHK(c, s.wub.ensure((size_t)B * nv * 8));
  HIPCHK(c, s.wrows.ensure((size_t)B * R * 8));
  HIPCHK(c, s.x.ensure((size_t)B * nv * 8));
  HIPCHK(c, s.cand.ensure((size_t)B * nv * 4 * 8));
  for (DevBuf *b : {&s.kinf, &s.knm, &s.st, &s.it, &s.dec, &s.bvar, &s.pos, &s.depth_in})
    HIPCHK(c, b->ensure((size_t)B * 4));
  for (DevBuf *b : {&s.obj, &s.bval}) HIPCHK(c, b->ensure((size_t)B * 8));
  for (DevBuf *b : {&s.bup, &s.bint}) HIPCHK(c, b->ensure((size_t)B));
  HIPCHK(c, s.out.ensure(sizeof(GlobOut)));
  if (s.T > 0) HIPCHK(c, s.wvals.ensure((size_t)B * (R + s.T) * 8));
  for (DevBuf *b : {&s.flag, &s.skip2, &s.st2, &s.it2, &s.skip_a}) HIPCHK(c, b->ensure((size_t)B * 4));
  HIPCHK(c, s.obj2.ensure((size_t)B * 8));
  HIPCHK(c, s.x2.ensure((size_t)B * nv * 8));
  HIPCHK(c, s.acc.ensure(16));
  if (s.order == 2) {
    HIPCHK(c, s.gsel.ensure((size_t)B * 4));
    HIPCHK(c, s.cslots.ensure((size_t)B * 2 * 4));
    HIPCHK(c, s.glb.ensure((size_t)B * nv * 8));
    HIPCHK(c, s.gub.ensure((size_t)B * nv * 8));
    HIPCHK(c, s.grows.ensure((size_t)B * R * 8));
    HIPCHK(c, s.gtan.ensure((size_t)B * (s.T > 0 ? s.T : 1) * 8));
    HIPCHK(c, s.gdepth.ensure((size_t)B * 4));
  }
  if (s.warm == 1) {
    const size_t m = (size_t)c->lp.m, N = (size_t)nv + m;
    HIPCHK(c, s.ghead.ensure((size_t)B * m * 4));
    HIPCHK(c, s.gst.ensure((size_t)B * N));
    HIPCHK(c, s.gok.ensure((size_t)B));
    HIPCHK(c, s.wo_head.ensure((size_t)B * m * 4));
    HIPCHK(c, s.wo_st.ensure((size_t)B * N));
    HIPCHK(c, s.wo_d.ensure((size_t)B * N * 8));
    HIPCHK(c, s.wo_binv.ensure((size_t)B * m * m * 8));
  }
  if (s.lin) {
    HIPCHK(c, s.flb.ensure((size_t)B * nv * 8));
    HIPCHK(c, s.fub.ensure((size_t)B * nv * 8));
    HIPCHK(c, s.finf.ensure((size_t)B * 4));
    HIPCHK(c, s.fflag.ensure((size_t)B * (s.M > 0 ? s.M : 1)));
  }
  s.maxb = B;
  return MGPU_OK;
}

// The relaxation's rows as LinearHandler sees them (the rows of
// quad.relaxation_lp, in its order): the linear rows with every product
// replaced by its auxiliary (duplicates summed, |a| <= 1e-9 dropped, terms
// ascending), one secant row per square, four McCormick rows per bilinear,
// S tangent rows per square.  Record offsets: the secant [a_x, rhs] at 2k,
// bilinear k's row t [a0, a1, rhs] at 2 nsq + 12 k + 3 t, tangent slot t of
// square k [2 xl, xl^2] at R + 2 (k S + t).
int build_linear_table(mgpu_ctx *c, GlobState &s) {
  const QuadState &q = *c->quad;
  const int nsq = (int)q.sq_x.size(), nbil = (int)q.bil_x0.size(), R = q.R, S = s.S;
  std::map<std::pair<int, int>, int> aux;
  for (int k = 0; k < nsq; ++k) aux[{q.sq_x[k], q.sq_x[k]}] = q.sq_y[k];
  for (int k = 0; k < nbil; ++k) aux[{q.bil_x0[k], q.bil_x1[k]}] = q.bil_y[k];
  struct T {
    int var, src;
    double val;
  };
  std::vector<int32_t> rptr{0}, tvar, tsrc, trow, rhsrc;
  std::vector<double> tval, rlo, rhi;
  auto add_row = [&](std::vector<T> terms, double lo, double hi, int hsrc) {
    std::sort(terms.begin(), terms.end(), [](const T &a, const T &b) { return a.var < b.var; });
    const int r = (int)rlo.size();
    for (const T &t : terms) {
      tvar.push_back(t.var);
      tsrc.push_back(t.src);
      tval.push_back(t.val);
      trow.push_back(r);
    }
    rptr.push_back((int32_t)tvar.size());
    rlo.push_back(lo);
    rhi.push_back(hi);
    rhsrc.push_back(hsrc);
  };
  auto linearize = [&](int f, std::vector<T> &out) -> int {
    std::map<int, double> d;
    for (int t = q.h_lptr[f]; t < q.h_lptr[f + 1]; ++t) d[q.h_lvar[t]] += q.h_lval[t];
    for (int t = q.h_qptr[f]; t < q.h_qptr[f + 1]; ++t) {
      auto it = aux.find({q.h_qv1[t], q.h_qv2[t]});
      if (it == aux.end()) it = aux.find({q.h_qv2[t], q.h_qv1[t]});
      if (it == aux.end()) return -1;
      d[it->second] += q.h_qval[t];
    }
    for (const auto &e : d)
      if (std::fabs(e.second) > 1e-9) out.push_back({e.first, -1, e.second});
    return 0;
  };
  int bad = 0;
  for (int f = 0; f < q.ncon; ++f) {
    std::vector<T> terms;
    if (linearize(f, terms) != 0)
      return fail(c, MGPU_ERR_ARG, "mgpu_glob_init: a product of function %d has no auxiliary", f);
    add_row(terms, q.h_clb[f], q.h_cub[f], -1);
    if (q.h_clb[f] > q.h_cub[f] + 1e-8) bad = 1;
  }
  for (int k = 0; k < nsq; ++k)
    add_row({{q.sq_x[k], 2 * k, 0.0}, {q.sq_y[k], -1, 1.0}}, -INFINITY, 0.0, 2 * k + 1);
  for (int k = 0; k < nbil; ++k)
    for (int t = 0; t < 4; ++t) {
      const int o = 2 * nsq + 12 * k + 3 * t;
      add_row({{q.bil_x0[k], o, 0.0}, {q.bil_x1[k], o + 1, 0.0},
               {q.bil_y[k], -1, t < 2 ? -1.0 : 1.0}}, -INFINITY, 0.0, o + 2);
    }
  for (int k = 0; k < nsq; ++k)
    for (int t = 0; t < S; ++t) {
      const int o = R + 2 * (k * S + t);
      add_row({{q.sq_x[k], o, 0.0}, {q.sq_y[k], -1, -1.0}}, -INFINITY, 0.0, o + 1);
    }
  std::vector<T> ob;
  if (q.has_obj && linearize(q.ncon, ob) != 0)
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_init: a product of the objective has no auxiliary");
  std::vector<int32_t> oidx;
  std::vector<double> oval;
  for (const T &t : ob) {
    oidx.push_back(t.var);
    oval.push_back(t.val);
  }
  // column incidence (term indices)
  const int nv = s.nv, nt = (int)tvar.size();
  std::vector<int32_t> cptr((size_t)nv + 1, 0), cterm((size_t)nt);
  for (int t = 0; t < nt; ++t) ++cptr[(size_t)tvar[t] + 1];
  for (int j = 0; j < nv; ++j) cptr[(size_t)j + 1] += cptr[(size_t)j];
  std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
  for (int t = 0; t < nt; ++t) cterm[(size_t)fill[(size_t)tvar[t]]++] = t;
  s.M = (int)rlo.size();
  s.nobj = (int)oidx.size();
  s.cons_bad = bad;
  s.h_rptr = rptr;
  s.h_tvar = tvar;
  s.h_tsrc = tsrc;
  s.h_tval = tval;
  s.h_rlo = rlo;
  s.h_rhi = rhi;
  s.h_rhsrc = rhsrc;
  s.h_oidx = oidx;
  s.h_oval = oval;
  if (!s.lin) return MGPU_OK;
  HIPCHK(c, upload(s.lrptr, rptr.data(), rptr.size()));
  HIPCHK(c, upload(s.ltvar, tvar.data(), tvar.size()));
  HIPCHK(c, upload(s.ltsrc, tsrc.data(), tsrc.size()));
  HIPCHK(c, upload(s.ltrow, trow.data(), trow.size()));
  HIPCHK(c, upload(s.ltval, tval.data(), tval.size()));
  HIPCHK(c, upload(s.lrlo, rlo.data(), rlo.size()));
  HIPCHK(c, upload(s.lrhi, rhi.data(), rhi.size()));
  HIPCHK(c, upload(s.lrhsrc, rhsrc.data(), rhsrc.size()));
  HIPCHK(c, upload(s.lcptr, cptr.data(), cptr.size()));
  HIPCHK(c, upload(s.lcterm, cterm.data(), cterm.size()));
  HIPCHK(c, upload(s.loidx, oidx.data(), oidx.size()));
  HIPCHK(c, upload(s.loval, oval.data(), oval.size()));
  return MGPU_OK;
}

// ---- root OBBT: QuadHandler::postSolveRootNode (QuadHandler.cpp:1397-1547)
// with tightenLP_ (:2218-2297), on the host around device LPs -- the same
// restatement as minotaur_amd/obbt.py obbt_chained (pinned bit for bit
// against the reference's postSolveRootNode), here inside the glob round.
constexpr double kObbtMaxVio = 1e-3, kObbtGap = 0.01, kObbtBTol = 1e-8, kObbtRTol = 1e-7;

// the itmp marks of postSolveRootNode (:1410-1517): 1 lower, 2 upper, 3 both
void obbt_marks(const QuadState &q, const double *x, const double *lb, const double *ub,
                std::vector<int> &itmp) {
  itmp.assign((size_t)q.nv, 0);
  for (size_t k = 0; k < q.sq_x.size(); ++k) {
    const int y = q.sq_y[k], x0 = q.sq_x[k];
    const double yv = x[y], xv = x[x0];
    double vio1 = std::fabs(xv * xv - yv);
    if (vio1 > kObbtMaxVio && vio1 > 0.1 * std::fabs(yv)) {
      if (ub[x0] - lb[x0] >= 2) itmp[(size_t)x0] = 3;
      if (ub[y] - lb[y] >= 2) {
        vio1 = yv - lb[y];
        itmp[(size_t)y] = (vio1 > kObbtMaxVio && vio1 > 0.1 * lb[y]) ? 3 : 2;
      }
    }
  }
  auto mark = [&](int v) {
    int &t = itmp[(size_t)v];
    if (!(ub[v] - lb[v] >= 2 && t != 3)) return;
    const double vio1 = x[v] - lb[v], vio2 = ub[v] - x[v];
    if (vio1 > kObbtMaxVio && vio1 > 0.1 * std::fabs(lb[v])) {
      if (vio2 > kObbtMaxVio && vio2 > 0.1 * std::fabs(ub[v])) t = 3;
      else t = t == 2 ? 3 : 1;
    } else if (vio2 > kObbtMaxVio && vio2 > std::fabs(ub[v])) {
      t = t == 1 ? 3 : 2;
    }
  };
  for (size_t k = 0; k < q.bil_x0.size(); ++k) {
    const int y = q.bil_y[k], x0 = q.bil_x0[k], x1 = q.bil_x1[k];
    const double yv = x[y];
    const double vio1 = std::fabs(x[x0] * x[x1] - yv);
    if (vio1 > kObbtMaxVio && vio1 > 0.1 * std::fabs(yv)) {
      mark(x0);
      mark(x1);
      mark(y);
    }
  }
}

// setItmpFromSol_ (:2173-2216) with p_'s current bounds
void obbt_itmp_from_sol(std::vector<int> &itmp, const double *xs, const double *lb,
                        const double *ub) {
  for (size_t v = 0; v < itmp.size(); ++v) {
    const int t = itmp[v];
    if (t == 0) continue;
    const double l = lb[v], u = ub[v], xv = xs[v];
    if (t == 1) {
      if ((xv - l) / (u - l) <= kObbtGap) itmp[v] = 0;
    } else if (t == 2) {
      if ((u - xv) / (u - l) <= kObbtGap) itmp[v] = 0;
    } else {
      if ((xv - l) / (u - l) <= kObbtGap) itmp[v] = 2;
      if ((u - xv) / (u - l) <= kObbtGap) itmp[v] = 1;
    }
  }
}

// updatePBounds_ (:3248-3320): -1 infeasible, 1 a bound moved, 0 none
int obbt_update_bounds(int v, double nlb, double nub, int vtype, double *lb, double *ub) {
  if (vtype <= 3) {
    nub = std::floor(nub);
    nlb = std::ceil(nlb);
  }
  const double L = lb[v], U = ub[v];
  if (nlb > U + kObbtBTol || nub < L - kObbtBTol) return -1;
  const bool lo = nlb > L + kObbtBTol && (L == -INFINITY || nlb > L + kObbtRTol * std::fabs(L));
  const bool up = nub < U - kObbtBTol && (U == INFINITY || nub < U - kObbtRTol * std::fabs(U));
  if (lo && up) {
    lb[v] = nlb;
    ub[v] = nub;
    return 1;
  }
  if (lo) {
    lb[v] = nlb;
    return 1;
  }
  if (up) {
    ub[v] = nub;
    return 1;
  }
  return 0;
}

// upSqCon_ / upBilCon_ (:3322-3419) over every square, then every bilinear,
// on the row state rows[R] with the box lb / ub
void obbt_update_rows(const QuadState &q, const double *lb, const double *ub, double *rows) {
  const double eps = 1e-6 / 10.0;
  auto keep = [](double a) { return std::fabs(a) > 1e-9 ? a : 0.0; };
  const int nsq = (int)q.sq_x.size();
  for (int k = 0; k < nsq; ++k) {
    double *r = rows + 2 * k;
    const double l = lb[q.sq_x[k]], u = ub[q.sq_x[k]], ax = r[0];
    if ((l * l + ax * l < r[1] - eps) || (u * u + ax * u < r[1] - eps)) {
      r[1] = -u * l;
      r[0] = std::fabs(u + l) > 1e-5 ? keep(-1. * (u + l)) : 0.0;
    }
  }
  for (size_t k = 0; k < q.bil_x0.size(); ++k) {
    const int x0 = q.bil_x0[k], x1 = q.bil_x1[k];
    const double l0 = lb[x0], u0 = ub[x0], l1 = lb[x1], u1 = ub[x1];
    double *r = rows + 2 * nsq + 12 * k;
    if (r[0] * l0 + r[1] * l1 - l0 * l1 < r[2] - eps || r[0] * l0 + r[1] * u1 - l0 * u1 < r[2] - eps ||
        r[0] * u0 + r[1] * l1 - u0 * l1 < r[2] - eps) {
      r[0] = keep(l1);
      r[1] = keep(l0);
      r[2] = l0 * l1;
    }
    r += 3;
    if (r[0] * l0 + r[1] * u1 - l0 * u1 < r[2] - eps || r[0] * u0 + r[1] * l1 - u0 * l1 < r[2] - eps ||
        r[0] * u0 + r[1] * u1 - u0 * u1 < r[2] - eps) {
      r[0] = keep(u1);
      r[1] = keep(u0);
      r[2] = u0 * u1;
    }
    r += 3;
    if (r[0] * l0 + r[1] * l1 + l0 * l1 < r[2] - eps || r[0] * l0 + r[1] * u1 + l0 * u1 < r[2] - eps ||
        r[0] * u0 + r[1] * u1 + u0 * u1 < r[2] - eps) {
      r[0] = keep(-1.0 * u1);
      r[1] = keep(-1.0 * l0);
      r[2] = -l0 * u1;
    }
    r += 3;
    if (r[0] * l0 + r[1] * l1 + l0 * l1 < r[2] - eps || r[0] * u0 + r[1] * l1 + u0 * l1 < r[2] - eps ||
        r[0] * u0 + r[1] * u1 + u0 * u1 < r[2] - eps) {
      r[0] = keep(-1.0 * l1);
      r[1] = keep(-1.0 * u0);
      r[2] = -u0 * l1;
    }
  }
}

// a row's weight / upper side with the node record rec [R + T]
inline double tab_w(const GlobState &s, const double *rec, int t) {
  return s.h_tsrc[(size_t)t] < 0 ? s.h_tval[(size_t)t] : rec[s.h_tsrc[(size_t)t]];
}
inline double tab_hi(const GlobState &s, const double *rec, int r) {
  return s.h_rhsrc[(size_t)r] < 0 ? s.h_rhi[(size_t)r] : rec[s.h_rhsrc[(size_t)r]];
}

// isFeasibleToRelaxation_ (:955-981): x against every relaxation row
bool obbt_rel_feasible(const GlobState &s, const double *rec, const double *x) {
  for (int r = 0; r < s.M; ++r) {
    double act = 0.0;
    for (int t = s.h_rptr[(size_t)r]; t < s.h_rptr[(size_t)r + 1]; ++t) {
      const double a = tab_w(s, rec, t);
      if (std::fabs(a) > 1e-9) act += a * x[s.h_tvar[(size_t)t]];
    }
    const double cub = tab_hi(s, rec, r), clb = s.h_rlo[(size_t)r];
    if ((act > cub + 1e-6) && (cub == 0 || act > cub + std::fabs(cub) * 1e-7)) return false;
    if ((act < clb - 1e-6) && (clb == 0 || act < clb - std::fabs(clb) * 1e-7)) return false;
  }
  return true;
}

// postSolveRootNode on the root (batch index 0 of the first round): x its LP
// point, lb / ub its box, rec its record; tightens lb / ub / rec in place.
// *changed: a bound moved (rows rewritten); *feasible: x still satisfies
// the tightened relaxation.  *nlps: bound LPs solved.
int glob_root_obbt(mgpu_ctx *c, GlobState &s, const double *x, std::vector<double> &lb,
                   std::vector<double> &ub, std::vector<double> &rec, bool *changed,
                   bool *feasible, long long *nlps) {
  const QuadState &q = *c->quad;
  const int nv = s.nv;
  *changed = false;
  *feasible = true;
  std::vector<int> itmp;
  obbt_marks(q, x, lb.data(), ub.data(), itmp);
  // tightenLP_: the relaxation cloned with the root's bounds and rows (the
  // free rows of unused tangent slots left out: the reference has no such
  // row), plus the objective cutoff row with an incumbent (:2232-2244)
  std::vector<int32_t> rptr{0}, cidx, ctype((size_t)nv);
  std::vector<double> val, rlo, rhi;
  const int R = s.R;
  for (int r = 0; r < s.M; ++r) {
    const double hi = tab_hi(s, rec.data(), r);
    if (s.h_rhsrc[(size_t)r] >= R && hi == INFINITY) continue;
    for (int t = s.h_rptr[(size_t)r]; t < s.h_rptr[(size_t)r + 1]; ++t) {
      const double a = tab_w(s, rec.data(), t);
      if (std::fabs(a) <= 1e-9) continue;
      cidx.push_back(s.h_tvar[(size_t)t]);
      val.push_back(a);
    }
    rptr.push_back((int32_t)cidx.size());
    rlo.push_back(s.h_rlo[(size_t)r]);
    rhi.push_back(hi);
  }
  if (std::isfinite(s.inc) && q.has_obj) {
    for (size_t k = 0; k < s.h_oidx.size(); ++k) {
      cidx.push_back(s.h_oidx[k]);
      val.push_back(s.h_oval[k]);
    }
    rptr.push_back((int32_t)cidx.size());
    rlo.push_back(-INFINITY);
    rhi.push_back(s.inc - q.obj_const);
  }
  for (int j = 0; j < nv; ++j) ctype[(size_t)j] = q.h_vtype[(size_t)j];
  const int m = (int)rlo.size(), N = nv + m;
  const std::vector<double> lb0 = lb, ub0 = ub;   // the clone's bounds stay as loaded
  if (!s.bte) {
    int rc = mgpu_create(c->device, &s.bte);
    if (rc != MGPU_OK) return fail(c, rc, "mgpu_glob_round: the OBBT engine: mgpu_create failed");
    mgpu_set_stream(s.bte, c->stream);
  }
  std::vector<double> obj((size_t)nv, 0.0), xs((size_t)nv), wd((size_t)N), wb((size_t)m * m),
      ib((size_t)m * m);
  std::vector<int32_t> wh((size_t)m), ih((size_t)m);
  std::vector<int8_t> wst((size_t)N), ist((size_t)N);
  bool have_ws = false;   // bte_->load drops the warm start: the first LP from the slack basis
  // getBndByLP_ (:2080-2109): the bound LP min sign x_v from the last
  // optimal basis (HipLPEngine keeps a basis after ProvenOptimal /
  // EngineIterationLimit), its reduced costs rebuilt for the new objective
  auto bound_lp = [&](int v, double sign, double *b, bool *inf) -> int {
    std::fill(obj.begin(), obj.end(), 0.0);
    obj[(size_t)v] = sign;
    int rc = mgpu_load_lp(s.bte, nv, m, rptr.data(), cidx.data(), val.data(), rlo.data(),
                          rhi.data(), lb0.data(), ub0.data(), ctype.data(), obj.data(), 0.0);
    if (rc != MGPU_OK) return fail(c, rc, "mgpu_glob_round: OBBT load: %s", mgpu_last_error(s.bte));
    int32_t st = 0, it = 0;
    double ov = 0.0;
    rc = mgpu_lp_solve(s.bte, 1, lb0.data(), ub0.data(), nullptr, have_ws ? ih.data() : nullptr,
                       have_ws ? ist.data() : nullptr, nullptr, have_ws ? ib.data() : nullptr, 1, 0,
                       &st, &ov, &it, xs.data(), wh.data(), wst.data(), wd.data(), wb.data());
    if (rc != MGPU_OK) return fail(c, rc, "mgpu_glob_round: OBBT solve: %s", mgpu_last_error(s.bte));
    ++*nlps;
    if (st == 0 || st == 6) {
      ih.swap(wh);
      ist.swap(wst);
      ib.swap(wb);
      have_ws = true;
    }
    *inf = !(st == 0 || st == 6 || st == 4);
    *b = *inf ? INFINITY : ov;
    return MGPU_OK;
  };
  for (int v = 0; v < nv; ++v) {
    const int t = itmp[(size_t)v];
    if (t == 0) continue;
    double nlb = -INFINITY, nub = INFINITY, b = 0.0;
    bool inf = false;
    if (t == 1 || t == 3) {
      int rc = bound_lp(v, 1.0, &b, &inf);
      if (rc != MGPU_OK) return rc;
      if (inf) continue;
      nlb = b;
      obbt_itmp_from_sol(itmp, xs.data(), lb.data(), ub.data());
    }
    if (t == 2) {
      int rc = bound_lp(v, -1.0, &b, &inf);
      if (rc != MGPU_OK) return rc;
      if (inf) continue;
      nub = -b;
      obbt_itmp_from_sol(itmp, xs.data(), lb.data(), ub.data());
    }
    const int u = obbt_update_bounds(v, nlb, nub, q.h_vtype[(size_t)v], lb.data(), ub.data());
    if (u < 0) break;   // tightenLP_ returns "infeasible" (only logged, :1519-1524)
    if (u > 0) *changed = true;
  }
  if (*changed) {
    obbt_update_rows(q, lb.data(), ub.data(), rec.data());
    *feasible = obbt_rel_feasible(s, rec.data(), x);
  }
  return MGPU_OK;
}

// ---- Glob's relstronger: StrongBrancher with reliabilitySetup(20, 50, 5)
// (Glob.cpp:171-181; StrongBrancher.cpp) on the reference's node at a time.
// The host runs PCBProcessor::process's loop for the popped node (batch 1,
// order 2, warm 1, lin 1) the way the reference does; every presolve
// (glob_linear, K2), LP (K3R + K3 through lp_solve_rows_wo) and decision
// (glob_decide) runs on the device.  The strong-branching children and the
// brancher's modifications are built here from QuadHandler / IntVarHandler::
// getBrMod (QuadHandler.cpp:616-692, IntVarHandler.cpp:113-130); the engine's
// basis is chained through two device slots (A: the node's gathered basis,
// B: the round's warm-start output) as the reference's one engine chains it.
constexpr int kSbCands = 20, kSbIter = 50, kSbThresh = 5;
constexpr double kSbEps = 1e-6;

struct RsCand {
  int var, isint;
  double dd, ud;
};

inline bool rs_at_bnds(double v, double l, double u) {
  return std::fabs(v - l) < 1e-8 || std::fabs(v - u) < 1e-8;
}

// IntVarHandler / QuadHandler getBranchingCandidates merged per variable
// (the later handler takes a candidate whose distance sum is >=; the
// distances stay the earlier one's: BrCand::setDist is an empty
// non-virtual), ascending by variable (CompareVarBrCand, Types.cpp:23-27);
// the arithmetic of glob_decide's candidate pass
void rs_candidates(const QuadState &q, const double *x, const double *lb, const double *ub,
                   std::vector<RsCand> &out) {
  const int nv = q.nv;
  std::vector<char> hi((size_t)nv, 0), hq((size_t)nv, 0);
  std::vector<double> idd((size_t)nv), iud((size_t)nv), qd((size_t)nv), qu((size_t)nv);
  for (int j = 0; j < nv; ++j) {
    const double v = x[j];
    if (q.h_vtype[(size_t)j] <= 1 && std::fabs(std::floor(v + 0.5) - v) > 1e-6) {
      hi[(size_t)j] = 1;
      idd[(size_t)j] = v - std::floor(v);
      iud[(size_t)j] = std::ceil(v) - v;
    }
  }
  auto add_q = [&](int j, double d, double u) {
    if (!hq[(size_t)j]) {
      hq[(size_t)j] = 1;
      qd[(size_t)j] = d;
      qu[(size_t)j] = u;
    } else {
      qd[(size_t)j] = d + qd[(size_t)j];
      qu[(size_t)j] = u + qu[(size_t)j];
    }
  };
  for (size_t k = 0; k < q.sq_x.size(); ++k) {
    const int j = q.sq_x[k], y = q.sq_y[k];
    const double x0 = x[j], yv = x[y];
    if (yv - x0 * x0 > std::fabs(yv) * 1e-7 && yv - x0 * x0 > 1e-6) {
      const double dd = (yv - x0 * x0) / std::sqrt(1.0 + (lb[j] + x0) * (lb[j] + x0));
      const double ud = (yv - x0 * x0) / std::sqrt(1.0 + (ub[j] + x0) * (ub[j] + x0));
      add_q(j, dd, ud);
    }
  }
  for (size_t k = 0; k < q.bil_x0.size(); ++k) {
    const int j0 = q.bil_x0[k], j1 = q.bil_x1[k], y = q.bil_y[k];
    const double v0 = x[j0], v1 = x[j1], yv = x[y], pr = v1 * v0;
    if (!(std::fabs(pr - yv) > 1e-5 && std::fabs(pr - yv) > std::fabs(yv) * 1e-4)) continue;
    if (!rs_at_bnds(v0, lb[j0], ub[j0])) {
      double dd, ud;
      if (v0 * v1 > yv) {
        dd = (-yv + v0 * v1) / std::sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1]);
        ud = (-yv + v0 * v1) / std::sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1]);
      } else {
        dd = (yv - v0 * v1) / std::sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1]);
        ud = (yv - v0 * v1) / std::sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1]);
      }
      add_q(j0, dd, ud);
    }
    if (!rs_at_bnds(v1, lb[j1], ub[j1])) {
      double dd, ud;
      if (v0 * v1 > yv) {
        dd = (-yv + v1 * v0) / std::sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0]);
        ud = (-yv + v1 * v0) / std::sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0]);
      } else {
        dd = (yv - v1 * v0) / std::sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0]);
        ud = (yv - v1 * v0) / std::sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0]);
      }
      add_q(j1, dd, ud);
    }
  }
  out.clear();
  for (int j = 0; j < nv; ++j) {
    const size_t u = (size_t)j;
    if (hi[u] && hq[u])
      out.push_back({j, idd[u] + iud[u] <= qd[u] + qu[u] ? 0 : 1, idd[u], iud[u]});
    else if (hi[u])
      out.push_back({j, 1, idd[u], iud[u]});
    else if (hq[u])
      out.push_back({j, 0, qd[u], qu[u]});
  }
}

inline double rs_keep(double a) { return std::fabs(a) > 1e-9 ? a : 0.0; }

// Handler::getBrMod of candidate (j, isint) in one direction on the node's
// box and record (in place): IntVarHandler floor / ceil of x_j;
// QuadHandler x_j itself plus the rows of x_j's violated terms rebuilt for
// the branch's box (getNewSqLf_, getNewBilLf_; with x_j the bilinear's
// second factor the arguments come swapped, as in the reference)
void rs_br_mod(const QuadState &q, std::vector<double> &rec, std::vector<double> &lb,
               std::vector<double> &ub, const double *x, int j, int isint, bool down) {
  const double v = x[j];
  if (isint) {
    if (down) ub[(size_t)j] = std::floor(v);
    else lb[(size_t)j] = std::ceil(v);
    return;
  }
  const int nsq = (int)q.sq_x.size();
  for (int k = 0; k < nsq; ++k) {
    if (q.sq_x[(size_t)k] != j) continue;
    const double yv = x[q.sq_y[(size_t)k]], vio = v * v - yv;
    if (vio > 1e-6 && vio > std::fabs(yv) * 1e-7) {
      const double lo = down ? lb[(size_t)j] : v, hi = down ? v : ub[(size_t)j];
      rec[(size_t)(2 * k + 1)] = -hi * lo;
      rec[(size_t)(2 * k)] = std::fabs(hi + lo) > 1e-5 ? rs_keep(-1. * (hi + lo)) : 0.0;
    }
  }
  for (size_t k = 0; k < q.bil_x0.size(); ++k) {
    const int X0 = q.bil_x0[k], X1 = q.bil_x1[k], y = q.bil_y[k];
    if (j != X0 && j != X1) continue;
    const double vio = std::fabs(x[X0] * x[X1] - x[y]);
    if (!(vio > 1e-5 && vio > std::fabs(x[y]) * 1e-4)) continue;
    const int a = j == X0 ? X0 : X1, bb = j == X0 ? X1 : X0;
    const double xa = x[a];
    const double lb0 = down ? lb[(size_t)a] : xa, ub0 = down ? xa : ub[(size_t)a];
    const double lb1 = lb[(size_t)bb], ub1 = ub[(size_t)bb];
    const size_t o0 = (size_t)(2 * nsq) + 12 * k;
    for (int t : {down ? 1 : 0, down ? 3 : 2}) {
      double ca, cb, rhs;   // getNewBilLf_ (QuadHandler.cpp:730-763): a's, b's coefficient
      if (t == 0) {
        ca = lb1; cb = lb0; rhs = lb0 * lb1;
      } else if (t == 1) {
        ca = ub1; cb = ub0; rhs = ub0 * ub1;
      } else if (t == 2) {
        ca = -1.0 * ub1; cb = -1.0 * lb0; rhs = -lb0 * ub1;
      } else {
        ca = -1.0 * lb1; cb = -1.0 * ub0; rhs = -ub0 * lb1;
      }
      const double c0 = a == X0 ? ca : cb, c1 = a == X0 ? cb : ca;
      double *r = rec.data() + o0 + 3 * (size_t)t;
      r[0] = rs_keep(c0);
      r[1] = rs_keep(c1);
      r[2] = rhs;
    }
  }
  if (down) ub[(size_t)j] = v;
  else lb[(size_t)j] = v;
}

// StrongBrancher::shouldPrune_ (:461-497): prune; *rel cleared when the
// status makes the candidate unreliable
inline bool rs_prune(double chcutoff, double change, int st, bool *rel) {
  if (st == 3 || st == 2 || st == 5) return true;
  if (st == 1 || st == 0) return change > chcutoff - kSbEps;
  if (st == 6) return false;
  *rel = false;
  return false;
}

inline double rs_score(double up, double down) {   // getScore_ (:381-389)
  return up > down ? down * 0.8 + up * 0.2 : up * 0.8 + down * 0.2;
}

int glob_node_rs(mgpu_ctx *c, GlobState &s, GlobIO &io, const GHeap &node,
                 mgpu_glob_stats *stats) {
  const QuadState &q = *c->quad;
  const int nv = s.nv, R = s.R, T = s.T, RT = R + T, m = c->lp.m, N = nv + m;
  hipStream_t stream = c->stream;
  // every copy ordered on the context's (non-blocking) stream and waited
  // for: the node's loop reads each kernel's result before the next step
  auto cp = [stream](void *dst, const void *src, size_t bytes, hipMemcpyKind kind) -> hipError_t {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, stream);
    return e != hipSuccess ? e : hipStreamSynchronize(stream);
  };
  // the engine's basis: 0 none (slack), 1 slot A (ghead / gst), 2 slot B (wo)
  int32_t *hA = io.ghead, *hB = s.wo_head.as<int32_t>();
  int8_t *sA = io.gst, *sB = s.wo_st.as<int8_t>();
  LpWarmOut woA{hA, sA, s.wo_d.as<double>(), s.wo_binv.as<double>()};
  LpWarmOut woB{hB, sB, s.wo_d.as<double>(), s.wo_binv.as<double>()};
  const double *dvals = io.wvals;   // the node's LP record (the rows, then the tangent slots)
  std::vector<double> x((size_t)nv), lb((size_t)nv), ub((size_t)nv), rec((size_t)(RT > 0 ? RT : 1));
  int32_t st = 0, it = 0, kinf = 0, dec = 0;
  double obj = 0.0;
  long long lps = 0, pivots = 0, sb_lps = 0, obbt_lps = 0, resolves = 0;
  // the node's first LP (the round's code ran it): results and basis
  HIPCHK(c, hipStreamSynchronize(stream));
  HIPCHK(c, cp(&kinf, io.kinf, 4, hipMemcpyDeviceToHost));
  const GlobState::BrInfo info = s.pinfo[(size_t)node.slot];
  int eng = 0;
  auto finish = [&](int d, const std::vector<GHeap> &kids) -> int {
    s.tot.rounds += 1;
    s.tot.nodes += 1;
    s.tot.ndec[d] += 1;
    s.tot.lps += lps;
    s.tot.pivots += pivots;
    s.tot.obbt_lps += obbt_lps;
    s.tot.sb_lps += sb_lps;
    s.tot.resolves += resolves;
    for (const GHeap &k : kids) {
      s.heap.push_back(k);
      std::push_heap(s.heap.begin(), s.heap.end(), gheap_greater);
    }
    s.count = (int)s.heap.size();
    s.tot.open = s.count;
    s.tot.last_batch = 1;
    s.tot.incumbent = s.inc;
    if (stats) *stats = s.tot;
    if (d == 4)
      return fail(c, MGPU_ERR_ENGINE, "mgpu_glob_round: an engine problem (K2 propagation cap / "
                  "default bound, or an unbounded / unknown LP status)");
    return MGPU_OK;
  };
  if (kinf != 0) return finish(kinf == 1 ? 1 : 4, {});
  auto pull = [&]() -> int {   // the LP result and decision at index 0
    HIPCHK(c, cp(&st, io.status, 4, hipMemcpyDeviceToHost));
    HIPCHK(c, cp(&it, io.iters, 4, hipMemcpyDeviceToHost));
    HIPCHK(c, cp(&obj, io.obj, 8, hipMemcpyDeviceToHost));
    HIPCHK(c, cp(&dec, io.dec, 4, hipMemcpyDeviceToHost));
    HIPCHK(c, cp(x.data(), io.x, (size_t)nv * 8, hipMemcpyDeviceToHost));
    return MGPU_OK;
  };
  int rc = pull();
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, cp(lb.data(), io.wlb, (size_t)nv * 8, hipMemcpyDeviceToHost));
  HIPCHK(c, cp(ub.data(), io.wub, (size_t)nv * 8, hipMemcpyDeviceToHost));
  if (RT > 0) HIPCHK(c, cp(rec.data(), dvals, (size_t)RT * 8, hipMemcpyDeviceToHost));
  lps += 1;
  pivots += it;
  s.last_val = obj;
  s.lp_log.push_back({st, it, obj});
  uint8_t gok = 0;
  HIPCHK(c, cp(&gok, io.gok, 1, hipMemcpyDeviceToHost));
  eng = (st == 0 || st == 6) ? 2 : (gok ? 1 : 0);
  // one LP of the node's current device state (wlb / wub / record at index
  // 0) from the engine's basis into the other slot
  auto lp = [&](int iter_limit, bool decide_after) -> int {
    const int out = eng == 2 ? 1 : 2;
    int r = lp_solve_rows_wo(c, 1, io.wlb, io.wub, nullptr, dvals, eng == 0 ? nullptr : eng == 1 ? hA : hB,
                             eng == 0 ? nullptr : eng == 1 ? sA : sB, 0, iter_limit, io.status, io.obj,
                             io.iters, io.x, nullptr, out == 1 ? &woA : &woB);
    if (r != MGPU_OK) return r;
    if (decide_after) {
      const int32_t zero = 0;
      HIPCHK(c, cp(const_cast<int32_t *>(io.kinf), &zero, 4, hipMemcpyHostToDevice));
      HIPCHK(c, launch_glob_decide(io, stream));
      r = pull();
      if (r != MGPU_OK) return r;
    } else {
      HIPCHK(c, cp(&st, io.status, 4, hipMemcpyDeviceToHost));
      HIPCHK(c, cp(&it, io.iters, 4, hipMemcpyDeviceToHost));
      HIPCHK(c, cp(&obj, io.obj, 8, hipMemcpyDeviceToHost));
    }
    lps += 1;
    s.last_val = obj;
    s.lp_log.push_back({st, it, obj});
    if (st == 0 || st == 6) eng = out;
    return MGPU_OK;
  };
  // a box and record through the handlers' presolveNode (glob_linear, K2)
  // into the node's device state; *inf: proven infeasible
  auto presolve = [&](const std::vector<double> &l, const std::vector<double> &u,
                      const std::vector<double> &r, bool *inf) -> int {
    HIPCHK(c, cp(io.glb, l.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
    HIPCHK(c, cp(io.gub, u.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
    if (R > 0) HIPCHK(c, cp(io.grows, r.data(), (size_t)R * 8, hipMemcpyHostToDevice));
    if (T > 0) HIPCHK(c, cp(io.gtan, r.data() + R, (size_t)T * 8, hipMemcpyHostToDevice));
    GlobIO pio = io;
    pio.flb_in = io.glb;
    pio.fub_in = io.gub;
    pio.frows = io.grows;
    pio.ftan = io.gtan;
    pio.in_tan = io.gtan;
    HIPCHK(c, launch_glob_linear(pio, stream));
    int r2 = mgpu_quad_fbbt_dev(c, 1, io.flb, io.fub, s.inc, s.qt, io.grows, 0, s.wlb.as<double>(),
                                s.wub.as<double>(), s.wrows.as<double>(), s.kinf.as<int32_t>(),
                                s.knm.as<int32_t>(), 0, nullptr, nullptr, nullptr, nullptr);
    if (r2 != MGPU_OK) return r2;
    HIPCHK(c, launch_glob_linear_verdict(pio, stream));
    if (T > 0) HIPCHK(c, launch_glob_pack(pio, stream));
    int32_t ki = 0;
    HIPCHK(c, cp(&ki, io.kinf, 4, hipMemcpyDeviceToHost));
    if (ki > 1)
      return fail(c, MGPU_ERR_ENGINE, "mgpu_glob_round: K2 failed on a strong-branching child");
    *inf = ki != 0;
    return MGPU_OK;
  };
  auto after_solve = [&]() {   // StrongBrancher::updateAfterSolve (:589-643)
    if (info.var < 0) return;
    const int j = info.var;
    double cost;
    bool down;
    if (info.isint) {
      cost = (obj - info.plb) / (std::fabs(x[(size_t)j] - info.act) + kSbEps);
      down = x[(size_t)j] < info.act;
    } else {
      down = info.act < 0;
      cost = (obj - info.plb) / ((down ? info.dd : info.ud) + kSbEps);
    }
    if (cost < 0.0 || std::isinf(cost) || std::isnan(cost)) cost = 0.0;
    if (down) {
      s.pc_dn[(size_t)j] = (s.pc_dn[(size_t)j] * s.tm_dn[(size_t)j] + cost) / (s.tm_dn[(size_t)j] + 1);
      s.tm_dn[(size_t)j] += 1;
    } else {
      s.pc_up[(size_t)j] = (s.pc_up[(size_t)j] * s.tm_up[(size_t)j] + cost) / (s.tm_up[(size_t)j] + 1);
      s.tm_up[(size_t)j] += 1;
    }
  };
  auto upd_pc = [&](int j, double cost, bool down) {   // updatePCost_ (:645-650)
    if (down) {
      s.pc_dn[(size_t)j] = (s.pc_dn[(size_t)j] * s.tm_dn[(size_t)j] + cost) / (s.tm_dn[(size_t)j] + 1);
      s.tm_dn[(size_t)j] += 1;
    } else {
      s.pc_up[(size_t)j] = (s.pc_up[(size_t)j] * s.tm_up[(size_t)j] + cost) / (s.tm_up[(size_t)j] + 1);
      s.tm_up[(size_t)j] += 1;
    }
  };
  std::vector<RsCand> cands;
  for (int iter = 1;; ++iter) {
    if (iter > 1) {   // re-solved: decide again
      rc = lp(0, true);
      if (rc != MGPU_OK) return rc;
      pivots += it;
    }
    if (dec == 1 || dec == 2 || dec == 4) return finish(dec, {});
    if (iter == 1) after_solve();
    if (dec == 3) {
      if (obj < s.inc) {
        s.inc = obj;
        s.best_x = x;
      }
      return finish(3, {});
    }
    if (iter == 1 && node.id == 0 && s.obbt) {   // tightenBounds_ (PCBProcessor.cpp:256-262)
      bool changed = false, feasible = true;
      rc = glob_root_obbt(c, s, x.data(), lb, ub, rec, &changed, &feasible, &obbt_lps);
      if (rc != MGPU_OK) return rc;
      if (changed) {
        HIPCHK(c, cp(s.wlb.p, lb.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
        HIPCHK(c, cp(s.wub.p, ub.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
        if (R > 0) HIPCHK(c, cp(s.wrows.p, rec.data(), (size_t)R * 8, hipMemcpyHostToDevice));
        if (T > 0) HIPCHK(c, cp(io.wvals, rec.data(), (size_t)RT * 8, hipMemcpyHostToDevice));
        if (!feasible) continue;
      }
    }
    if (T > 0) {   // separate_: the squares' tangents (glob_separate), then re-solve
      HIPCHK(c, hipMemsetAsync(s.acc.p, 0, 16, stream));
      HIPCHK(c, launch_glob_separate(io, stream));
      unsigned long long a[2] = {0, 0};
      HIPCHK(c, hipMemcpyAsync(a, s.acc.p, 16, hipMemcpyDeviceToHost, stream));
      HIPCHK(c, hipStreamSynchronize(stream));
      if (a[1] > 0) {
        s.tot.cuts += (long long)a[0];
        resolves += 1;
        HIPCHK(c, cp(rec.data(), io.wvals, (size_t)RT * 8, hipMemcpyDeviceToHost));
        continue;
      }
    }
    // ---- StrongBrancher::findBranches (StrongBrancher.cpp:184-264) ----
    // the children's warm start: the engine's basis now (PCBProcessor.cpp:
    // 282, getWarmStartCopy before findBranches), saved before the strong-
    // branching LPs chain through both slots
    const int ws_children = eng;
    int32_t *ch_head = s.rs_head.as<int32_t>();
    int8_t *ch_st = s.rs_st.as<int8_t>();
    if (eng != 0) {
      HIPCHK(c, cp(ch_head, eng == 1 ? hA : hB, (size_t)m * 4, hipMemcpyDeviceToDevice));
      HIPCHK(c, cp(ch_st, eng == 1 ? sA : sB, (size_t)N, hipMemcpyDeviceToDevice));
    }
    rs_candidates(q, x.data(), lb.data(), ub.data(), cands);
    if (cands.empty()) return finish(5, {});
    auto reliable = [&](int j) {
      return s.tm_up[(size_t)j] >= kSbThresh && s.tm_dn[(size_t)j] >= kSbThresh;
    };
    std::vector<RsCand> rel, unrel;
    for (const RsCand &cd : cands) (reliable(cd.var) ? rel : unrel).push_back(cd);
    // the node's value (the strong-branching LPs overwrite obj): the
    // children's bound and the pseudocosts' reference
    const double objval = obj, maxchange = s.inc - objval;
    const std::vector<double> xs = x;   // x_ (StrongBrancher copies x: solves overwrite it)
    double best = -INFINITY;
    int bc = -1;                          // the best candidate's variable
    std::vector<signed char> dirs((size_t)nv, -1);   // setDir; default UpBranch
    auto pick = [&](const RsCand &cd, double sc, double chu, double chd) {
      if (sc > best) {
        best = sc;
        bc = cd.var;
        dirs[(size_t)cd.var] = chu > chd ? 0 : 1;
      }
    };
    auto pcscore = [&](const RsCand &cd, double *chd, double *chu) {
      *chd = cd.dd * s.pc_dn[(size_t)cd.var];
      *chu = cd.ud * s.pc_up[(size_t)cd.var];
      return rs_score(*chu, *chd);
    };
    for (const RsCand &cd : rel) {
      double chd, chu;
      const double sc = pcscore(cd, &chd, &chu);
      pick(cd, sc, chu, chd);
    }
    // sortUnrelCands_ (:429-459)
    std::vector<double> vio;
    for (const RsCand &cd : unrel)
      vio.push_back(rs_score(cd.ud, cd.dd) /
                    (double)(std::max(s.tm_dn[(size_t)cd.var], s.tm_up[(size_t)cd.var]) + 1));
    double minscore = 0.0;
    if (!unrel.empty()) {
      std::vector<double> top = vio;
      std::sort(top.begin(), top.end(), [](double a, double b) { return a > b; });
      minscore = top[(size_t)std::min<size_t>(top.size(), (size_t)kSbCands) - 1];
    }
    int status = 0;   // 0 none, 1 pruned, 2 modified
    std::vector<double> mlb, mub, mrec;
    int cnt = 0;
    size_t i = 0;
    for (; i < unrel.size(); ++i) {
      if (cnt >= kSbCands) break;
      if (!(vio[i] >= minscore)) continue;
      const RsCand &cd = unrel[i];
      ++cnt;
      int sres[2];
      double ores[2];
      for (int side = 0; side < 2; ++side) {   // strongBranch_ (:499-587): down, then up
        std::vector<double> blb = lb, bub = ub, brec = rec;
        rs_br_mod(q, brec, blb, bub, xs.data(), cd.var, cd.isint, side == 0);
        bool inf = false;
        rc = presolve(blb, bub, brec, &inf);
        if (rc != MGPU_OK) return rc;
        if (inf) {
          sres[side] = 2;
          ores[side] = s.last_val;
          continue;
        }
        rc = lp(kSbIter, false);
        if (rc != MGPU_OK) return rc;
        sb_lps += 1;
        sres[side] = st;
        ores[side] = obj;
      }
      double chu = std::max(ores[1] - objval, 0.0), chd = std::max(ores[0] - objval, 0.0);
      // useStrongBranchInfo_ (:652-689)
      bool is_rel = true;
      const bool pdn = rs_prune(maxchange, chd, sres[0], &is_rel);
      const bool pup = rs_prune(maxchange, chu, sres[1], &is_rel);
      if (!is_rel) {
        chu = chd = 0.0;
      } else if (pup && pdn) {
        status = 1;
      } else if (pup || pdn) {
        status = 2;
        mlb = lb;
        mub = ub;
        mrec = rec;
        rs_br_mod(q, mrec, mlb, mub, xs.data(), cd.var, cd.isint, pup);
      } else {
        upd_pc(cd.var, std::fabs(chd) / (std::fabs(cd.dd) + kSbEps), true);
        upd_pc(cd.var, std::fabs(chu) / (std::fabs(cd.ud) + kSbEps), false);
      }
      const double sc = rs_score(chu, chd);
      if (status != 0) break;
      pick(cd, sc, chu, chd);
    }
    if (status == 1) return finish(1, {});
    if (status == 2) {   // ModifiedByBrancher: the mod, presolveNode_, re-solve
      lb = mlb;
      ub = mub;
      rec = mrec;
      bool inf = false;
      rc = presolve(lb, ub, rec, &inf);
      if (rc != MGPU_OK) return rc;
      if (inf) return finish(1, {});
      HIPCHK(c, cp(lb.data(), io.wlb, (size_t)nv * 8, hipMemcpyDeviceToHost));
      HIPCHK(c, cp(ub.data(), io.wub, (size_t)nv * 8, hipMemcpyDeviceToHost));
      if (RT > 0) HIPCHK(c, cp(rec.data(), dvals, (size_t)RT * 8, hipMemcpyDeviceToHost));
      continue;
    }
    for (size_t jx = 0; jx < unrel.size(); ++jx) {   // :149-169
      if (vio[jx] < minscore || jx >= i) {
        double chd, chu;
        const double sc = pcscore(unrel[jx], &chd, &chu);
        pick(unrel[jx], sc, chu, chd);
      }
    }
    if (best == 0 && rel.empty())   // :170-180: the first largest violation
      bc = unrel[(size_t)(std::max_element(vio.begin(), vio.end()) - vio.begin())].var;
    if (bc < 0) return finish(5, {});
    const RsCand *bcand = nullptr;
    for (const RsCand &cd : cands)
      if (cd.var == bc) bcand = &cd;
    // the children (QuadHandler::getBranches down, up; IntVarHandler's
    // guided dive, else the candidate's direction), each with the node's box,
    // record and basis
    const int j = bcand->var;
    const double v = xs[(size_t)j];
    const bool up_first = dirs[(size_t)j] != 0;
    bool down_first = true;
    if (bcand->isint) {
      down_first = !up_first;
      if (std::isfinite(s.inc) && !std::isnan(s.best_x[(size_t)j])) down_first = s.best_x[(size_t)j] < v;
    }
    if (bcand->isint) s.tot.br_int += 1;
    else s.tot.br_cont += 1;
    std::vector<GHeap> kids;
    for (int k = 0; k < 2; ++k) {
      const bool upc = down_first ? k == 1 : k == 0;
      int slot;
      if (!s.free_slots.empty()) {
        slot = s.free_slots.back();
        s.free_slots.pop_back();
      } else {
        if (s.hw >= s.cap) return fail(c, MGPU_ERR_NOMEM, "mgpu_glob_round: node pool full (%d slots)", s.cap);
        slot = s.hw++;
      }
      std::vector<double> clb = lb, cub = ub;
      if (upc) clb[(size_t)j] = bcand->isint ? std::ceil(v) : v;
      else cub[(size_t)j] = bcand->isint ? std::floor(v) : v;
      const size_t so = (size_t)slot;
      HIPCHK(c, cp(s.plb.as<double>() + so * nv, clb.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
      HIPCHK(c, cp(s.pub.as<double>() + so * nv, cub.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
      if (R > 0) HIPCHK(c, cp(s.prows.as<double>() + so * R, rec.data(), (size_t)R * 8, hipMemcpyHostToDevice));
      if (T > 0) HIPCHK(c, cp(s.ptan.as<double>() + so * T, rec.data() + R, (size_t)T * 8, hipMemcpyHostToDevice));
      const uint8_t ok = ws_children != 0 ? 1 : 0;
      if (ok) {
        HIPCHK(c, cp(s.pws_head.as<int32_t>() + so * m, ch_head, (size_t)m * 4, hipMemcpyDeviceToDevice));
        HIPCHK(c, cp(s.pws_st.as<int8_t>() + so * N, ch_st, (size_t)N, hipMemcpyDeviceToDevice));
      }
      HIPCHK(c, cp(s.pws_ok.as<uint8_t>() + so, &ok, 1, hipMemcpyHostToDevice));
      const int32_t dep = node.depth + 1;
      HIPCHK(c, cp(s.pnlb.as<double>() + so, &objval, 8, hipMemcpyHostToDevice));
      HIPCHK(c, cp(s.pdepth.as<int32_t>() + so, &dep, 4, hipMemcpyHostToDevice));
      GlobState::BrInfo bi;
      bi.var = j;
      bi.isint = bcand->isint;
      bi.act = bcand->isint ? v : (upc ? 1.0 : -1.0);
      bi.dd = bcand->dd;
      bi.ud = bcand->ud;
      bi.plb = objval;
      s.pinfo[so] = bi;
      kids.push_back(GHeap{objval, node.depth + 1, s.next_id++, slot});
    }
    return finish(0, kids);
  }
}

}  // namespace

extern "C" {

int mgpu_glob_brancher(mgpu_ctx *c, int kind) {
  if (!c) return MGPU_ERR_ARG;
  if (kind < 0 || kind > 1)
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_brancher: kind %d (0 MaxVio, 1 relstronger)", kind);
  c->glob_brancher = kind;
  return MGPU_OK;
}

int mgpu_glob_config(mgpu_ctx *c, int order, int warm, int qt, int lin, int obbt) {
  if (!c) return MGPU_ERR_ARG;
  if ((order != 0 && order != 2) || warm < 0 || warm > 1 || qt < 0 || qt > 1 || lin < 0 ||
      lin > 1 || obbt < 0 || obbt > 1)
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_config: order %d (0, 2), warm %d (0, 1), qt %d (0, 1), "
                "lin %d (0, 1), obbt %d (0, 1)", order, warm, qt, lin, obbt);
  c->glob_order = order;
  c->glob_warm = warm;
  c->glob_qt = qt;
  c->glob_lin = lin;
  c->glob_obbt = obbt;
  return MGPU_OK;
}

int mgpu_glob_init(mgpu_ctx *c, int capacity, double incumbent) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded || !c->quad || !c->nr_set)
    return fail(c, MGPU_ERR_STATE, "mgpu_glob_init: load the relaxation LP (mgpu_load_lp), the "
                "quadratic problem (mgpu_load_quad) and the node-rows map first");
  const QuadState &q = *c->quad;
  const int nsq = (int)q.sq_x.size();
  // record = R row-state values, then 2 S tangent values per square
  const int extra = c->nr_stride - q.R;
  if (c->lp.n != q.nv || extra < 0 || (extra > 0 && (nsq == 0 || extra % (2 * nsq) != 0)))
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_init: LP columns (%d) / row-record stride (%d) do "
                "not match the quadratic problem (%d vars, %d row values, %d squares)", c->lp.n,
                c->nr_stride, q.nv, q.R, nsq);
  if (capacity < 1) return fail(c, MGPU_ERR_ARG, "mgpu_glob_init: capacity < 1");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  glob_state_free(c);
  GlobState *s = new GlobState();
  c->glob = s;
  const int nv = q.nv, R = q.R, m = c->lp.m, N = nv + m;
  s->nv = nv;
  s->R = R;
  s->order = c->glob_order;
  s->warm = c->glob_warm;
  s->qt = c->glob_qt;
  s->lin = c->glob_lin;
  s->obbt = c->glob_obbt;
  s->brancher = c->glob_brancher;
  if (s->brancher == 1 && (s->order != 2 || s->warm != 1 || s->lin != 1))
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_init: relstronger needs order 2, warm 1 and lin 1 "
                "(a brancher's modification reaches p_ only through LinearHandler's "
                "copyBndsFromRel_)");
  if (s->brancher == 1) {
    HIPCHK(c, s->rs_head.ensure((size_t)c->lp.m * 4 + 4));
    HIPCHK(c, s->rs_st.ensure((size_t)(nv + c->lp.m)));
    s->pinfo.assign((size_t)capacity, GlobState::BrInfo{});
    s->pc_up.assign((size_t)nv, 0.0);
    s->pc_dn.assign((size_t)nv, 0.0);
    s->tm_up.assign((size_t)nv, 0);
    s->tm_dn.assign((size_t)nv, 0);
  }
  s->T = extra;
  s->S = nsq > 0 ? extra / (2 * nsq) : 0;
  if (s->lin || s->obbt) {
    const int rc0 = build_linear_table(c, *s);
    if (rc0 != MGPU_OK) return rc0;
  }
  s->cap = capacity;
  s->inc = incumbent;
  s->best_x.assign((size_t)nv, NAN);
  s->tot.incumbent = incumbent;
  HIPCHK(c, s->plb.ensure((size_t)capacity * nv * 8));
  HIPCHK(c, s->pub.ensure((size_t)capacity * nv * 8));
  HIPCHK(c, s->prows.ensure((size_t)capacity * (R > 0 ? R : 1) * 8));
  HIPCHK(c, s->pnlb.ensure((size_t)capacity * 8));
  HIPCHK(c, s->pdepth.ensure((size_t)capacity * 4));
  // the problem data of the decision kernel
  std::vector<uint8_t> vt((size_t)nv);
  for (int j = 0; j < nv; ++j) vt[(size_t)j] = (uint8_t)q.h_vtype[(size_t)j];
  HIPCHK(c, upload(s->fvtype, vt.data(), vt.size()));
  HIPCHK(c, upload(s->flptr, q.h_lptr.data(), q.h_lptr.size()));
  HIPCHK(c, upload(s->flvar, q.h_lvar.data(), q.h_lvar.size()));
  HIPCHK(c, upload(s->flval, q.h_lval.data(), q.h_lval.size()));
  HIPCHK(c, upload(s->fqptr, q.h_qptr.data(), q.h_qptr.size()));
  HIPCHK(c, upload(s->fqv1, q.h_qv1.data(), q.h_qv1.size()));
  HIPCHK(c, upload(s->fqv2, q.h_qv2.data(), q.h_qv2.size()));
  HIPCHK(c, upload(s->fqval, q.h_qval.data(), q.h_qval.size()));
  HIPCHK(c, upload(s->fclb, q.h_clb.data(), q.h_clb.size()));
  HIPCHK(c, upload(s->fcub, q.h_cub.data(), q.h_cub.size()));
  // the root: the loaded column bounds, QuadHandler::relax_'s rows there
  std::vector<double> lb((size_t)nv), ub((size_t)nv), rows((size_t)(R > 0 ? R : 1));
  HIPCHK(c, hipMemcpy(lb.data(), c->collb.p, (size_t)nv * 8, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(ub.data(), c->colub.p, (size_t)nv * 8, hipMemcpyDeviceToHost));
  int rc = mgpu_quad_rows(c, lb.data(), ub.data(), rows.data(), nullptr);
  if (rc != MGPU_OK) return rc;
  const double ninf = -INFINITY;
  const int32_t zero = 0;
  HIPCHK(c, hipMemcpy(s->plb.p, lb.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(s->pub.p, ub.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
  if (R > 0) HIPCHK(c, hipMemcpy(s->prows.p, rows.data(), (size_t)R * 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(s->pnlb.p, &ninf, 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(s->pdepth.p, &zero, 4, hipMemcpyHostToDevice));
  if (s->T > 0) {   // the root's tangent slots, all free: [0, +inf]
    HIPCHK(c, s->ptan.ensure((size_t)capacity * s->T * 8));
    std::vector<double> t0((size_t)s->T, 0.0);
    for (int k = 1; k < s->T; k += 2) t0[(size_t)k] = INFINITY;
    HIPCHK(c, hipMemcpy(s->ptan.p, t0.data(), (size_t)s->T * 8, hipMemcpyHostToDevice));
  }
  s->count = 1;
  if (s->order == 2) {   // the root is node 0 in slot 0
    s->heap.push_back(GHeap{-INFINITY, 0, 0, 0});
    s->next_id = 1;
    s->hw = 1;
  }
  if (s->warm == 1) {    // per slot: the parent's basis; the root has none (slack basis)
    HIPCHK(c, s->pws_head.ensure((size_t)capacity * m * 4));
    HIPCHK(c, s->pws_st.ensure((size_t)capacity * N));
    HIPCHK(c, s->pws_ok.ensure((size_t)capacity));
    HIPCHK(c, hipMemset(s->pws_ok.p, 0, (size_t)capacity));
  }
  // the root basis every node LP refactors for its own rows: the loaded LP
  // (the root's rows) from the slack basis
  HIPCHK(c, s->ws_head.ensure((size_t)m * 4 + 4));
  HIPCHK(c, s->ws_st.ensure((size_t)N));
  HIPCHK(c, s->ws_d.ensure((size_t)N * 8));
  HIPCHK(c, s->ws_binv.ensure((size_t)m * m * 8 + 8));
  for (DevBuf *b : {&s->r_st, &s->r_it}) HIPCHK(c, b->ensure(4));
  HIPCHK(c, s->r_obj.ensure(8));
  rc = mgpu_lp_solve_dev(c, 1, c->collb.as<double>(), c->colub.as<double>(), nullptr, nullptr,
                         nullptr, nullptr, nullptr, 1, 0, s->r_st.as<int32_t>(),
                         s->r_obj.as<double>(), s->r_it.as<int32_t>(), nullptr,
                         s->ws_head.as<int32_t>(), s->ws_st.as<int8_t>(), s->ws_d.as<double>(),
                         s->ws_binv.as<double>());
  if (rc != MGPU_OK) return rc;
  int32_t rst = 0;
  HIPCHK(c, hipMemcpyAsync(&rst, s->r_st.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  s->root_ws = rst == 0;
  s->tot.open = 1;
  return MGPU_OK;
}

int mgpu_glob_round(mgpu_ctx *c, int batch, double incumbent, mgpu_glob_stats *stats) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->glob) return fail(c, MGPU_ERR_STATE, "mgpu_glob_round: mgpu_glob_init first");
  if (batch < 1) return fail(c, MGPU_ERR_ARG, "mgpu_glob_round: batch < 1");
  GlobState &s = *c->glob;
  if (s.brancher == 1) batch = 1;   // relstronger: the reference's node at a time
  const QuadState &q = *c->quad;
  HIPCHK(c, hipSetDevice(c->device));
  if (incumbent < s.inc) {  // an outside incumbent: no point of ours matches it
    s.inc = incumbent;
    std::fill(s.best_x.begin(), s.best_x.end(), NAN);
  }
  const bool heap = s.order == 2;
  const int nv = s.nv, R = s.R, m = c->lp.m, N = nv + m;
  int nb = 0, base = 0;
  std::vector<int32_t> sel;
  std::vector<GHeap> popped;
  if (heap) {
    // TreeManager::getCandidate: the heap top, pruned lazily by the
    // incumbent (TreeManager::shouldPrune_, :403-413)
    while ((int)sel.size() < batch && !s.heap.empty()) {
      const GHeap top = s.heap.front();
      std::pop_heap(s.heap.begin(), s.heap.end(), gheap_greater);
      s.heap.pop_back();
      if (top.lb > s.inc - 1e-6 ||
          std::fabs(s.inc - top.lb) / (std::fabs(s.inc) + 1e-6) * 100.0 < 1e-6) {
        s.free_slots.push_back(top.slot);
        continue;
      }
      sel.push_back(top.slot);
      popped.push_back(top);
    }
    nb = (int)sel.size();
    // children: two per node in the round's own slots, the free ones, then new
    const long need = (long)nb - (long)s.free_slots.size();
    if (nb > 0 && s.hw + (need > 0 ? need : 0) > s.cap)
      return fail(c, MGPU_ERR_NOMEM, "mgpu_glob_round: node pool full (%d slots)", s.cap);
  } else {
    nb = batch < s.count ? batch : s.count;
    if (s.count + nb > s.cap) nb = s.cap - s.count;  // children must fit: base + 2 nb <= cap
    if (nb <= 0 && s.count > 0) return fail(c, MGPU_ERR_NOMEM, "mgpu_glob_round: node pool full");
    base = s.count - nb;
  }
  if (nb <= 0) {
    s.count = heap ? 0 : s.count;
    s.tot.open = 0;
    if (stats) *stats = s.tot;
    return MGPU_OK;
  }
  int rc = ensure_glob_batch(c, s, nb);
  if (rc != MGPU_OK) return rc;
  GlobIO io{};
  io.nb = nb;
  io.base = base;
  io.nv = nv;
  io.R = R;
  io.m = m;
  io.N = N;
  io.vtype = s.fvtype.as<uint8_t>();
  io.nsq = (int)q.sq_x.size();
  io.nbil = (int)q.bil_x0.size();
  io.ncon = q.ncon;
  io.nfun = q.ncon + (q.has_obj ? 1 : 0);
  io.sq = q.dq.sq;
  io.bil = q.dq.bil;
  io.lptr = s.flptr.as<int32_t>();
  io.lvar = s.flvar.as<int32_t>();
  io.lval = s.flval.as<double>();
  io.qptr = s.fqptr.as<int32_t>();
  io.qv1 = s.fqv1.as<int32_t>();
  io.qv2 = s.fqv2.as<int32_t>();
  io.qval = s.fqval.as<double>();
  io.clb = s.fclb.as<double>();
  io.cub = s.fcub.as<double>();
  io.obj_const = q.obj_const;
  io.inc = s.inc;
  io.abs_tol = 1e-6;   // solAbs_tol / solRel_tol (Environment.cpp:486, 509-528)
  io.rel_tol = 1e-6;
  io.kinf = s.kinf.as<int32_t>();
  io.wlb = s.wlb.as<double>();
  io.wub = s.wub.as<double>();
  io.wrows = s.wrows.as<double>();
  io.status = s.st.as<int32_t>();
  io.iters = s.it.as<int32_t>();
  io.obj = s.obj.as<double>();
  io.x = s.x.as<double>();
  io.cand = s.cand.as<double>();
  io.dec = s.dec.as<int32_t>();
  io.bvar = s.bvar.as<int32_t>();
  io.pos = s.pos.as<int32_t>();
  io.depth_in = s.depth_in.as<int32_t>();
  io.bval = s.bval.as<double>();
  io.bup = s.bup.as<int8_t>();
  io.bint = s.bint.as<int8_t>();
  io.out = s.out.as<GlobOut>();
  io.plb = s.plb.as<double>();
  io.pub = s.pub.as<double>();
  io.prows = s.prows.as<double>();
  io.pnlb = s.pnlb.as<double>();
  io.pdepth = s.pdepth.as<int32_t>();
  io.S = s.S;
  io.T = s.T;
  io.ptan = s.T > 0 ? s.ptan.as<double>() : nullptr;
  io.wvals = s.T > 0 ? s.wvals.as<double>() : s.wrows.as<double>();
  io.flag = s.flag.as<int32_t>();
  io.skip2 = s.skip2.as<int32_t>();
  io.skip_a = s.skip_a.as<int32_t>();
  io.st2 = s.st2.as<int32_t>();
  io.it2 = s.it2.as<int32_t>();
  io.obj2 = s.obj2.as<double>();
  io.x2 = s.x2.as<double>();
  io.acc = s.acc.as<unsigned long long>();
  if (s.warm == 1) {
    io.pws_head = s.pws_head.as<int32_t>();
    io.pws_st = s.pws_st.as<int8_t>();
    io.pws_ok = s.pws_ok.as<uint8_t>();
    io.ghead = s.ghead.as<int32_t>();
    io.gst = s.gst.as<int8_t>();
    io.gok = s.gok.as<uint8_t>();
    io.wo_head = s.wo_head.as<int32_t>();
    io.wo_st = s.wo_st.as<int8_t>();
  }
  // the round's input nodes
  const double *in_lb, *in_ub, *in_rows;
  if (heap) {
    HIPCHK(c, hipMemcpyAsync(s.gsel.p, sel.data(), (size_t)nb * 4, hipMemcpyHostToDevice,
                             c->stream));
    io.sel = s.gsel.as<int32_t>();
    io.glb = s.glb.as<double>();
    io.gub = s.gub.as<double>();
    io.grows = s.grows.as<double>();
    io.gtan = s.gtan.as<double>();
    io.gdepth = s.gdepth.as<int32_t>();
    HIPCHK(c, launch_glob_gather(io, c->stream));
    for (int32_t sl : sel) s.free_slots.push_back(sl);   // the round's slots are free now
    in_lb = io.glb;
    in_ub = io.gub;
    in_rows = io.grows;
    io.in_depth = io.gdepth;
    io.in_tan = io.gtan;
  } else {
    if (s.warm == 1) {   // the stack's top nb slots: their bases in place
      io.ghead = s.pws_head.as<int32_t>() + (size_t)base * m;
      io.gst = s.pws_st.as<int8_t>() + (size_t)base * N;
      io.gok = s.pws_ok.as<uint8_t>() + base;
    }
    in_lb = s.plb.as<double>() + (size_t)base * nv;
    in_ub = s.pub.as<double>() + (size_t)base * nv;
    in_rows = s.prows.as<double>() + (size_t)base * R;
    io.in_depth = s.pdepth.as<int32_t>() + base;
    io.in_tan = s.T > 0 ? s.ptan.as<double>() + (size_t)base * s.T : nullptr;
  }
  // the handlers' presolveNode in order (PCBProcessor.cpp:148-167):
  // LinearHandler's over the node's relaxation rows as the node inherited
  // them, then QuadHandler's on the box that leaves
  if (s.lin) {
    io.M = s.M;
    io.nobj = s.nobj;
    io.cons_bad = s.cons_bad;
    // a solution in the pool (LinearHandler.cpp:1636-1640)
    io.has_inc = std::isfinite(s.inc) ? 1 : 0;
    io.inc_ub = s.inc - q.obj_const;
    io.lrptr = s.lrptr.as<int32_t>();
    io.ltvar = s.ltvar.as<int32_t>();
    io.ltsrc = s.ltsrc.as<int32_t>();
    io.ltrow = s.ltrow.as<int32_t>();
    io.lrhsrc = s.lrhsrc.as<int32_t>();
    io.lcptr = s.lcptr.as<int32_t>();
    io.lcterm = s.lcterm.as<int32_t>();
    io.loidx = s.loidx.as<int32_t>();
    io.ltval = s.ltval.as<double>();
    io.lrlo = s.lrlo.as<double>();
    io.lrhi = s.lrhi.as<double>();
    io.loval = s.loval.as<double>();
    io.flb_in = in_lb;
    io.fub_in = in_ub;
    io.frows = in_rows;
    io.ftan = io.in_tan;
    io.flb = s.flb.as<double>();
    io.fub = s.fub.as<double>();
    io.finf = s.finf.as<int32_t>();
    io.fflag = s.fflag.as<uint8_t>();
    HIPCHK(c, launch_glob_linear(io, c->stream));
    in_lb = io.flb;
    in_ub = io.fub;
  }
  // K2 from the parents' rows; tightenQuad_ at every node (doQT_, set by
  // Glob's presolve) or only at the first presolveNode call (QuadHandler.cpp:
  // 1215, 1241: niters <= 1)
  const int qt = (s.qt || s.tot.nodes == 0) ? 1 : 0;
  rc = mgpu_quad_fbbt_dev(c, nb, in_lb, in_ub, s.inc, qt, in_rows, 0, s.wlb.as<double>(),
                          s.wub.as<double>(), s.wrows.as<double>(), s.kinf.as<int32_t>(),
                          s.knm.as<int32_t>(), 0, nullptr, nullptr, nullptr, nullptr);
  if (rc != MGPU_OK) return rc;
  if (s.lin) HIPCHK(c, launch_glob_linear_verdict(io, c->stream));
  // the node records: K2's rows and the node's tangent slots
  if (s.T > 0) HIPCHK(c, launch_glob_pack(io, c->stream));
  // the node LPs with their own rows (K3R + K3), K2-infeasible nodes skipped.
  // warm 0: every node from the root basis refactored for its rows; warm 1:
  // from its parent's optimal basis refactored for its rows, as HipLPEngine
  // refactors the kept basis after NodeIncRelaxer replays the rows
  // (HipLPEngine::refactor_; OsiLPEngine: Clp), the root from the slack basis
  LpWarmOut wo{s.wo_head.as<int32_t>(), s.wo_st.as<int8_t>(), s.wo_d.as<double>(),
               s.wo_binv.as<double>()};
  auto solve = [&](const int32_t *skip, const int32_t *head, const int8_t *st_in, int shared,
                   const double *binv, int32_t *st, double *obj, int32_t *it, double *x) {
    return lp_solve_rows_wo(c, nb, s.wlb.as<double>(), s.wub.as<double>(), skip, io.wvals, head,
                            st_in, shared, 0, st, obj, it, x, binv,
                            s.warm == 1 ? &wo : nullptr);
  };
  if (s.warm == 1) {
    HIPCHK(c, launch_glob_skips(io, c->stream));
    rc = solve(io.skip_a, io.ghead, io.gst, 0, nullptr, s.st.as<int32_t>(), s.obj.as<double>(),
               s.it.as<int32_t>(), s.x.as<double>());
    if (rc != MGPU_OK) return rc;
    // the nodes without a basis (the root): from the slack basis, into the
    // same x and bases, merged by flag
    bool cold = !heap;
    if (heap)
      for (const GHeap &g : popped) cold |= g.id == 0;
    if (cold) {
      rc = solve(io.skip2, nullptr, nullptr, 1, nullptr, s.st2.as<int32_t>(), s.obj2.as<double>(),
                 s.it2.as<int32_t>(), s.x.as<double>());
      if (rc != MGPU_OK) return rc;
      GlobIO mio = io;
      mio.x2 = io.x;   // (the cold call wrote x in place)
      HIPCHK(c, launch_glob_merge(mio, c->stream));
    }
  } else {
    rc = solve(s.kinf.as<int32_t>(), s.root_ws ? s.ws_head.as<int32_t>() : nullptr,
               s.root_ws ? s.ws_st.as<int8_t>() : nullptr, 1,
               s.root_ws ? s.ws_binv.as<double>() : nullptr, s.st.as<int32_t>(),
               s.obj.as<double>(), s.it.as<int32_t>(), s.x.as<double>());
    if (rc != MGPU_OK) return rc;
  }
  HIPCHK(c, launch_glob_decide(io, c->stream));
  if (s.brancher == 1) return glob_node_rs(c, s, io, popped[0], stats);
  // the flagged nodes (flag / skip2) re-solved -- from the root basis (warm
  // 0) or the node's last basis refactored for its rows (warm 1) -- merged
  // back and decided again
  auto resolve_flagged = [&]() -> int {
    int r;
    if (s.warm == 1)
      r = solve(io.skip2, s.wo_head.as<int32_t>(), s.wo_st.as<int8_t>(), 0, nullptr,
                s.st2.as<int32_t>(), s.obj2.as<double>(), s.it2.as<int32_t>(), s.x2.as<double>());
    else
      r = solve(io.skip2, s.root_ws ? s.ws_head.as<int32_t>() : nullptr,
                s.root_ws ? s.ws_st.as<int8_t>() : nullptr, 1,
                s.root_ws ? s.ws_binv.as<double>() : nullptr, s.st2.as<int32_t>(),
                s.obj2.as<double>(), s.it2.as<int32_t>(), s.x2.as<double>());
    if (r != MGPU_OK) return r;
    HIPCHK(c, launch_glob_merge(io, c->stream));
    GlobIO again = io;
    again.only = io.flag;
    HIPCHK(c, launch_glob_decide(again, c->stream));
    return MGPU_OK;
  };
  // root OBBT (PCBProcessor::process, :256-280): at the root's first solve,
  // when it is neither pruned nor feasible, QuadHandler::postSolveRootNode;
  // if its point leaves the tightened relaxation the root is re-solved
  // (SepaResolve, no separation in between), else it is decided again on the
  // same point with the tightened box
  long long obbt_lps = 0, obbt_resolves = 0;
  if (s.obbt && s.tot.nodes == 0 && nb == 1) {
    int32_t d0 = -1;
    HIPCHK(c, hipMemcpyAsync(&d0, io.dec, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (d0 == 0 || d0 == 5) {
      const int RT = R + s.T;
      std::vector<double> x0((size_t)nv), lb0((size_t)nv), ub0((size_t)nv), rec((size_t)RT);
      HIPCHK(c, hipMemcpy(x0.data(), io.x, (size_t)nv * 8, hipMemcpyDeviceToHost));
      HIPCHK(c, hipMemcpy(lb0.data(), io.wlb, (size_t)nv * 8, hipMemcpyDeviceToHost));
      HIPCHK(c, hipMemcpy(ub0.data(), io.wub, (size_t)nv * 8, hipMemcpyDeviceToHost));
      if (RT > 0) HIPCHK(c, hipMemcpy(rec.data(), io.wvals, (size_t)RT * 8, hipMemcpyDeviceToHost));
      bool changed = false, feasible = true;
      rc = glob_root_obbt(c, s, x0.data(), lb0, ub0, rec, &changed, &feasible, &obbt_lps);
      if (rc != MGPU_OK) return rc;
      if (changed) {
        HIPCHK(c, hipMemcpy(s.wlb.p, lb0.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(s.wub.p, ub0.data(), (size_t)nv * 8, hipMemcpyHostToDevice));
        if (R > 0) HIPCHK(c, hipMemcpy(s.wrows.p, rec.data(), (size_t)R * 8, hipMemcpyHostToDevice));
        if (s.T > 0) HIPCHK(c, hipMemcpy(io.wvals, rec.data(), (size_t)RT * 8, hipMemcpyHostToDevice));
        const int32_t one = 1, zero = 0;
        HIPCHK(c, hipMemcpy(io.flag, &one, 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(io.skip2, &zero, 4, hipMemcpyHostToDevice));
        if (!feasible) {
          rc = resolve_flagged();
          if (rc != MGPU_OK) return rc;
          obbt_resolves = 1;
        } else {
          GlobIO again = io;
          again.only = io.flag;
          HIPCHK(c, launch_glob_decide(again, c->stream));
        }
      }
    }
  }
  // the separation loop (PCBProcessor.cpp:267-280): every pass adds at least
  // one cut to a free slot, so it ends within nsq S passes
  long long cuts = 0, resolves = 0;
  for (int pass = 0; s.T > 0 && pass <= s.T / 2; ++pass) {
    HIPCHK(c, hipMemsetAsync(s.acc.p, 0, 16, c->stream));
    HIPCHK(c, launch_glob_separate(io, c->stream));
    unsigned long long a[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(a, s.acc.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (a[1] == 0) break;
    cuts += (long long)a[0];
    resolves += (long long)a[1];
    rc = resolve_flagged();
    if (rc != MGPU_OK) return rc;
  }
  HIPCHK(c, launch_glob_summary(io, c->stream));
  GlobOut o;
  if (heap) {
    // the children in the reference's branch order: QuadHandler::getBranches
    // down then up (QuadHandler.cpp:422-471); IntVarHandler::getBranches the
    // guided dive's side first with an incumbent, else the candidate's
    // preferred direction (IntVarHandler.cpp:133-190)
    std::vector<int32_t> dec(nb), bvar(nb), pos(nb), dep(nb);
    std::vector<double> obj(nb), bval(nb);
    std::vector<int8_t> bup(nb), bint(nb);
    HIPCHK(c, hipMemcpyAsync(&o, s.out.p, sizeof o, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(dec.data(), io.dec, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(bvar.data(), io.bvar, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(pos.data(), io.pos, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(dep.data(), io.depth_in, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(obj.data(), io.obj, (size_t)nb * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(bval.data(), io.bval, (size_t)nb * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(bup.data(), io.bup, (size_t)nb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(bint.data(), io.bint, (size_t)nb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // the incumbent this round found (for the guided dive of its own nodes'
    // children the reference already has it: a node's solution enters the
    // pool before the next node branches; at batch 1 no other node shares
    // the round)
    std::vector<int32_t> cs((size_t)o.nchild);
    size_t nfree = 0;
    auto take = [&]() -> int {
      if (nfree < s.free_slots.size()) return s.free_slots[nfree++];
      return s.hw++;
    };
    struct Kid {
      double lb;
      int depth, slot;
    };
    std::vector<Kid> kids;
    for (int i = 0; i < nb; ++i) {
      if (dec[i] != 0) continue;
      const int s_down = take(), s_up = take();
      cs[(size_t)pos[i]] = s_down;
      cs[(size_t)pos[i] + 1] = s_up;
      bool down_first = true;
      if (bint[i]) {
        down_first = bup[i] == 0;
        if (std::isfinite(s.inc) && !std::isnan(s.best_x[(size_t)bvar[i]]))
          down_first = s.best_x[(size_t)bvar[i]] < bval[i];
      }
      kids.push_back({obj[i], dep[i] + 1, down_first ? s_down : s_up});
      kids.push_back({obj[i], dep[i] + 1, down_first ? s_up : s_down});
    }
    s.free_slots.erase(s.free_slots.begin(), s.free_slots.begin() + (long)nfree);
    if (!cs.empty()) {
      HIPCHK(c, hipMemcpyAsync(s.cslots.p, cs.data(), cs.size() * 4, hipMemcpyHostToDevice,
                               c->stream));
      io.child_slots = s.cslots.as<int32_t>();
      HIPCHK(c, launch_glob_children(io, c->stream));
    }
    for (const Kid &k : kids) {
      s.heap.push_back(GHeap{k.lb, k.depth, s.next_id++, k.slot});
      std::push_heap(s.heap.begin(), s.heap.end(), gheap_greater);
    }
    s.count = (int)s.heap.size();
  } else {
    HIPCHK(c, launch_glob_children(io, c->stream));
    HIPCHK(c, hipMemcpyAsync(&o, s.out.p, sizeof o, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    s.count = base + o.nchild;
  }
  if (o.best_idx >= 0 && o.best < s.inc) {
    s.inc = o.best;
    HIPCHK(c, hipMemcpy(s.best_x.data(), s.x.as<double>() + (size_t)o.best_idx * nv,
                        (size_t)nv * 8, hipMemcpyDeviceToHost));
  }
  s.tot.rounds += 1;
  s.tot.nodes += nb;
  for (int k = 0; k < 6; ++k) s.tot.ndec[k] += o.ndec[k];
  s.tot.lps += o.lps + resolves + obbt_resolves;
  s.tot.obbt_lps += obbt_lps;
  s.tot.pivots += o.pivots;
  s.tot.cuts += cuts;
  s.tot.resolves += resolves;
  s.tot.br_int += o.br_int;
  s.tot.br_cont += o.ndec[0] - o.br_int;
  s.tot.open = s.count;
  s.tot.last_batch = nb;
  s.tot.incumbent = s.inc;
  if (stats) *stats = s.tot;
  if (o.ndec[4] > 0)
    return fail(c, MGPU_ERR_ENGINE, "mgpu_glob_round: %lld nodes ended with an engine problem "
                "(K2 propagation cap / default bound, or an unbounded / unknown LP status)",
                (long long)o.ndec[4]);
  return MGPU_OK;
}

int mgpu_glob_lp_log(mgpu_ctx *c, int cap, int32_t *status, double *value, int32_t *iters) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->glob) return fail(c, MGPU_ERR_STATE, "mgpu_glob_lp_log: mgpu_glob_init first");
  const auto &lg = c->glob->lp_log;
  for (size_t k = 0; k < lg.size() && (int)k < cap; ++k) {
    if (status) status[k] = lg[k].status;
    if (value) value[k] = lg[k].value;
    if (iters) iters[k] = lg[k].iters;
  }
  return (int)lg.size();
}

int mgpu_glob_best(mgpu_ctx *c, double *obj, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->glob) return fail(c, MGPU_ERR_STATE, "mgpu_glob_best: mgpu_glob_init first");
  if (obj) *obj = c->glob->inc;
  if (x) std::memcpy(x, c->glob->best_x.data(), (size_t)c->glob->nv * 8);
  return MGPU_OK;
}

}  // extern "C"
