// Batched spatial branch-and-bound over the McCormick relaxation: the node
// loop of the reference's glob solver (Glob::createBab_, src/solvers/
// Glob.cpp:134-220: BranchAndBound + NodeIncRelaxer + PCBProcessor with
// IntVarHandler, LinearHandler, QuadHandler and, brancher=maxvio,
// MaxVioBrancher; BranchAndBound.cpp:424-514) for a QCQP after
// SimpleTransformer: one round pops the top B open nodes of an HBM stack and
// runs, all on the device,
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
//   children   two per branched node, each with the node's tightened box,
//        the branching bound and the node's rows.
// One small record comes back per round (counts, best feasible node).
#include <algorithm>
#include <cmath>
#include <cstring>
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
  int order = 0, warm = 0, qt = 1;
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
  void release() {
    for (DevBuf *b : {&plb, &pub, &prows, &pnlb, &pdepth, &ptan, &wlb, &wub, &wrows, &kinf,
                      &knm, &st, &obj, &it, &x, &cand, &dec, &bvar, &bval, &bup, &bint, &pos,
                      &depth_in, &out, &wvals, &flag, &skip2, &st2, &obj2, &it2, &x2, &acc,
                      &ws_head, &ws_st, &ws_d, &ws_binv, &r_st, &r_obj, &r_it, &fvtype, &fsq,
                      &fbil, &flptr, &flvar, &flval, &fqptr, &fqv1, &fqv2, &fqval, &fclb, &fcub,
                      &pws_head, &pws_st, &pws_ok, &gsel, &cslots, &glb, &gub, &grows, &gtan,
                      &gdepth, &ghead, &gst, &gok, &skip_a, &wo_head, &wo_st, &wo_d, &wo_binv})
      b->release();
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
  s.maxb = B;
  return MGPU_OK;
}

}  // namespace

extern "C" {

int mgpu_glob_config(mgpu_ctx *c, int order, int warm, int qt) {
  if (!c) return MGPU_ERR_ARG;
  if ((order != 0 && order != 2) || warm < 0 || warm > 1 || qt < 0 || qt > 1)
    return fail(c, MGPU_ERR_ARG, "mgpu_glob_config: order %d (0, 2), warm %d (0, 1), qt %d (0, 1)",
                order, warm, qt);
  c->glob_order = order;
  c->glob_warm = warm;
  c->glob_qt = qt;
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
  s->T = extra;
  s->S = nsq > 0 ? extra / (2 * nsq) : 0;
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
  // K2 from the parents' rows; tightenQuad_ at every node (doQT_, set by
  // Glob's presolve) or only at the first presolveNode call (QuadHandler.cpp:
  // 1215, 1241: niters <= 1)
  const int qt = (s.qt || s.tot.nodes == 0) ? 1 : 0;
  rc = mgpu_quad_fbbt_dev(c, nb, in_lb, in_ub, s.inc, qt, in_rows, 0, s.wlb.as<double>(),
                          s.wub.as<double>(), s.wrows.as<double>(), s.kinf.as<int32_t>(),
                          s.knm.as<int32_t>(), 0, nullptr, nullptr, nullptr, nullptr);
  if (rc != MGPU_OK) return rc;
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
  // the separation loop (PCBProcessor.cpp:267-280): every pass adds at least
  // one cut to a free slot, so it ends within nsq S passes; a re-solve starts
  // from the root basis (warm 0) or the node's last basis (warm 1)
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
    if (s.warm == 1)
      rc = solve(io.skip2, s.wo_head.as<int32_t>(), s.wo_st.as<int8_t>(), 0, nullptr,
                 s.st2.as<int32_t>(), s.obj2.as<double>(), s.it2.as<int32_t>(),
                 s.x2.as<double>());
    else
      rc = solve(io.skip2, s.root_ws ? s.ws_head.as<int32_t>() : nullptr,
                 s.root_ws ? s.ws_st.as<int8_t>() : nullptr, 1,
                 s.root_ws ? s.ws_binv.as<double>() : nullptr, s.st2.as<int32_t>(),
                 s.obj2.as<double>(), s.it2.as<int32_t>(), s.x2.as<double>());
    if (rc != MGPU_OK) return rc;
    HIPCHK(c, launch_glob_merge(io, c->stream));
    GlobIO again = io;
    again.only = io.flag;
    HIPCHK(c, launch_glob_decide(again, c->stream));
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
  s.tot.lps += o.lps + resolves;
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

int mgpu_glob_best(mgpu_ctx *c, double *obj, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->glob) return fail(c, MGPU_ERR_STATE, "mgpu_glob_best: mgpu_glob_init first");
  if (obj) *obj = c->glob->inc;
  if (x) std::memcpy(x, c->glob->best_x.data(), (size_t)c->glob->nv * 8);
  return MGPU_OK;
}

}  // extern "C"
