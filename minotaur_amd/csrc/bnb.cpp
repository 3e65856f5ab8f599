// Batched branch-and-bound driver: the caller of the hot
// path, MI355X-first.  It replaces the node loop of BranchAndBound::solve
// (src/base/BranchAndBound.cpp:355-526) for linear relaxations: instead of
// one node at a time through NodeIncRelaxer / PCBProcessor / OsiLPEngine, a
// round pops B open nodes from an HBM-resident stack and runs them through
// K1 (LinearHandler::presolveNode), K3 (OsiLPEngine::solve, warm-started
// from the root basis), the decision kernel (PCBProcessor::shouldPrune_ +
// IntVarHandler::isFeasible + MaxVioBrancher's choice) and the branching
// tail (IntVarHandler::getBranches), then reads back one small record.
//
// Search order: depth-first over batches (the pool is a stack and the
// preferred child is pushed last), which keeps the pool at O(depth * B)
// nodes; the incumbent prunes by bound with the reference tolerances
// (solAbs_tol / solRel_tol 1e-6, Environment.cpp:486,509-528).  Multi-GPU
// runs shard the tree after the first rounds (minotaur_amd/bnb.py) and
// exchange the incumbent with an RCCL all-reduce MIN between rounds.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "bnb_internal.h"
#include "ctx.h"

// Reference node order (mgpu_bnb_config order 2): TreeManager's "bfs"
// NodeHeap with the reference's comparator valueGreaterThan (NodeHeap.cpp:
// 24-47: bound within 1e-6, tie-break score (0 in BranchAndBound), shallower
// first, then the larger node id), kept on the host with the same
// std::push_heap / std::pop_heap, node ids assigned as TreeManager does
// (root 0, children in branch order, TreeManager.cpp:97-136, 232-249), open
// nodes pruned lazily at the top (TreeManager::getCandidate, :162-186).
struct HeapNode {
  double lb;
  int depth;
  long long id;
  int slot;
};
static bool heap_greater(const HeapNode &a, const HeapNode &b) {
  if (a.lb > b.lb + 1e-6) return true;
  if (a.lb < b.lb - 1e-6) return false;
  if (a.depth < b.depth) return false;
  if (a.depth > b.depth) return true;
  return a.id < b.id;
}

struct BnbState {
  int n = 0, cap = 0, count = 0, maxb = 0;
  int grow = 0;                // mgpu_bnb_growth of this tree
  bool root_ok = false;
  double inc = INFINITY;
  std::vector<double> best_x;
  mgpu_bnb_stats tot{};
  int order = 0, warm = 0;     // mgpu_bnb_config at init
  int qp = 0;                  // mgpu_bnb_relaxation at init: node QPs by K5
  int rel = 0;                 // mgpu_bnb_brancher at init: 1 = reliability branching
  long long calls = 0;         // ReliabilityBrancher stats_->calls (findBranches calls)
  int maxsb = 0;               // strong-branching LP capacity of the child buffers
  int hw = 0;                  // best-first: pool high-water mark
  size_t sort_bytes = 0;
  DevBuf plb, pub, pnlb, pdepth;
  DevBuf wlb, wub, inf, nm, st, obj, it, x, dec, cand, bvar, bval, bup, depth_in, pos, bsum,
      bidx, boff, bmin, bcnt, out;
  DevBuf ws_head, ws_st, ws_d, ws_binv, r_st, r_obj, r_it;
  // best-first selection
  DevBuf plive, keys, keys2, vals, vals2, sort_tmp, counts;
  // parent warm starts: per pool slot, per batch (gathered in) and out
  DevBuf pws_head, pws_st, pws_d, pws_binv, bws_head, bws_st, bws_d, bws_binv, wo_head, wo_st,
      wo_d, wo_binv;
  // reliability branching: pseudocost state [n], parent branching data per
  // pool slot, per-batch and strong-branching child workspaces
  DevBuf pc_up, pc_dn, cnt_up, cnt_dn, last, last_new, ppvar, ppval, bnlb, bpvar, bpval, rflag, rrank,
      nsb, sb_off, sb_var, sb_val, dec2, nev, ev_var, ev_side, ev_cost, rcnt, clb, cub, cnode,
      cst, cobj, cit, ev_off, cv_var, cv_side, cv_cost;
  // chained strong branching: per batch node, its chain slot, stop flag,
  // the step's LP list and count
  DevBuf ch_head, ch_st, ch_d, ch_binv, sbstop, sblist, sbcnt;
  // path warm starts (warm 2): per pool slot, per batch (gathered in) and out
  DevBuf ppk, ppath, ppst, bpk, bppath, bpst, opk, oppath, opst;
  int inherit = 0;             // longest path handed to children (<= the eta cap)
  // order 2: the host heap, free pool slots, next node id
  std::vector<HeapNode> heap;
  std::vector<HeapNode> front;  // nodes modified by the brancher: solved again next
  std::vector<int> free_slots;
  long long next_id = 0;
  bool guided = true;          // IntVarHandler guided_dive (Environment.cpp:160-163)
  DevBuf cslots;               // [2 nb] child slots
  // grow-only workspaces of the migration path (shard, export, import), so a
  // rebalance inside a timed multi-GPU run allocates nothing once warm
  DevBuf mw_slots, mw_ft, mw_tmp, mw_tlb, mw_tub, mw_tnlb, mw_tdep;
  std::vector<int> pick;       // mgpu_bnb_pick: pool slots of the picked nodes, in pick order
  std::vector<DevBuf *> bufs() {
    return {&plb, &pub, &pnlb, &pdepth, &wlb, &wub, &inf, &nm, &st, &obj, &it, &x,
                      &dec, &cand, &bvar, &bval, &bup, &depth_in, &pos, &bsum, &bidx, &boff,
                      &bmin, &bcnt, &out, &ws_head, &ws_st, &ws_d, &ws_binv, &r_st, &r_obj,
                      &r_it, &plive, &keys, &keys2, &vals, &vals2, &sort_tmp, &counts,
                      &pws_head, &pws_st, &pws_d, &pws_binv, &bws_head, &bws_st, &bws_d,
                      &bws_binv, &wo_head, &wo_st, &wo_d, &wo_binv, &pc_up, &pc_dn, &cnt_up,
                      &cnt_dn, &last, &last_new, &ppvar, &ppval, &bnlb, &bpvar, &bpval, &rflag, &rrank,
                      &nsb, &sb_off, &sb_var, &sb_val, &dec2, &nev, &ev_var, &ev_side, &ev_cost,
                      &rcnt, &clb, &cub, &cnode, &cst, &cobj, &cit, &ev_off, &cv_var, &cv_side,
                      &cv_cost, &ppk, &ppath, &ppst, &bpk, &bppath, &bpst, &opk, &oppath, &opst,
                      &cslots, &ch_head, &ch_st, &ch_d, &ch_binv, &sbstop, &sblist, &sbcnt,
                      &mw_slots, &mw_ft, &mw_tmp, &mw_tlb, &mw_tub, &mw_tnlb, &mw_tdep};
  }
  void release() {
    for (DevBuf *b : bufs()) b->release();
  }
  // takes over another state's device buffers (grow-only DevBufs): a new
  // tree on the same context reuses the pool instead of freeing and
  // allocating gigabytes again (mgpu_bnb_init)
  void adopt(BnbState &o) {
    std::vector<DevBuf *> a = bufs(), b = o.bufs();
    for (size_t i = 0; i < a.size(); ++i) {
      std::swap(a[i]->p, b[i]->p);
      std::swap(a[i]->bytes, b[i]->bytes);
    }
  }
};

void bnb_state_free(mgpu_ctx *c) {
  if (c && c->bnb) {
    c->bnb->release();
    delete c->bnb;
    c->bnb = nullptr;
  }
}

namespace {

int ensure_batch(mgpu_ctx *c, BnbState &s, int B) {
  if (B <= s.maxb) return MGPU_OK;
  const size_t n = (size_t)s.n, m = (size_t)c->lp.m;
  const size_t nblk = ((size_t)B + 255) / 256;
  HIPCHK(c, s.wlb.ensure((size_t)B * n * 8));
  HIPCHK(c, s.wub.ensure((size_t)B * n * 8));
  HIPCHK(c, s.x.ensure((size_t)B * n * 8));
  for (DevBuf *b : {&s.inf, &s.nm, &s.st, &s.it, &s.dec, &s.bvar, &s.depth_in, &s.pos})
    HIPCHK(c, b->ensure((size_t)B * 4));
  for (DevBuf *b : {&s.obj, &s.cand, &s.bval}) HIPCHK(c, b->ensure((size_t)B * 8));
  HIPCHK(c, s.bup.ensure((size_t)B));
  for (DevBuf *b : {&s.bsum, &s.bidx, &s.boff}) HIPCHK(c, b->ensure(nblk * 4));
  HIPCHK(c, s.bmin.ensure(nblk * 8));
  HIPCHK(c, s.bcnt.ensure(nblk * 8 * 4));
  HIPCHK(c, s.out.ensure(sizeof(BnbOut)));
  if (s.rel) {
    for (DevBuf *b : {&s.bpvar, &s.rflag, &s.rrank, &s.nsb, &s.sb_off, &s.dec2, &s.nev,
                      &s.ev_off})
      HIPCHK(c, b->ensure((size_t)B * 4));
    HIPCHK(c, s.cv_var.ensure((size_t)B * kRelEvents * 4));
    HIPCHK(c, s.cv_side.ensure((size_t)B * kRelEvents));
    HIPCHK(c, s.cv_cost.ensure((size_t)B * kRelEvents * 8));
    for (DevBuf *b : {&s.bnlb, &s.bpval}) HIPCHK(c, b->ensure((size_t)B * 8));
    HIPCHK(c, s.sb_var.ensure((size_t)B * kRelMaxCands * 4));
    HIPCHK(c, s.sb_val.ensure((size_t)B * kRelMaxCands * 8));
    HIPCHK(c, s.ev_var.ensure((size_t)B * kRelEvents * 4));
    HIPCHK(c, s.ev_side.ensure((size_t)B * kRelEvents));
    HIPCHK(c, s.ev_cost.ensure((size_t)B * kRelEvents * 8));
    const size_t N = n + m;
    HIPCHK(c, s.ch_head.ensure((size_t)B * m * 4 + 4));
    HIPCHK(c, s.ch_st.ensure((size_t)B * N + 4));
    HIPCHK(c, s.ch_d.ensure((size_t)B * N * 8));
    HIPCHK(c, s.ch_binv.ensure((size_t)B * m * m * 8 + 8));
    HIPCHK(c, s.sbstop.ensure((size_t)B + 4));
    HIPCHK(c, s.sblist.ensure((size_t)B * 4));
    HIPCHK(c, s.sbcnt.ensure(16));
  }
  if (s.warm == 1 || s.rel) {  // reliability branching needs each node's optimal basis
    const size_t N = n + m;
    HIPCHK(c, s.wo_head.ensure((size_t)B * m * 4 + 4));
    HIPCHK(c, s.wo_st.ensure((size_t)B * N + 4));
    HIPCHK(c, s.wo_d.ensure((size_t)B * N * 8));
    HIPCHK(c, s.wo_binv.ensure((size_t)B * m * m * 8 + 8));
  }
  if (s.warm == 2) {
    const size_t N = n + m;
    for (DevBuf *b : {&s.bpk, &s.opk}) HIPCHK(c, b->ensure((size_t)B * 4));
    for (DevBuf *b : {&s.bppath, &s.oppath}) HIPCHK(c, b->ensure((size_t)B * kPathMax * 4));
    for (DevBuf *b : {&s.bpst, &s.opst}) HIPCHK(c, b->ensure((size_t)B * N + 16));
  }
  if (s.warm == 1) {
    const size_t N = n + m;
    HIPCHK(c, s.bws_head.ensure((size_t)B * m * 4 + 4));
    HIPCHK(c, s.bws_st.ensure((size_t)B * N + 4));
    HIPCHK(c, s.bws_d.ensure((size_t)B * N * 8));
    HIPCHK(c, s.bws_binv.ensure((size_t)B * m * m * 8 + 8));
    HIPCHK(c, s.wo_head.ensure((size_t)B * m * 4 + 4));
    HIPCHK(c, s.wo_st.ensure((size_t)B * N + 4));
    HIPCHK(c, s.wo_d.ensure((size_t)B * N * 8));
    HIPCHK(c, s.wo_binv.ensure((size_t)B * m * m * 8 + 8));
  }
  s.maxb = B;
  return MGPU_OK;
}

// Reliability branching for the round's nodes (bnb_rel.hip): candidates
// and strong-branching lists, the strong-branching LPs in one K3/K3L batch
// (each from its node's optimal basis, iteration limit 25), the choice, and
// the pseudocost update.  Leaves the final decisions in s.dec2 and the
// choice / bound change in s.bvar / s.bval / s.bup.
int rel_round(mgpu_ctx *c, BnbState &s, int nb, int base, bool bfs) {
  const int n = s.n, m = c->lp.m, N = n + m;
  HIPCHK(c, launch_rel_gather(nb, base, bfs ? s.vals2.as<uint32_t>() : nullptr,
                              s.pnlb.as<double>(), s.ppvar.as<int32_t>(), s.ppval.as<double>(),
                              s.bnlb.as<double>(), s.bpvar.as<int32_t>(), s.bpval.as<double>(),
                              c->stream));
  // after the counters: [0] branching nodes, [1] strong-branching candidates,
  // [2] observations, [3] the largest candidate count of a node
  int32_t *tot = reinterpret_cast<int32_t *>(s.rcnt.as<char>() + 32);
  HIPCHK(c, hipMemsetAsync(s.rcnt.p, 0, 48, c->stream));
  RelIO r{};
  r.nb = nb;
  r.n = n;
  r.vtype = c->lp.vtype;
  r.decision = s.dec.as<int32_t>();
  r.x = s.x.as<double>();
  r.obj = s.obj.as<double>();
  r.nlb = s.bnlb.as<double>();
  // node depths: gathered for best-first; the stack's popped slice in place
  r.depth = bfs ? s.depth_in.as<int32_t>() : s.pdepth.as<int32_t>() + base;
  r.pvar = s.bpvar.as<int32_t>();
  r.pval = s.bpval.as<double>();
  r.pc_up = s.pc_up.as<double>();
  r.pc_dn = s.pc_dn.as<double>();
  r.cnt_up = s.cnt_up.as<int32_t>();
  r.cnt_dn = s.cnt_dn.as<int32_t>();
  r.last = s.last.as<int32_t>();
  r.last_new = s.last_new.as<int32_t>();
  HIPCHK(c, hipMemsetAsync(s.last_new.p, 0xFF, (size_t)n * 4, c->stream));
  r.calls0 = s.calls;
  r.rank = s.rrank.as<int32_t>();
  r.cutoff = s.inc;
  r.nsb = s.nsb.as<int32_t>();
  r.sb_var = s.sb_var.as<int32_t>();
  r.sb_val = s.sb_val.as<double>();
  r.sb_off = s.sb_off.as<int32_t>();
  r.dec_out = s.dec2.as<int32_t>();
  r.bvar = s.bvar.as<int32_t>();
  r.bval = s.bval.as<double>();
  r.bup = s.bup.as<int8_t>();
  r.nev = s.nev.as<int32_t>();
  r.ev_var = s.ev_var.as<int32_t>();
  r.ev_side = s.ev_side.as<int8_t>();
  r.ev_cost = s.ev_cost.as<double>();
  r.ev_off = s.ev_off.as<int32_t>();
  r.ev_total = tot + 2;
  r.cv_var = s.cv_var.as<int32_t>();
  r.cv_side = s.cv_side.as<int8_t>();
  r.cv_cost = s.cv_cost.as<double>();
  r.counters = s.rcnt.as<unsigned long long>();
  r.nsb_max = tot + 3;
  HIPCHK(c, launch_rel_rank(r, s.rflag.as<int32_t>(), s.rrank.as<int32_t>(), tot, c->stream));
  HIPCHK(c, launch_rel_prepare(r, s.sb_off.as<int32_t>(), tot + 1, c->stream));
  int32_t h_tot[4] = {0, 0, 0, 0};
  HIPCHK(c, hipMemcpyAsync(h_tot, tot, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int nchild = 2 * h_tot[1];
  if (nchild > 0) {
    if (nchild > s.maxsb) {
      HIPCHK(c, s.clb.ensure((size_t)nchild * n * 8));
      HIPCHK(c, s.cub.ensure((size_t)nchild * n * 8));
      for (DevBuf *b : {&s.cnode, &s.cst, &s.cit}) HIPCHK(c, b->ensure((size_t)nchild * 4));
      HIPCHK(c, s.cobj.ensure((size_t)nchild * 8));
      s.maxsb = nchild;
    }
    HIPCHK(c, launch_rel_children(r, s.wlb.as<double>(), s.wub.as<double>(), s.clb.as<double>(),
                                  s.cub.as<double>(), s.cnode.as<int32_t>(), c->stream));
    r.c_status = s.cst.as<int32_t>();
    r.c_obj = s.cobj.as<double>();
    r.c_iters = s.cit.as<int32_t>();
    // the strong-branching LPs, chained per node as the reference's engine
    // runs them: every LP from the node's chain slot (its optimal basis, then
    // whatever basis the last optimal / iteration-limited LP left) and back
    // into it; ReliabilityBrancher's iteration cap; after each candidate's
    // pair the nodes with a verdict stop (the next step's list kernel takes
    // the verdict before it lists the step's LPs)
    const LpWarm node_ws{s.wo_head.as<int32_t>(), s.wo_st.as<int8_t>(), s.wo_d.as<double>(),
                         s.wo_binv.as<double>(), m, N, N, (long)m * m};
    HIPCHK(c, launch_rel_chain_init(r, node_ws, s.ch_head.as<int32_t>(), s.ch_st.as<int8_t>(),
                                    s.ch_d.as<double>(), s.ch_binv.as<double>(),
                                    s.sbstop.as<uint8_t>(), m, c->stream));
    LpIO io{};
    io.batch = nb;                    // at most one LP per node and step
    io.lb = s.clb.as<double>();
    io.ub = s.cub.as<double>();
    io.box_stride = n;
    io.ws = LpWarm{s.ch_head.as<int32_t>(), s.ch_st.as<int8_t>(), s.ch_d.as<double>(),
                   s.ch_binv.as<double>(), m, N, N, (long)m * m};
    io.ws_index = s.cnode.as<int32_t>();
    io.wo_head = s.ch_head.as<int32_t>();
    io.wo_st = s.ch_st.as<int8_t>();
    io.wo_d = s.ch_d.as<double>();
    io.wo_binv = s.ch_binv.as<double>();
    io.wo_index = s.cnode.as<int32_t>();
    io.node_list = s.sblist.as<int32_t>();
    io.list_lo = 0;
    io.list_hi = 0x7fffffff;
    io.iter_limit = kRelIterLimit;
    io.status = s.cst.as<int32_t>();
    io.obj = s.cobj.as<double>();
    io.iters = s.cit.as<int32_t>();
    if (c->sb_chain && lp_chain_ok(c)) {
      // every node's whole chain in ONE K3 launch, one wave per node: no
      // launch, matrix staging or list kernel per step, and a node no longer
      // waits for the slowest LP of each step (LpIO::chain_*)
      io.batch = nb;
      io.node_list = nullptr;
      io.chain_off = r.sb_off;
      io.chain_n = r.nsb;
      io.chain_nobj = r.obj;
      io.chain_cutoff = r.cutoff;
      const int lrc = launch_lp_nodes(c, io);
      if (lrc != MGPU_OK) return lrc;
      HIPCHK(c, launch_rel_decide(r, c->stream));
      s.calls += h_tot[0];
      return MGPU_OK;
    }
    // one list counter per chain step, zeroed together (one fill per round
    // instead of one per step: the rounds of a reliability tree are short)
    const int nsteps = 2 * h_tot[3];
    HIPCHK(c, s.sbcnt.ensure((size_t)(nsteps > 4 ? nsteps : 4) * 4));
    if (nsteps > 0) HIPCHK(c, hipMemsetAsync(s.sbcnt.p, 0, (size_t)nsteps * 4, c->stream));
    for (int step = 0; step < nsteps; ++step) {
      io.node_count = s.sbcnt.as<int32_t>() + step;
      HIPCHK(c, launch_rel_chain_list(r, step, s.sbstop.as<uint8_t>(), s.sblist.as<int32_t>(),
                                      s.sbcnt.as<int32_t>() + step, c->stream));
      const int lrc = launch_lp_nodes(c, io);
      if (lrc != MGPU_OK) return lrc;
    }
  }
  HIPCHK(c, launch_rel_decide(r, c->stream));
  s.calls += h_tot[0];
  return MGPU_OK;
}

// Reference-heap mode, after the round's scans: the host reads each node's
// decision, bound, depth and branching choice, assigns pool slots to the
// children (the round's own slots first, then older free slots, then new
// ones), launches the children writer and pushes the children onto the heap
// in the reference's branch order with the next node ids: the preferred
// direction first, or — guided dive, with an incumbent — down first when the
// incumbent's value of the variable is below the node's (IntVarHandler::
// getBranches, IntVarHandler.cpp:125-175).
int heap_children(mgpu_ctx *c, BnbState &s, BnbIO &io, int nb, const std::vector<uint32_t> &sel,
                  const std::vector<HeapNode> &popped) {
  std::vector<int32_t> dec(nb), bvar(nb), dep(nb);
  std::vector<double> obj(nb), bval(nb);
  std::vector<int8_t> bup(nb);
  HIPCHK(c, hipMemcpyAsync(dec.data(), io.decision, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(bvar.data(), io.bvar, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(dep.data(), io.depth_in, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(obj.data(), io.obj, (size_t)nb * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(bval.data(), io.bval, (size_t)nb * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(bup.data(), io.bup, (size_t)nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // free slots in the order children take them
  std::vector<int> pool(sel.begin(), sel.end());
  for (auto it = s.free_slots.rbegin(); it != s.free_slots.rend(); ++it) pool.push_back(*it);
  s.free_slots.clear();
  size_t next = 0;
  auto take = [&]() -> int { return next < pool.size() ? pool[next++] : s.hw++; };
  std::vector<int32_t> cs;
  struct Kid {
    double lb;
    int depth, slot, down;
  };
  std::vector<Kid> kids;
  for (int i = 0; i < nb; ++i) {
    if (dec[i] != 0 && dec[i] != 5) continue;
    if (dec[i] == 5) {
      // ModifiedByBrancher: the same node (its id) is solved again right
      // away with the bound change (PCBProcessor.cpp:295-310), ahead of
      // the heap
      const int sl = take();
      cs.push_back(sl);
      s.front.push_back(HeapNode{obj[i], dep[i], popped[i].id, sl});
      continue;
    }
    const int s_pref = take(), s_other = take();   // child index p (preferred), p + 1
    cs.push_back(s_pref);
    cs.push_back(s_other);
    const bool pref_up = bup[i] != 0;
    bool down_first = !pref_up;
    if (s.guided && std::isfinite(s.inc) && !std::isnan(s.best_x[bvar[i]]))
      down_first = s.best_x[bvar[i]] < bval[i];
    const int s_down = pref_up ? s_other : s_pref, s_up = pref_up ? s_pref : s_other;
    kids.push_back({obj[i], dep[i] + 1, down_first ? s_down : s_up, 0});
    kids.push_back({obj[i], dep[i] + 1, down_first ? s_up : s_down, 0});
  }
  for (size_t k = next; k < pool.size(); ++k) s.free_slots.push_back(pool[k]);
  if (!cs.empty()) {
    HIPCHK(c, s.cslots.ensure(cs.size() * 4));
    HIPCHK(c, hipMemcpyAsync(s.cslots.p, cs.data(), cs.size() * 4, hipMemcpyHostToDevice,
                             c->stream));
    io.child_slots = s.cslots.as<int32_t>();
    HIPCHK(c, launch_bnb_children(io, s.n, c->stream));
  }
  for (const Kid &k : kids) {
    s.heap.push_back(HeapNode{k.lb, k.depth, s.next_id++, k.slot});
    std::push_heap(s.heap.begin(), s.heap.end(), heap_greater);
  }
  s.count = (int)(s.heap.size() + s.front.size());
  return MGPU_OK;
}

}  // namespace

extern "C" {

int mgpu_bnb_config(mgpu_ctx *c, int order, int warm) {
  if (!c) return MGPU_ERR_ARG;
  if (order < 0 || order > 2 || warm < 0 || warm > 2)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_config: order 0/1/2, warm 0/1/2");
  c->bnb_order = order;
  c->bnb_warm = warm;
  return MGPU_OK;
}

int mgpu_bnb_guided_dive(mgpu_ctx *c, int on) {
  if (!c) return MGPU_ERR_ARG;
  c->bnb_guided = on ? 1 : 0;
  return MGPU_OK;
}

int mgpu_bnb_relaxation(mgpu_ctx *c, int kind) {
  if (!c) return MGPU_ERR_ARG;
  if (kind < 0 || kind > 1)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_relaxation: 0 (LP) or 1 (the loaded QP)");
  c->bnb_relax = kind;
  return MGPU_OK;
}

int mgpu_bnb_growth(mgpu_ctx *c, int div) {
  if (!c) return MGPU_ERR_ARG;
  if (div < 0) return fail(c, MGPU_ERR_ARG, "mgpu_bnb_growth: div must be >= 0");
  c->bnb_grow = div;
  return MGPU_OK;
}

int mgpu_bnb_brancher(mgpu_ctx *c, int kind) {
  if (!c) return MGPU_ERR_ARG;
  if (kind < 0 || kind > 1)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_brancher: 0 (MaxVio) or 1 (reliability)");
  c->bnb_brancher = kind;
  return MGPU_OK;
}

int mgpu_bnb_init(mgpu_ctx *c, int capacity, const double *root_lb, const double *root_ub,
                  double incumbent) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_bnb_init: no problem loaded");
  if (capacity < 2 || !root_lb || !root_ub)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_init: bad argument");
  HIPCHK(c, hipSetDevice(c->device));
  BnbState *s = new BnbState();
  if (c->bnb) {
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the old tree's kernels are done with them
    s->adopt(*c->bnb);
  }
  bnb_state_free(c);
  c->bnb = s;
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  s->n = n;
  s->cap = capacity;
  s->inc = incumbent;
  s->order = c->bnb_order;
  s->warm = c->bnb_warm;
  s->rel = c->bnb_brancher;
  s->qp = c->bnb_relax;
  s->grow = c->bnb_grow;
  s->tot.incumbent = incumbent;
  if (s->qp && (!c->qp || s->warm != 0 || s->rel))
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_init: QP relaxations need mgpu_load_qp (same columns as "
                "the loaded rows), root warm starts (warm 0) and MaxVio branching");
  if (s->warm == 2) {
    // path warm starts run on K3P's eta file: the tree hands children paths
    // of at most min(kPathInherit, eta cap) pivots
    const int kcap = mgpu_lp_pfi_cap(c);
    if (s->rel || m > kLpMaxM || kcap <= 0 || kcap > kPfiBig)
      return fail(c, MGPU_ERR_ARG, "mgpu_bnb_init: path warm starts (warm 2) need MaxVio "
                  "branching and K3P (m <= 64, eta cap 1..%d)", kPfiBig);
    // MGPU_PATH_INHERIT (tuning experiments only; the CPU restatement
    // assumes the default) overrides the longest inherited path
    int inh = kPathInherit;
    if (const char *e = std::getenv("MGPU_PATH_INHERIT")) inh = std::atoi(e);
    if (inh < 0) inh = 0;
    if (inh > kPathMax) inh = kPathMax;   // the path slots
    s->inherit = kcap < inh ? kcap : inh;
  }
  if (s->rel) {
    if (m > kLpMaxM && !(lp_large_lds_bytes(n, m) <= (size_t)kLargeLdsMax))
      return fail(c, MGPU_ERR_ARG, "mgpu_bnb_init: reliability branching needs K3 or K3L");
    // ReliabilityBrancher::initialize (:384-398): pseudocosts 0, counts 0,
    // lastStrBranched_ 20000
    for (DevBuf *b : {&s->pc_up, &s->pc_dn}) HIPCHK(c, b->ensure((size_t)n * 8));
    for (DevBuf *b : {&s->cnt_up, &s->cnt_dn, &s->last, &s->last_new})
      HIPCHK(c, b->ensure((size_t)n * 4));
    for (DevBuf *b : {&s->pc_up, &s->pc_dn, &s->cnt_up, &s->cnt_dn})
      HIPCHK(c, hipMemsetAsync(b->p, 0, b->bytes, c->stream));
    std::vector<int32_t> l20k(n, 20000);
    HIPCHK(c, hipMemcpyAsync(s->last.p, l20k.data(), (size_t)n * 4, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, s->ppvar.ensure((size_t)capacity * 4));
    HIPCHK(c, s->ppval.ensure((size_t)capacity * 8));
    HIPCHK(c, hipMemsetAsync(s->ppvar.p, 0xFF, (size_t)capacity * 4, c->stream));  // -1: root
    HIPCHK(c, s->rcnt.ensure(64));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  HIPCHK(c, s->plb.ensure((size_t)capacity * n * 8));
  HIPCHK(c, s->pub.ensure((size_t)capacity * n * 8));
  HIPCHK(c, s->pnlb.ensure((size_t)capacity * 8));
  HIPCHK(c, s->pdepth.ensure((size_t)capacity * 4));
  HIPCHK(c, s->ws_head.ensure((size_t)m * 4 + 4));
  HIPCHK(c, s->ws_st.ensure((size_t)N + 4));
  HIPCHK(c, s->ws_d.ensure((size_t)N * 8));
  HIPCHK(c, s->ws_binv.ensure((size_t)m * m * 8 + 8));
  HIPCHK(c, s->r_st.ensure(4));
  HIPCHK(c, s->r_obj.ensure(8));
  HIPCHK(c, s->r_it.ensure(4));
  // root: its box is the first open node; its LP optimum is the shared warm
  // start of every node LP (NodeIncRelaxer loads the parent's basis,
  // NodeIncRelaxer.cpp:146-150; the root's is the one every node shares)
  HIPCHK(c, hipMemcpyAsync(s->plb.p, root_lb, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(s->pub.p, root_ub, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
  const double ninf = -INFINITY;
  const int32_t zero = 0;
  HIPCHK(c, hipMemcpyAsync(s->pnlb.p, &ninf, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(s->pdepth.p, &zero, 4, hipMemcpyHostToDevice, c->stream));
  int32_t rst = -1;   // QP relaxations: no LP basis to share
  if (!s->qp) {
    int rc = mgpu_lp_solve_dev(c, 1, s->plb.as<double>(), s->pub.as<double>(), nullptr, nullptr,
                               nullptr, nullptr, nullptr, 1, 0, s->r_st.as<int32_t>(),
                               s->r_obj.as<double>(), s->r_it.as<int32_t>(), nullptr,
                               s->ws_head.as<int32_t>(), s->ws_st.as<int8_t>(),
                               s->ws_d.as<double>(), s->ws_binv.as<double>());
    if (rc != MGPU_OK) return rc;
    HIPCHK(c, hipMemcpyAsync(&rst, s->r_st.p, 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  s->root_ok = rst == 0;
  s->count = 1;
  s->best_x.assign(n, NAN);
  if (s->order == 2) {
    // reference heap: the root is node 0 in slot 0; slots and live flags
    // as in best-first (the gather clears a taken slot's flag)
    HIPCHK(c, s->plive.ensure((size_t)capacity));
    HIPCHK(c, hipMemsetAsync(s->plive.p, 0, (size_t)capacity, c->stream));
    HIPCHK(c, s->vals2.ensure((size_t)capacity * 4));
    s->heap.push_back(HeapNode{-INFINITY, 0, 0, 0});
    s->next_id = 1;
    s->hw = 1;
    s->guided = c->bnb_guided;
  }
  if (s->order == 1) {
    // best-first pool: slot array with live flags, sort keys and scratch
    HIPCHK(c, s->plive.ensure((size_t)capacity));
    HIPCHK(c, hipMemsetAsync(s->plive.p, 0, (size_t)capacity, c->stream));
    const uint8_t one = 1;
    HIPCHK(c, hipMemcpyAsync(s->plive.p, &one, 1, hipMemcpyHostToDevice, c->stream));
    for (DevBuf *b : {&s->keys, &s->keys2}) HIPCHK(c, b->ensure((size_t)capacity * 8));
    for (DevBuf *b : {&s->vals, &s->vals2}) HIPCHK(c, b->ensure((size_t)capacity * 4));
    HIPCHK(c, s->counts.ensure(16));
    size_t tb = 0;
    HIPCHK(c, bnb_sort_pairs(nullptr, tb, s->keys.as<uint64_t>(), s->keys2.as<uint64_t>(),
                             s->vals.as<uint32_t>(), s->vals2.as<uint32_t>(), capacity,
                             c->stream));
    HIPCHK(c, s->sort_tmp.ensure(tb + 16));
    s->sort_bytes = tb;
    s->hw = 1;
  }
  if (s->warm == 2) {
    if (!s->root_ok)
      return fail(c, MGPU_ERR_STATE, "mgpu_bnb_init: path warm starts need an optimal root");
    // per pool slot: path length (0: the root basis), pivots, column statuses
    HIPCHK(c, s->ppk.ensure((size_t)capacity * 4));
    HIPCHK(c, s->ppath.ensure((size_t)capacity * kPathMax * 4));
    HIPCHK(c, s->ppst.ensure((size_t)capacity * N + 16));
    HIPCHK(c, hipMemsetAsync(s->ppk.p, 0, (size_t)capacity * 4, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (s->warm == 1) {
    if (!s->root_ok)
      return fail(c, MGPU_ERR_STATE, "mgpu_bnb_init: parent warm starts need an optimal root");
    // every pool slot keeps its node's warm start (the parent's optimal basis)
    HIPCHK(c, s->pws_head.ensure((size_t)capacity * m * 4 + 4));
    HIPCHK(c, s->pws_st.ensure((size_t)capacity * N + 4));
    HIPCHK(c, s->pws_d.ensure((size_t)capacity * N * 8));
    HIPCHK(c, s->pws_binv.ensure((size_t)capacity * m * m * 8 + 8));
    HIPCHK(c, hipMemcpyAsync(s->pws_head.p, s->ws_head.p, (size_t)m * 4, hipMemcpyDeviceToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(s->pws_st.p, s->ws_st.p, (size_t)N, hipMemcpyDeviceToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(s->pws_d.p, s->ws_d.p, (size_t)N * 8, hipMemcpyDeviceToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(s->pws_binv.p, s->ws_binv.p, (size_t)m * m * 8,
                             hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return MGPU_OK;
}

int mgpu_bnb_round(mgpu_ctx *c, int batch, double incumbent, mgpu_bnb_stats *stats) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->bnb) return fail(c, MGPU_ERR_STATE, "mgpu_bnb_round: mgpu_bnb_init first");
  if (batch <= 0) return fail(c, MGPU_ERR_ARG, "mgpu_bnb_round: batch must be > 0");
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  if (incumbent < s.inc) s.inc = incumbent;
  if (s.grow > 0) {   // mgpu_bnb_growth: at most 1/grow of the nodes so far
    const long long g = s.tot.nodes / s.grow;
    if ((long long)batch > (g > 1 ? g : 1)) batch = (int)(g > 1 ? g : 1);
  }
  const int n = s.n, m = c->lp.m, N = n + m;
  const bool bfs = s.order >= 1;      // the round's nodes are gathered from pool slots
  const bool heap = s.order == 2;
  const bool root_round = heap && s.tot.rounds == 0;
  int nb, base = 0, live = 0, holes = 0;
  std::vector<uint32_t> sel;
  std::vector<HeapNode> popped;
  if (heap) {
    // nodes modified by the brancher first (their process() call goes on),
    // then TreeManager::getCandidate: the heap top, pruned lazily by the
    // incumbent (TreeManager::shouldPrune_, :403-413), then removed
    size_t nf = 0;
    for (; nf < s.front.size() && (int)sel.size() < batch; ++nf) {
      sel.push_back((uint32_t)s.front[nf].slot);
      popped.push_back(s.front[nf]);
    }
    s.front.erase(s.front.begin(), s.front.begin() + nf);
    while ((int)sel.size() < batch && !s.heap.empty()) {
      const HeapNode top = s.heap.front();
      std::pop_heap(s.heap.begin(), s.heap.end(), heap_greater);
      s.heap.pop_back();
      if (top.lb > s.inc - 1e-6 || std::fabs(s.inc - top.lb) / (std::fabs(s.inc) + 1e-6) * 100.0 < 1e-6) {
        s.free_slots.push_back(top.slot);
        s.tot.pruned += 1;
        continue;
      }
      sel.push_back((uint32_t)top.slot);
      popped.push_back(top);
    }
    nb = (int)sel.size();
    live = (int)(s.heap.size() + s.front.size()) + nb;
    s.count = live;
    if (nb <= 0) {
      s.tot.open = 0;
      if (stats) *stats = s.tot;
      return MGPU_OK;
    }
    const long need = 2L * nb - nb - (long)s.free_slots.size();
    if (s.hw + (need > 0 ? need : 0) > s.cap)
      return fail(c, MGPU_ERR_NOMEM, "mgpu_bnb_round: node pool full (%d slots)", s.cap);
    HIPCHK(c, hipMemcpyAsync(s.vals2.p, sel.data(), (size_t)nb * 4, hipMemcpyHostToDevice,
                             c->stream));
  } else if (!bfs) {
    nb = batch < s.count ? batch : s.count;
    if (s.count + nb > s.cap) nb = s.cap - s.count;  // children must fit: base + 2 nb <= cap
    if (nb <= 0) {
      if (s.count > 0) return fail(c, MGPU_ERR_NOMEM, "mgpu_bnb_round: node pool full");
      if (stats) *stats = s.tot;
      return MGPU_OK;
    }
    base = s.count - nb;
  } else {
    // TreeManager::getCandidate's pruning by the incumbent, then the keys of
    // the live nodes; one small read-back gives the live count
    HIPCHK(c, hipMemsetAsync(s.counts.p, 0, 8, c->stream));
    HIPCHK(c, launch_bnb_keys(s.pnlb.as<double>(), s.plive.as<uint8_t>(), s.hw, s.inc, s.inc,
                              s.keys.as<uint64_t>(), s.vals.as<uint32_t>(),
                              s.counts.as<int32_t>(), c->stream));
    int32_t cnt[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(cnt, s.counts.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    live = cnt[0];
    s.tot.pruned += cnt[1];
    s.count = live;
    holes = s.hw - live;
    nb = batch < live ? batch : live;
    if (nb <= 0) {
      s.tot.open = 0;
      if (stats) *stats = s.tot;
      return MGPU_OK;
    }
    const long grow = 2L * nb - nb - holes;  // new slots the children may need
    if (s.hw + (grow > 0 ? grow : 0) > s.cap)
      return fail(c, MGPU_ERR_NOMEM, "mgpu_bnb_round: node pool full (%d slots)", s.cap);
  }
  int rc = ensure_batch(c, s, nb);
  if (rc != MGPU_OK) return rc;
  const double *lb, *ub;
  const int32_t *w_head = nullptr;
  const int8_t *w_st = nullptr;
  const double *w_d = nullptr, *w_binv = nullptr;
  if (!bfs) {
    lb = s.plb.as<double>() + (size_t)base * n;
    ub = s.pub.as<double>() + (size_t)base * n;
    if (s.warm == 1) {  // the popped nodes are contiguous: their bases are read in place
      w_head = s.pws_head.as<int32_t>() + (size_t)base * m;
      w_st = s.pws_st.as<int8_t>() + (size_t)base * N;
      w_d = s.pws_d.as<double>() + (size_t)base * N;
      w_binv = s.pws_binv.as<double>() + (size_t)base * m * m;
    }
  } else {
    size_t tb = s.sort_bytes;
    if (!heap)
      HIPCHK(c, bnb_sort_pairs(s.sort_tmp.p, tb, s.keys.as<uint64_t>(), s.keys2.as<uint64_t>(),
                               s.vals.as<uint32_t>(), s.vals2.as<uint32_t>(), s.hw, c->stream));
    BnbSelIO g{};
    g.nb = nb;
    g.n = n;
    g.m = m;
    g.N = N;
    g.slots = s.vals2.as<uint32_t>();
    g.plb = s.plb.as<double>();
    g.pub = s.pub.as<double>();
    g.pdepth = s.pdepth.as<int32_t>();
    g.plive = s.plive.as<uint8_t>();
    g.wlb = s.wlb.as<double>();
    g.wub = s.wub.as<double>();
    g.depth_in = s.depth_in.as<int32_t>();
    if (s.warm == 2) {
      g.pk = s.ppk.as<int32_t>();
      g.ppath = s.ppath.as<uint32_t>();
      g.pst = s.ppst.as<int8_t>();
      g.bpk = s.bpk.as<int32_t>();
      g.bppath = s.bppath.as<uint32_t>();
      g.bpst = s.bpst.as<int8_t>();
    }
    if (s.warm == 1) {
      g.ws_head = s.pws_head.as<int32_t>();
      g.ws_st = s.pws_st.as<int8_t>();
      g.ws_d = s.pws_d.as<double>();
      g.ws_binv = s.pws_binv.as<double>();
      g.bws_head = s.bws_head.as<int32_t>();
      g.bws_st = s.bws_st.as<int8_t>();
      g.bws_d = s.bws_d.as<double>();
      g.bws_binv = s.bws_binv.as<double>();
      w_head = g.bws_head;
      w_st = g.bws_st;
      w_d = g.bws_d;
      w_binv = g.bws_binv;
    }
    HIPCHK(c, launch_bnb_gather(g, c->stream));
    lb = s.wlb.as<double>();
    ub = s.wub.as<double>();
  }
  // LinearHandler::varBndsFromObj_ propagates a linear objective only: a
  // QP's node FBBT runs without the incumbent
  rc = mgpu_fbbt_dev(c, nb, lb, ub, s.qp ? INFINITY : s.inc, s.wlb.as<double>(),
                     s.wub.as<double>(), s.inf.as<int32_t>(), s.nm.as<int32_t>(), 0, nullptr,
                     nullptr, nullptr);
  if (rc != MGPU_OK) return rc;
  // the node decision (shouldPrune_ + isFeasible + MaxVio), fused into K3P's
  // epilogue when the round's LPs run the product form (no x read back)
  DecideIO d{};
  d.batch = nb;
  d.fbbt_infeas = s.inf.as<int32_t>();
  d.status = s.st.as<int32_t>();
  d.obj = s.obj.as<double>();
  d.x = s.x.as<double>();
  d.incumbent = s.inc;
  d.abs_tol = 1e-6;
  d.rel_tol = 1e-6;
  d.cutoff = INFINITY;
  d.int_tol = 1e-6;
  d.decision = s.dec.as<int32_t>();
  d.cand_obj = s.cand.as<double>();
  d.bvar = s.bvar.as<int32_t>();
  d.bval = s.bval.as<double>();
  d.bup = s.bup.as<int8_t>();
  c->lp_decided = false;
  c->pfi_decide = (!s.qp && !s.rel && (s.warm == 0 || s.warm == 2)) ? &d : nullptr;
  if (s.qp) {
    // the node's QP relaxation (QPDRelaxer -> BqpdEngine::solve,
    // examples/QPDRelaxer.cpp:56-126): K5 on the FBBT-tightened boxes, the
    // FBBT-infeasible nodes skipped
    rc = qp_solve_nodes(c, nb, s.wlb.as<double>(), s.wub.as<double>(), s.inf.as<int32_t>(), 0,
                        s.st.as<int32_t>(), s.obj.as<double>(), s.it.as<int32_t>(),
                        s.x.as<double>());
  } else if (s.warm == 2) {
    // each node from its parent's optimal basis (NodeIncRelaxer.cpp:146-150)
    // kept as its pivot path from the root basis; its own final path comes
    // back for its children
    const int32_t *pk = bfs ? s.bpk.as<int32_t>() : s.ppk.as<int32_t>() + base;
    const uint32_t *pp = bfs ? s.bppath.as<uint32_t>()
                             : s.ppath.as<uint32_t>() + (size_t)base * kPathMax;
    const int8_t *ps = bfs ? s.bpst.as<int8_t>() : s.ppst.as<int8_t>() + (size_t)base * N;
    rc = mgpu_lp_solve_path_dev(c, nb, s.wlb.as<double>(), s.wub.as<double>(),
                                s.inf.as<int32_t>(), s.ws_head.as<int32_t>(),
                                s.ws_st.as<int8_t>(), s.ws_d.as<double>(),
                                s.ws_binv.as<double>(), pk, pp, ps, s.inherit, 0,
                                s.st.as<int32_t>(), s.obj.as<double>(), s.it.as<int32_t>(),
                                s.x.as<double>(), s.opk.as<int32_t>(), s.oppath.as<uint32_t>(),
                                s.opst.as<int8_t>());
  } else if (s.warm) {
    // each node from its parent's optimal basis (NodeIncRelaxer.cpp:146-150);
    // its own optimal basis comes back for its children.  The reference's
    // root has no warm start: its LP runs from the slack basis after the
    // root's presolve (BranchAndBound::processRoot_), as in heap mode here.
    rc = mgpu_lp_solve_dev(c, nb, s.wlb.as<double>(), s.wub.as<double>(), s.inf.as<int32_t>(),
                           root_round ? nullptr : w_head, root_round ? nullptr : w_st,
                           root_round ? nullptr : w_d, root_round ? nullptr : w_binv, 0, 0,
                           s.st.as<int32_t>(),
                           s.obj.as<double>(), s.it.as<int32_t>(), s.x.as<double>(),
                           s.wo_head.as<int32_t>(), s.wo_st.as<int8_t>(), s.wo_d.as<double>(),
                           s.wo_binv.as<double>());
  } else {
    // reliability branching strong-branches from each node's optimal basis:
    // the node LPs give it back (dense K3 instead of K3P)
    rc = mgpu_lp_solve_dev(c, nb, s.wlb.as<double>(), s.wub.as<double>(), s.inf.as<int32_t>(),
                           s.root_ok ? s.ws_head.as<int32_t>() : nullptr,
                           s.root_ok ? s.ws_st.as<int8_t>() : nullptr,
                           s.root_ok ? s.ws_d.as<double>() : nullptr,
                           s.root_ok ? s.ws_binv.as<double>() : nullptr, 1, 0,
                           s.st.as<int32_t>(), s.obj.as<double>(), s.it.as<int32_t>(),
                           s.x.as<double>(), s.rel ? s.wo_head.as<int32_t>() : nullptr,
                           s.rel ? s.wo_st.as<int8_t>() : nullptr,
                           s.rel ? s.wo_d.as<double>() : nullptr,
                           s.rel ? s.wo_binv.as<double>() : nullptr);
  }
  c->pfi_decide = nullptr;
  if (rc != MGPU_OK) return rc;
  if (!c->lp_decided) HIPCHK(c, launch_node_decide(c->lp, d, c->stream));
  c->lp_decided = false;
  const int32_t *decision = s.dec.as<int32_t>();
  unsigned long long rcnt[4] = {0, 0, 0, 0};
  if (s.rel) {
    rc = rel_round(c, s, nb, base, bfs);
    if (rc != MGPU_OK) return rc;
    decision = s.dec2.as<int32_t>();
  }
  BnbIO io{};
  io.nb = nb;
  io.base = base;
  io.decision = decision;
  if (s.rel) {
    io.ppvar = s.ppvar.as<int32_t>();
    io.ppval = s.ppval.as<double>();
  }
  io.status = s.st.as<int32_t>();
  io.iters = s.it.as<int32_t>();
  // the shared-root-basis node LPs ran the product form (K3P / K3PW) when the
  // context selects it; per-node bases (warm 1, reliability) run K3 / K3L
  io.pfi_cap = ((s.warm == 0 || s.warm == 2) && !s.rel && s.root_ok) ? mgpu_lp_pfi_cap(c) : 0;
  io.pfi_piv = io.pfi_cap > 0 && c->last_lp_pfi ? c->pfi_piv.as<unsigned long long>() : nullptr;
  io.cand_obj = s.cand.as<double>();
  io.obj = s.obj.as<double>();
  io.bvar = s.bvar.as<int32_t>();
  io.bval = s.bval.as<double>();
  io.bup = s.bup.as<int8_t>();
  io.wlb = s.wlb.as<double>();
  io.wub = s.wub.as<double>();
  io.depth_in = s.depth_in.as<int32_t>();
  io.plb = s.plb.as<double>();
  io.pub = s.pub.as<double>();
  io.pnlb = s.pnlb.as<double>();
  io.pdepth = s.pdepth.as<int32_t>();
  io.pos = s.pos.as<int32_t>();
  io.bsum = s.bsum.as<int32_t>();
  io.bidx = s.bidx.as<int32_t>();
  io.boff = s.boff.as<int32_t>();
  io.bmin = s.bmin.as<double>();
  io.bcnt = s.bcnt.as<int32_t>();
  io.out = s.out.as<BnbOut>();
  if (bfs) {
    io.slots = s.vals2.as<uint32_t>();
    io.live = live;
    io.hw = s.hw;
    io.plive = s.plive.as<uint8_t>();
  }
  if (s.warm == 2) {  // children inherit the node's final basis
    io.kin = bfs ? s.bpk.as<int32_t>() : s.ppk.as<int32_t>() + base;
    io.N = N;
    io.opk = s.opk.as<int32_t>();
    io.oppath = s.oppath.as<uint32_t>();
    io.opst = s.opst.as<int8_t>();
    io.ppk = s.ppk.as<int32_t>();
    io.ppath = s.ppath.as<uint32_t>();
    io.ppst = s.ppst.as<int8_t>();
  }
  if (s.warm == 1) {  // (reliability alone: children keep the root warm start)
    io.m = m;
    io.N = N;
    io.wo_head = s.wo_head.as<int32_t>();
    io.wo_st = s.wo_st.as<int8_t>();
    io.wo_d = s.wo_d.as<double>();
    io.wo_binv = s.wo_binv.as<double>();
    io.ws_head = s.pws_head.as<int32_t>();
    io.ws_st = s.pws_st.as<int8_t>();
    io.ws_d = s.pws_d.as<double>();
    io.ws_binv = s.pws_binv.as<double>();
    if (s.rel) {  // a modified node resumes from its strong branching's basis
      io.mo_head = s.ch_head.as<int32_t>();
      io.mo_st = s.ch_st.as<int8_t>();
      io.mo_d = s.ch_d.as<double>();
      io.mo_binv = s.ch_binv.as<double>();
    }
  }
  HIPCHK(c, hipMemsetAsync(s.out.p, 0, sizeof(BnbOut), c->stream));
  io.defer_children = heap ? 1 : 0;
  HIPCHK(c, launch_bnb_tail(io, n, c->stream));
  BnbOut o;
  HIPCHK(c, hipMemcpyAsync(&o, s.out.p, sizeof o, hipMemcpyDeviceToHost, c->stream));
  if (s.rel)
    HIPCHK(c, hipMemcpyAsync(rcnt, s.rcnt.p, sizeof rcnt, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (heap) {
    rc = heap_children(c, s, io, nb, sel, popped);
    if (rc != MGPU_OK) return rc;
  } else if (!bfs) {
    s.count = base + o.nchild;
  } else if (!heap) {
    s.count = live - nb + o.nchild;
    const long grow = (long)o.nchild - nb - holes;
    if (grow > 0) s.hw += (int)grow;
  }
  s.tot.sb_lps += (long long)rcnt[0];
  s.tot.sb_pruned += (long long)rcnt[1];
  s.tot.sb_modified += (long long)rcnt[2];
  s.tot.sb_pivots += (long long)rcnt[3];
  if (o.best_idx >= 0 && o.best < s.inc) {
    s.inc = o.best;
    HIPCHK(c, hipMemcpy(s.best_x.data(), s.x.as<double>() + (size_t)o.best_idx * n,
                        (size_t)n * 8, hipMemcpyDeviceToHost));
  }
  s.tot.rounds += 1;
  s.tot.nodes += nb;
  for (int k = 0; k < 5; ++k) s.tot.ndec[k] += o.ndec[k];
  s.tot.lps += o.lps;
  s.tot.pivots += o.pivots;
  s.tot.pfi_pivots += o.pfi_pivots;
  s.tot.open = s.count;
  s.tot.incumbent = s.inc;
  s.tot.last_batch = nb;
  if (stats) *stats = s.tot;
  // decision 4 (ProvenUnbounded / EngineUnknownStatus): the reference asserts
  // on an unbounded relaxation (PCBProcessor.cpp:437-442); such a node is not
  // branched, so the tree would end on a wrong optimum: report it
  if (o.ndec[4] > 0)
    return fail(c, MGPU_ERR_ENGINE, "mgpu_bnb_round: %lld node LPs ended unbounded or with an "
                "unknown status; their subtrees were not searched", (long long)o.ndec[4]);
  return MGPU_OK;
}

int mgpu_bnb_shard(mgpu_ctx *c, int rank, int world, int *kept) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->bnb) return fail(c, MGPU_ERR_STATE, "mgpu_bnb_shard: mgpu_bnb_init first");
  if (c->bnb->order == 2)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_shard: not in the reference-heap order (order 2)");
  if (world < 1 || rank < 0 || rank >= world)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_shard: bad rank/world");
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  if (s.order == 1) {
    // best-first pool: keep the live nodes whose index among the live nodes
    // in slot order is rank (mod world); the others become free slots
    std::vector<uint8_t> live((size_t)(s.hw > 0 ? s.hw : 1));
    HIPCHK(c, hipMemcpyAsync(live.data(), s.plive.p, (size_t)s.hw, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int k = 0, idx = 0;
    for (int i = 0; i < s.hw; ++i) {
      if (!live[i]) continue;
      if (idx++ % world == rank) ++k;
      else live[i] = 0;
    }
    HIPCHK(c, hipMemcpy(s.plive.p, live.data(), (size_t)s.hw, hipMemcpyHostToDevice));
    s.count = k;
    s.tot.open = k;
    if (kept) *kept = k;
    return MGPU_OK;
  }
  const size_t cnt = (size_t)(s.count > 0 ? s.count : 1);
  DevBuf &tlb = s.mw_tlb, &tub = s.mw_tub, &tnlb = s.mw_tnlb, &tdep = s.mw_tdep;
  HIPCHK(c, tlb.ensure(cnt * s.n * 8));
  HIPCHK(c, tub.ensure(cnt * s.n * 8));
  HIPCHK(c, tnlb.ensure(cnt * 8));
  HIPCHK(c, tdep.ensure(cnt * 4));
  int k = 0;
  hipError_t e = launch_bnb_shard(s.plb.as<double>(), s.pub.as<double>(), s.pnlb.as<double>(),
                                  s.pdepth.as<int32_t>(), tlb.as<double>(), tub.as<double>(),
                                  tnlb.as<double>(), tdep.as<int32_t>(), s.count, s.n, rank,
                                  world, &k, c->stream);
  // every other per-slot array moves with its node (parent warm starts,
  // parent branching data, paths): slot k <- slot rank + k * world
  if (e == hipSuccess && k > 0) {
    const int m = c->lp.m, N = s.n + m;
    std::vector<std::pair<DevBuf *, size_t>> rows;
    if (s.warm == 1)
      rows = {{&s.pws_head, (size_t)m * 4}, {&s.pws_st, (size_t)N}, {&s.pws_d, (size_t)N * 8},
              {&s.pws_binv, (size_t)m * m * 8}};
    if (s.warm == 2)
      rows = {{&s.ppk, 4}, {&s.ppath, (size_t)kPathMax * 4}, {&s.ppst, (size_t)N}};
    if (s.rel) {
      rows.push_back({&s.ppvar, 4});
      rows.push_back({&s.ppval, 8});
    }
    size_t most = 0;
    for (auto &r : rows) most = r.second > most ? r.second : most;
    DevBuf &tmp = s.mw_tmp;
    if (most > 0) e = tmp.ensure((size_t)k * most);
    for (auto &r : rows)
      if (e == hipSuccess)
        e = launch_bnb_shard_rows(r.first->as<unsigned char>(), tmp.as<unsigned char>(), r.second,
                                  k, rank, world, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  } else if (e == hipSuccess) {
    e = hipStreamSynchronize(c->stream);
  }
  HIPCHK(c, e);
  s.count = k;
  s.tot.open = k;
  if (kept) *kept = k;
  return MGPU_OK;
}

int mgpu_strong_branch_dev(mgpu_ctx *c, const double *lb, const double *ub, int ncand,
                           const int32_t *cand_var, const double *cand_val,
                           const int32_t *ws_head, const int8_t *ws_st, const double *ws_d,
                           const double *ws_binv, int iter_limit, double *child_lb,
                           double *child_ub, int32_t *status, double *obj, int32_t *iters) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_strong_branch: no problem loaded");
  if (ncand < 0 || (ncand > 0 && (!lb || !ub || !cand_var || !cand_val || !child_lb ||
                                  !child_ub || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_strong_branch: bad argument");
  if (ncand == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, launch_sb_boxes(lb, ub, cand_var, cand_val, ncand, c->lp.n, child_lb, child_ub,
                            c->stream));
  return mgpu_lp_solve_dev(c, 2 * ncand, child_lb, child_ub, nullptr, ws_head, ws_st, ws_d,
                           ws_binv, 1, iter_limit, status, obj, iters, nullptr, nullptr,
                           nullptr, nullptr, nullptr);
}

int mgpu_strong_branch(mgpu_ctx *c, const double *lb, const double *ub, int ncand,
                       const int32_t *cand_var, const double *cand_val, const int32_t *ws_head,
                       const int8_t *ws_st, const double *ws_d, const double *ws_binv,
                       int iter_limit, int32_t *status, double *obj, int32_t *iters) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_strong_branch: no problem loaded");
  if (ncand < 0 || (ncand > 0 && (!lb || !ub || !cand_var || !cand_val || !status || !obj ||
                                  !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_strong_branch: bad argument");
  if (ncand == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = c->lp.n, m = c->lp.m, N = n + m, nch = 2 * ncand;
  DevBuf box, cb, io, wsb;  // per-call workspace
  const size_t nb = (size_t)n * 8;
  HIPCHK(c, box.ensure(2 * nb + (size_t)ncand * 12));
  HIPCHK(c, cb.ensure(2 * (size_t)nch * nb));
  HIPCHK(c, io.ensure((size_t)nch * 16));
  double *d_lb = box.as<double>(), *d_ub = d_lb + n;
  double *d_val = d_ub + n;
  int32_t *d_var = reinterpret_cast<int32_t *>(d_val + ncand);
  double *d_clb = cb.as<double>(), *d_cub = d_clb + (size_t)nch * n;
  int32_t *d_st = io.as<int32_t>(), *d_it = d_st + nch;
  double *d_obj = reinterpret_cast<double *>(d_it + nch);
  const int32_t *w_head = nullptr;
  const int8_t *w_st = nullptr;
  const double *w_d = nullptr, *w_binv = nullptr;
  if (ws_head) {
    if (!ws_st || !ws_d || !ws_binv)
      return fail(c, MGPU_ERR_ARG, "mgpu_strong_branch: warm start needs head, st, d and binv");
    HIPCHK(c, wsb.ensure((size_t)m * 4 + (size_t)N * 9 + (size_t)m * m * 8 + 64));
    char *w = wsb.as<char>();
    double *pb = reinterpret_cast<double *>(w);
    double *pd = pb + (size_t)m * m;
    int32_t *ph = reinterpret_cast<int32_t *>(pd + N);
    int8_t *ps = reinterpret_cast<int8_t *>(ph + m);
    HIPCHK(c, hipMemcpyAsync(pb, ws_binv, (size_t)m * m * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(pd, ws_d, (size_t)N * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(ph, ws_head, (size_t)m * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(ps, ws_st, (size_t)N, hipMemcpyHostToDevice, c->stream));
    w_head = ph;
    w_st = ps;
    w_d = pd;
    w_binv = pb;
  }
  HIPCHK(c, hipMemcpyAsync(d_lb, lb, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_ub, ub, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_val, cand_val, (size_t)ncand * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_var, cand_var, (size_t)ncand * 4, hipMemcpyHostToDevice, c->stream));
  int rc = mgpu_strong_branch_dev(c, d_lb, d_ub, ncand, d_var, d_val, w_head, w_st, w_d, w_binv,
                                  iter_limit, d_clb, d_cub, d_st, d_obj, d_it);
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(status, d_st, (size_t)nch * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(obj, d_obj, (size_t)nch * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(iters, d_it, (size_t)nch * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

// Node migration for load balancing across ranks (MpiBranchAndBound::
// LoadBalance_, MpiBranchAndBound.cpp:78-195).  LoadBalance_ pops each rank's
// next 50 P candidates (:93-105), all-gathers their lower bounds (:107),
// sorts them globally and deals the i-th best to rank i mod P (:111-188).
// mgpu_bnb_pick is the pop (the nodes stay in the pool, only their bounds
// leave), mgpu_bnb_export_dev packs the chosen ones into device rows and
// removes them, mgpu_bnb_import_dev places received rows.  Rows are
// [lb n | ub n | bound | depth] f64, plus the node's basis in warm mode 2
// (bnb_migrate.hip; mgpu_bnb_row_width).
}  // extern "C"

namespace {

// every per-slot array of the pool (a node's box, bound, depth and the state
// that travels with it inside one pool)
std::vector<std::pair<DevBuf *, size_t>> slot_rows(BnbState &s, int m) {
  const size_t n = (size_t)s.n, N = n + (size_t)m;
  std::vector<std::pair<DevBuf *, size_t>> r = {
      {&s.plb, n * 8}, {&s.pub, n * 8}, {&s.pnlb, 8}, {&s.pdepth, 4}};
  if (s.warm == 1) {
    r.push_back({&s.pws_head, (size_t)m * 4});
    r.push_back({&s.pws_st, N});
    r.push_back({&s.pws_d, N * 8});
    r.push_back({&s.pws_binv, (size_t)m * m * 8});
  }
  if (s.warm == 2) {
    r.push_back({&s.ppk, 4});
    r.push_back({&s.ppath, (size_t)kPathMax * 4});
    r.push_back({&s.ppst, N});
  }
  if (s.rel) {
    r.push_back({&s.ppvar, 4});
    r.push_back({&s.ppval, 8});
  }
  return r;
}

// migration row width in doubles: [lb | ub | bound | depth], plus in warm
// mode 2 [k | path (kPathMax) | statuses, 16 per double] (bnb_migrate.hip)
size_t mig_width(const BnbState &s, int m) {
  const size_t N = (size_t)s.n + (size_t)m;
  return 2 * (size_t)s.n + 2 + (s.warm == 2 ? 1 + (size_t)kPathMax + (N + 15) / 16 : 0);
}

inline double key_to_double(uint64_t k) {
  const uint64_t b = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  double v;
  std::memcpy(&v, &b, 8);
  return v;
}

// removes the nodes at pool slots `slots` after packing them into `buf`
// (device rows); depth-first: the slots must lie in the stack's top `region`
// slots, the others of that region keep their order and close the gaps
int take_nodes(mgpu_ctx *c, BnbState &s, const std::vector<int32_t> &slots, int region,
               double *buf) {
  const int k = (int)slots.size();
  if (k == 0) return MGPU_OK;
  DevBuf &dsl = s.mw_slots;
  HIPCHK(c, dsl.ensure((size_t)k * 4));
  HIPCHK(c, hipMemcpyAsync(dsl.p, slots.data(), (size_t)k * 4, hipMemcpyHostToDevice,
                           c->stream));
  MigratePack pk{};
  pk.k = k;
  pk.n = s.n;
  pk.N = s.n + c->lp.m;
  pk.W = (int)mig_width(s, c->lp.m);
  pk.slots = dsl.as<int32_t>();
  pk.plb = s.plb.as<double>();
  pk.pub = s.pub.as<double>();
  pk.pnlb = s.pnlb.as<double>();
  pk.pdepth = s.pdepth.as<int32_t>();
  pk.plive = s.order == 1 ? s.plive.as<uint8_t>() : nullptr;
  if (s.warm == 2) {
    pk.ppk = s.ppk.as<int32_t>();
    pk.ppath = s.ppath.as<uint32_t>();
    pk.ppst = s.ppst.as<int8_t>();
  }
  pk.buf = buf;
  HIPCHK(c, launch_bnb_pack(pk, c->stream));
  if (s.order == 0) {
    const int base = s.count - region;
    std::vector<uint8_t> gone((size_t)region, 0);
    for (int32_t v : slots) gone[(size_t)(v - base)] = 1;
    // the kept nodes of the region close up in order; only rows that change
    // place move
    std::vector<int32_t> f2, t2;
    int w = 0;
    for (int t = 0; t < region; ++t) {
      if (gone[(size_t)t]) continue;
      if (t != w) {
        f2.push_back(base + t);
        t2.push_back(base + w);
      }
      ++w;
    }
    if (!f2.empty()) {
      const int km = (int)f2.size();
      DevBuf &ft = s.mw_ft, &tmp = s.mw_tmp;
      HIPCHK(c, ft.ensure((size_t)km * 8));
      HIPCHK(c, hipMemcpyAsync(ft.p, f2.data(), (size_t)km * 4, hipMemcpyHostToDevice,
                               c->stream));
      HIPCHK(c, hipMemcpyAsync(ft.as<int32_t>() + km, t2.data(), (size_t)km * 4,
                               hipMemcpyHostToDevice, c->stream));
      auto rows = slot_rows(s, c->lp.m);
      size_t most = 0;
      for (auto &r : rows) most = r.second > most ? r.second : most;
      HIPCHK(c, tmp.ensure((size_t)km * most));
      for (auto &r : rows)
        HIPCHK(c, launch_bnb_move_rows(r.first->as<unsigned char>(), tmp.as<unsigned char>(),
                                       r.second, ft.as<int32_t>(), ft.as<int32_t>() + km, km,
                                       c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  s.count -= k;
  s.tot.open = s.count;
  return MGPU_OK;
}

// places k device rows: on top of the stack, or (best-first) into the
// lowest free pool slots first and past the high-water mark for the rest
int place_nodes(mgpu_ctx *c, BnbState &s, int k, const double *buf) {
  if (k == 0) return MGPU_OK;
  const int m = c->lp.m, N = s.n + m;
  std::vector<int32_t> slots;
  slots.reserve((size_t)k);
  if (s.order == 0) {
    if (s.count + k > s.cap) return fail(c, MGPU_ERR_NOMEM, "mgpu_bnb_import: node pool full");
    for (int t = 0; t < k; ++t) slots.push_back(s.count + t);
  } else {
    std::vector<uint8_t> live((size_t)(s.hw > 0 ? s.hw : 1), 0);
    if (s.hw > 0) {
      HIPCHK(c, hipMemcpyAsync(live.data(), s.plive.p, (size_t)s.hw, hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    for (int i = 0; i < s.hw && (int)slots.size() < k; ++i)
      if (!live[(size_t)i]) slots.push_back(i);
    const int extra = k - (int)slots.size();
    if (s.hw + extra > s.cap) return fail(c, MGPU_ERR_NOMEM, "mgpu_bnb_import: node pool full");
    for (int t = 0; t < extra; ++t) slots.push_back(s.hw + t);
    s.hw += extra;
  }
  DevBuf &dsl = s.mw_slots;
  HIPCHK(c, dsl.ensure((size_t)k * 4));
  HIPCHK(c, hipMemcpyAsync(dsl.p, slots.data(), (size_t)k * 4, hipMemcpyHostToDevice,
                           c->stream));
  MigrateIO io{};
  io.k = k;
  io.n = s.n;
  io.m = m;
  io.N = N;
  io.W = (int)mig_width(s, m);
  io.slots = dsl.as<int32_t>();
  io.buf = buf;
  io.plb = s.plb.as<double>();
  io.pub = s.pub.as<double>();
  io.pnlb = s.pnlb.as<double>();
  io.pdepth = s.pdepth.as<int32_t>();
  io.plive = s.order == 1 ? s.plive.as<uint8_t>() : nullptr;
  io.ppvar = s.rel ? s.ppvar.as<int32_t>() : nullptr;
  if (s.warm == 2) {  // the basis each row carries (k 0: the root basis)
    io.ppk = s.ppk.as<int32_t>();
    io.ppath = s.ppath.as<uint32_t>();
    io.ppst = s.ppst.as<int8_t>();
  }
  if (s.warm == 1) {  // a migrated node starts from the root basis
    io.ws_head = s.pws_head.as<int32_t>();
    io.ws_st = s.pws_st.as<int8_t>();
    io.ws_d = s.pws_d.as<double>();
    io.ws_binv = s.pws_binv.as<double>();
    io.r_head = s.ws_head.as<int32_t>();
    io.r_st = s.ws_st.as<int8_t>();
    io.r_d = s.ws_d.as<double>();
    io.r_binv = s.ws_binv.as<double>();
  }
  HIPCHK(c, launch_bnb_unpack(io, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  s.count += k;
  s.tot.open = s.count;
  return MGPU_OK;
}

int check_migrate(mgpu_ctx *c, const char *what) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->bnb) return fail(c, MGPU_ERR_STATE, "%s: mgpu_bnb_init first", what);
  if (c->bnb->order == 2)
    return fail(c, MGPU_ERR_ARG, "%s: not in the reference-heap order (order 2)", what);
  return MGPU_OK;
}

}  // namespace

extern "C" {

// The pool-side migration workspaces for an exchange of up to S rows (a
// pick of S, then an export of k <= S rows from those S slots and an import
// of k <= S rows): sized once for that worst case, so a rebalance inside a
// timed region never allocates (mgpu_bnb_rebalance calls this first).
extern "C++" int bnb_reserve_migration(mgpu_ctx *c, int S) {
  int rc = check_migrate(c, "mgpu_bnb_rebalance");
  if (rc != MGPU_OK) return rc;
  BnbState &s = *c->bnb;
  const size_t k = (size_t)(S > 0 ? S : 1);
  size_t most = 0;
  for (auto &r : slot_rows(s, c->lp.m)) most = r.second > most ? r.second : most;
  HIPCHK(c, s.mw_slots.ensure(k * 4));
  HIPCHK(c, s.mw_ft.ensure(k * 8));
  HIPCHK(c, s.mw_tmp.ensure(k * most));
  return MGPU_OK;
}

int mgpu_bnb_pick(mgpu_ctx *c, int S, double *lbs, int *got) {
  int rc = check_migrate(c, "mgpu_bnb_pick");
  if (rc != MGPU_OK) return rc;
  if (S < 0 || (S > 0 && !lbs) || !got) return fail(c, MGPU_ERR_ARG, "mgpu_bnb_pick: bad argument");
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  s.pick.clear();
  *got = 0;
  if (s.order == 0) {
    // the stack's next candidates: its top, topmost first
    const int k = S < s.count ? S : s.count;
    if (k > 0) {
      std::vector<double> v((size_t)k);
      HIPCHK(c, hipMemcpyAsync(v.data(), s.pnlb.as<double>() + (s.count - k), (size_t)k * 8,
                               hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int t = 0; t < k; ++t) {
        lbs[t] = v[(size_t)(k - 1 - t)];
        s.pick.push_back(s.count - 1 - t);
      }
    }
    *got = k;
    return MGPU_OK;
  }
  // best-first: TreeManager::getCandidate's pruning by the incumbent, then
  // the live nodes in (bound, slot) order, as a round selects them
  if (s.hw <= 0) {
    s.count = 0;
    s.tot.open = 0;
    return MGPU_OK;
  }
  HIPCHK(c, hipMemsetAsync(s.counts.p, 0, 8, c->stream));
  HIPCHK(c, launch_bnb_keys(s.pnlb.as<double>(), s.plive.as<uint8_t>(), s.hw, s.inc, s.inc,
                            s.keys.as<uint64_t>(), s.vals.as<uint32_t>(), s.counts.as<int32_t>(),
                            c->stream));
  size_t tb = s.sort_bytes;
  HIPCHK(c, bnb_sort_pairs(s.sort_tmp.p, tb, s.keys.as<uint64_t>(), s.keys2.as<uint64_t>(),
                           s.vals.as<uint32_t>(), s.vals2.as<uint32_t>(), s.hw, c->stream));
  int32_t cnt[2] = {0, 0};
  HIPCHK(c, hipMemcpyAsync(cnt, s.counts.p, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  s.count = cnt[0];
  s.tot.pruned += cnt[1];
  s.tot.open = s.count;
  const int k = S < s.count ? S : s.count;
  if (k > 0) {
    std::vector<uint64_t> keys((size_t)k);
    std::vector<uint32_t> sl((size_t)k);
    HIPCHK(c, hipMemcpyAsync(keys.data(), s.keys2.p, (size_t)k * 8, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(sl.data(), s.vals2.p, (size_t)k * 4, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int t = 0; t < k; ++t) {
      lbs[t] = key_to_double(keys[(size_t)t]);
      s.pick.push_back((int)sl[(size_t)t]);
    }
  }
  *got = k;
  return MGPU_OK;
}

int mgpu_bnb_export_dev(mgpu_ctx *c, int k, const int32_t *idx, double *buf) {
  int rc = check_migrate(c, "mgpu_bnb_export_dev");
  if (rc != MGPU_OK) return rc;
  BnbState &s = *c->bnb;
  if (k < 0 || (k > 0 && (!idx || !buf)))
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_export_dev: bad argument");
  const int np = (int)s.pick.size();
  std::vector<uint8_t> seen((size_t)(np > 0 ? np : 1), 0);
  std::vector<int32_t> slots;
  for (int t = 0; t < k; ++t) {
    if (idx[t] < 0 || idx[t] >= np || seen[(size_t)idx[t]])
      return fail(c, MGPU_ERR_ARG, "mgpu_bnb_export_dev: index %d is not a distinct entry of "
                  "the last mgpu_bnb_pick (%d nodes)", idx[t], np);
    seen[(size_t)idx[t]] = 1;
    slots.push_back(s.pick[(size_t)idx[t]]);
  }
  HIPCHK(c, hipSetDevice(c->device));
  rc = take_nodes(c, s, slots, np, buf);
  s.pick.clear();
  return rc;
}

int mgpu_bnb_import_dev(mgpu_ctx *c, int k, const double *buf) {
  int rc = check_migrate(c, "mgpu_bnb_import_dev");
  if (rc != MGPU_OK) return rc;
  if (k < 0 || (k > 0 && !buf)) return fail(c, MGPU_ERR_ARG, "mgpu_bnb_import_dev: bad argument");
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  s.pick.clear();
  return place_nodes(c, s, k, buf);
}

int mgpu_bnb_row_width(mgpu_ctx *c) {
  int rc = check_migrate(c, "mgpu_bnb_row_width");
  if (rc != MGPU_OK) return rc;
  return (int)mig_width(*c->bnb, c->lp.m);
}

int mgpu_bnb_count(mgpu_ctx *c, int *open, int *spare) {
  int rc = check_migrate(c, "mgpu_bnb_count");
  if (rc != MGPU_OK) return rc;
  if (open) *open = c->bnb->count;
  if (spare) *spare = c->bnb->cap - c->bnb->count;
  return MGPU_OK;
}

// Host-buffer forms (boxes [k][n]): the stack's top k / the first k live
// slots leave; imports go through the same placement as the device rows.
int mgpu_bnb_export(mgpu_ctx *c, int k, double *lb, double *ub, double *nlb, int32_t *depth,
                    int *got) {
  int rc = check_migrate(c, "mgpu_bnb_export");
  if (rc != MGPU_OK) return rc;
  if (k < 0 || (k > 0 && (!lb || !ub || !nlb || !depth)) || !got)
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_export: bad argument");
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = s.n;
  if (k > s.count) k = s.count;
  *got = 0;
  s.pick.clear();
  if (k == 0) return MGPU_OK;
  std::vector<int32_t> slots;
  if (s.order == 0) {
    for (int t = 0; t < k; ++t) slots.push_back(s.count - k + t);
  } else {
    std::vector<uint8_t> live((size_t)s.hw);
    HIPCHK(c, hipMemcpyAsync(live.data(), s.plive.p, (size_t)s.hw, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < s.hw && (int)slots.size() < k; ++i)
      if (live[(size_t)i]) slots.push_back(i);
    k = (int)slots.size();
  }
  const size_t W = mig_width(s, c->lp.m);
  DevBuf rows;
  HIPCHK(c, rows.ensure((size_t)k * W * 8));
  rc = take_nodes(c, s, slots, k, rows.as<double>());
  if (rc != MGPU_OK) return rc;
  std::vector<double> h((size_t)k * W);
  HIPCHK(c, hipMemcpy(h.data(), rows.p, h.size() * 8, hipMemcpyDeviceToHost));
  for (int t = 0; t < k; ++t) {
    const double *r = h.data() + (size_t)t * W;
    std::memcpy(lb + (size_t)t * n, r, (size_t)n * 8);
    std::memcpy(ub + (size_t)t * n, r + n, (size_t)n * 8);
    nlb[t] = r[2 * n];
    depth[t] = (int32_t)r[2 * n + 1];
  }
  *got = k;
  return MGPU_OK;
}

int mgpu_bnb_import(mgpu_ctx *c, int k, const double *lb, const double *ub, const double *nlb,
                    const int32_t *depth) {
  int rc = check_migrate(c, "mgpu_bnb_import");
  if (rc != MGPU_OK) return rc;
  if (k < 0 || (k > 0 && (!lb || !ub || !nlb || !depth)))
    return fail(c, MGPU_ERR_ARG, "mgpu_bnb_import: bad argument");
  if (k == 0) return MGPU_OK;
  BnbState &s = *c->bnb;
  HIPCHK(c, hipSetDevice(c->device));
  s.pick.clear();
  const int n = s.n;
  const size_t W = mig_width(s, c->lp.m);   // (host boxes: k 0, the root basis)
  std::vector<double> h((size_t)k * W, 0.0);
  for (int t = 0; t < k; ++t) {
    double *r = h.data() + (size_t)t * W;
    std::memcpy(r, lb + (size_t)t * n, (size_t)n * 8);
    std::memcpy(r + n, ub + (size_t)t * n, (size_t)n * 8);
    r[2 * n] = nlb[t];
    r[2 * n + 1] = (double)depth[t];
  }
  DevBuf rows;
  HIPCHK(c, rows.ensure(h.size() * 8));
  HIPCHK(c, hipMemcpyAsync(rows.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, c->stream));
  return place_nodes(c, s, k, rows.as<double>());
}

int mgpu_bnb_best(mgpu_ctx *c, double *obj, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->bnb) return fail(c, MGPU_ERR_STATE, "mgpu_bnb_best: mgpu_bnb_init first");
  BnbState &s = *c->bnb;
  if (obj) *obj = s.inc;
  if (x) std::memcpy(x, s.best_x.data(), (size_t)s.n * 8);
  return MGPU_OK;
}

}  // extern "C"
