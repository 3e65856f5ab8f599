// Batched reliability branching (ReliabilityBrancher, src/base/
// ReliabilityBrancher.cpp, the reference's default brancher), gfx950.
//
// The reference runs findBranches node by node: pseudocost state is updated
// after every node solve (updateAfterSolve, :508-530) and after every
// strong-branched candidate (useStrongBranchInfo_, :539-576).  A batched
// round processes B nodes at once, so here every node of a round sees the
// pseudocost state of the round's start plus its OWN updateAfterSolve
// observation; the round's observations are then folded into the state in
// node order (the reference's order).  With one node per round this is the
// reference's sequence exactly.
//
// Kernels of one round (bnb.cpp drives them after node_decide):
//   rel_flags / excl_scan : rank of each branching node among the round's
//                           (findBranches call number = calls0 + rank + 1);
//   rel_prepare           : per node, the IntVarHandler candidates
//                           (IntVarHandler.cpp:86-108), the reliable test
//                           (findCandidates_, :238-320) and the first
//                           maxStrongCands_ (20) unreliable ones in
//                           CompareScore order (score, then index);
//   excl_scan             : offsets of the nodes' strong-branching LPs;
//   rel_children          : their child boxes (getBrMod: down ub = floor x,
//                           up lb = ceil x) and warm-start index (the node's
//                           own optimal basis);
//   rel_chain_*           : the strong-branching LPs chained per node through
//                           one warm-start slot (K3 / K3L steps, iteration
//                           limit 25, :101), stopping at the first verdict;
//   rel_decide            : findBestCandidate_ (:75-159) per node: reliable
//                           pseudocost scores, the strong-branching results
//                           (shouldPrune_, useStrongBranchInfo_: prune / one-
//                           sided bound change / pseudocost observation),
//                           the remaining unreliable candidates; direction
//                           = down first when change_up > change_down;
//   pc_fold               : the round's observations into the pseudocosts,
//                           per variable in node order (updatePCost_).
// One wave per node in rel_prepare / rel_decide (round 5; one thread per node
// before): the candidate scans are wave reductions over the reference's
// (score, index) keys, which took the per-round latency of the two kernels
// from ~90 us each on a tree's narrow rounds.
#include "bnb_internal.h"
#include "sb_rule.h"
#include "wave.h"

#include <climits>

namespace mgpu {
namespace {

__device__ __forceinline__ bool is_int(uint8_t t) { return t == kBinary || t == kInteger; }

// IntVarHandler::getBranchingCandidates: |floor(x + 0.5) - x| > intTol
__device__ __forceinline__ bool fractional(double v) {
  return fabs(floor(v + 0.5) - v) > kIntTol;
}

// ReliabilityBrancher::getScore_ (:368-377)
__device__ __forceinline__ double rel_score(double up, double down) {
  return up > down ? down * 0.8 + up * 0.2 : up * 0.8 + down * 0.2;
}

// updateAfterSolve's observation of this node (:508-530): cost of the
// parent's branching, (lb - parent lb) / (|x_j - x_j(parent)| + eTol), 0 when
// negative / inf / nan; side 0 down (x_j decreased), 1 up.
__device__ __forceinline__ bool after_solve_obs(const RelIO &io, int b, int &var, int &side,
                                                double &cost) {
  const int dec = io.decision[b];
  var = io.pvar[b];
  if (var < 0 || !(dec == 0 || dec == 3)) return false;
  const double oldval = io.pval[b], newval = io.x[(size_t)b * io.n + var];
  double c = (io.obj[b] - io.nlb[b]) / (fabs(newval - oldval) + kRelETol);
  if (c < 0.0 || isinf(c) || isnan(c)) c = 0.0;
  cost = c;
  side = newval < oldval ? 0 : 1;
  return true;
}

// the state of variable j as this node sees it: the round's start plus its
// own updateAfterSolve observation (updatePCost_, :532-537)
struct PcView {
  double pu, pd;
  int cu, cd;
};
__device__ __forceinline__ PcView pc_view(const RelIO &io, int j, bool own, int ov, int os,
                                          double oc) {
  PcView v{io.pc_up[j], io.pc_dn[j], io.cnt_up[j], io.cnt_dn[j]};
  if (own && j == ov) {
    if (os == 0) {
      v.pd = (v.pd * v.cd + oc) / (v.cd + 1);
      v.cd += 1;
    } else {
      v.pu = (v.pu * v.cu + oc) / (v.cu + 1);
      v.cu += 1;
    }
  }
  return v;
}

__device__ __forceinline__ long long calls_of(const RelIO &io, int b) {
  return io.calls0 + io.rank[b] + 1;
}

// findCandidates_ reliable test (:297-300).  calls and lastStrBranched_
// are UInt: their difference wraps around as the reference's does.
__device__ __forceinline__ bool reliable(const RelIO &io, int j, long long calls, const PcView &v) {
  const unsigned d = (unsigned)calls - (unsigned)io.last[j];
  return (double)kRelMinDist > fabs((double)d) || (v.cu >= kRelThresh && v.cd >= kRelThresh);
}

// unreliable score (:301-304): times - s_wt * (pseudo up + down) - i_wt * max(dd, ud)
__device__ __forceinline__ double unrel_score(const PcView &v, double dd, double ud) {
  return (double)(v.cu + v.cd) - 1e-5 * (v.pu + v.pd) - 1e-6 * fmax(dd, ud);
}

__global__ __launch_bounds__(256) void rel_flags(RelIO io, int32_t *flag) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < io.nb) flag[b] = io.decision[b] == 0 ? 1 : 0;
}

// exclusive scan of in[0, nb) into out, total into *total (one workgroup)
__global__ __launch_bounds__(1024) void excl_scan(const int32_t *in, int32_t *out, int nb,
                                                  int32_t *total) {
  __shared__ int s[1024];
  __shared__ int carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < nb; c0 += 1024) {
    const int i = c0 + t;
    const int v = i < nb ? in[i] : 0;
    s[t] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int u = t >= o ? s[t - o] : 0;
      __syncthreads();
      s[t] += u;
      __syncthreads();
    }
    if (i < nb) out[i] = carry + s[t] - v;
    __syncthreads();
    if (t == 1023) carry += s[1023];
    __syncthreads();
  }
  if (t == 0) *total = carry;
}

// Lexicographic (u, j) minimum over the wave: the smallest u, the smallest j
// among its holders (u = +INF, j = INT_MAX: no candidate).  Wave uniform.
__device__ __forceinline__ void wave_min_key(double &u, int &j) {
  const double mu = wave_min_dpp(u);
  j = wave_min_i32_dpp(u == mu ? j : INT_MAX);
  u = mu;
}
// (v, key u, j) maximum over the wave: the largest v, then the smallest (u, j)
// among its holders.  v = -INF: no candidate.  Wave uniform.
__device__ __forceinline__ void wave_max_key(double &v, double &u, int &j) {
  const double mv = wave_max_dpp(v);
  double uu = v == mv ? u : INFINITY;
  int jj = v == mv ? j : INT_MAX;
  wave_min_key(uu, jj);
  v = mv;
  u = uu;
  j = jj;
}

// One wave per node: the candidates are spread over the lanes (column j of
// lane j % 64); every selection is a wave reduction over (score, index) keys,
// the same keys and the same order as the reference's serial scans.  The keys
// are computed once into registers (kPrepSlots columns per lane; the
// repeated selection then reads no memory) and the owner lane of each chosen
// column writes it: the selection loop is register work and DPP reductions,
// not up to 20 rounds of dependent global loads.
constexpr int kPrepSlots = 4;   // n <= 256 keeps the keys in registers

__global__ __launch_bounds__(256) void rel_prepare(RelIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  int nsb = 0;
  if (io.decision[b] == 0) {
    const double *x = io.x + (size_t)b * io.n;
    int ov = -1, os = 0;
    double oc = 0.0;
    const bool own = after_solve_obs(io, b, ov, os, oc);
    const long long calls = calls_of(io, b);
    // the first kRelMaxCands unreliable candidates in (score, index) order:
    // repeated selection of the next larger key; none below maxDepth_
    // (findBestCandidate_: maxcnt = depth > maxDepth_ ? 0 : maxStrongCands_)
    const int maxcnt = io.depth[b] > kRelMaxDepth ? 0 : kRelMaxCands;
    double ps = -INFINITY;
    int pj = -1;
    if (io.n <= 64 * kPrepSlots) {
      bool cand[kPrepSlots];
      double key[kPrepSlots], xv[kPrepSlots];
#pragma unroll
      for (int t = 0; t < kPrepSlots; ++t) {
        const int j = lane + 64 * t;
        cand[t] = false;
        key[t] = 0.0;
        xv[t] = 0.0;
        if (j < io.n && maxcnt > 0 && is_int(io.vtype[j])) {
          const double v = x[j];
          if (fractional(v)) {
            const PcView pv = pc_view(io, j, own, ov, os, oc);
            if (!reliable(io, j, calls, pv)) {
              cand[t] = true;
              key[t] = unrel_score(pv, v - floor(v), ceil(v) - v);
              xv[t] = v;
            }
          }
        }
      }
      for (int k = 0; k < maxcnt; ++k) {
        double bs = INFINITY;
        int bj = INT_MAX;
#pragma unroll
        for (int t = 0; t < kPrepSlots; ++t) {
          const int j = lane + 64 * t;
          const double sc = key[t];
          const bool after = sc > ps || (sc == ps && j > pj);
          if (cand[t] && after && (sc < bs || (sc == bs && j < bj))) {
            bs = sc;
            bj = j;
          }
        }
        wave_min_key(bs, bj);
        if (bj == INT_MAX) break;
        if ((bj & 63) == lane) {   // the column's own lane holds its value
          const int t = bj >> 6;
          double v = xv[0];
#pragma unroll
          for (int u = 1; u < kPrepSlots; ++u)
            if (u == t) v = xv[u];
          io.sb_var[(size_t)b * kRelMaxCands + k] = bj;
          io.sb_val[(size_t)b * kRelMaxCands + k] = v;
        }
        ++nsb;
        ps = bs;
        pj = bj;
      }
    } else {
      for (int k = 0; k < maxcnt; ++k) {
        double bs = INFINITY;
        int bj = INT_MAX;
        for (int j = lane; j < io.n; j += 64) {
          if (!is_int(io.vtype[j])) continue;
          const double v = x[j];
          if (!fractional(v)) continue;
          const PcView pv = pc_view(io, j, own, ov, os, oc);
          if (reliable(io, j, calls, pv)) continue;
          const double sc = unrel_score(pv, v - floor(v), ceil(v) - v);
          const bool after = sc > ps || (sc == ps && j > pj);
          if (after && (sc < bs || (sc == bs && j < bj))) {
            bs = sc;
            bj = j;
          }
        }
        wave_min_key(bs, bj);
        if (bj == INT_MAX) break;
        if (lane == 0) {
          io.sb_var[(size_t)b * kRelMaxCands + k] = bj;
          io.sb_val[(size_t)b * kRelMaxCands + k] = x[bj];
        }
        ++nsb;
        ps = bs;
        pj = bj;
      }
    }
  }
  if (lane == 0) {
    io.nsb[b] = nsb;
    if (nsb > 0) atomicMax(io.nsb_max, nsb);
  }
}

// one wave per strong-branching child: the node's (FBBT-tightened) box with
// the candidate's bound change
__global__ __launch_bounds__(256) void rel_children(RelIO io, const double *wlb, const double *wub,
                                                    double *clb, double *cub, int32_t *cnode) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  const int k2 = 2 * io.nsb[b];
  const size_t off = 2 * (size_t)io.sb_off[b];
  for (int ch = 0; ch < k2; ++ch) {
    const int j = io.sb_var[(size_t)b * kRelMaxCands + (ch >> 1)];
    const double v = io.sb_val[(size_t)b * kRelMaxCands + (ch >> 1)];
    const bool up = ch & 1;
    double *dl = clb + (off + ch) * io.n, *du = cub + (off + ch) * io.n;
    for (int k = lane; k < io.n; k += 64) {
      double l = wlb[(size_t)b * io.n + k], u = wub[(size_t)b * io.n + k];
      if (k == j) {
        if (up) l = ceil(v);
        else u = floor(v);
      }
      dl[k] = l;
      du[k] = u;
    }
    if (lane == 0) cnode[off + ch] = b;
  }
}

static_assert(kSbETol == kRelETol, "one eTol_ for the strong-branching verdict");

// candidate k of node b after both strong-branching LPs (sb_verdict)
__device__ __forceinline__ int sb_outcome(const RelIO &io, size_t off, int k, double objval,
                                          double maxchange, double &cd, double &cu) {
  return sb_verdict(io.c_status[off + 2 * k], io.c_obj[off + 2 * k], io.c_status[off + 2 * k + 1],
                    io.c_obj[off + 2 * k + 1], objval, maxchange, cd, cu);
}

// One wave per node (as rel_prepare): the candidate scans are wave
// reductions, the strong-branching results a uniform loop; the winner is the
// first maximum of the reference's scan order -- reliable candidates by
// ascending index, then the strong-branched ones, then the remaining
// unreliable ones in CompareScore order -- which the reductions restate as
// (score max, order key min).
__global__ __launch_bounds__(256) void rel_decide(RelIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  const size_t e0 = (size_t)b * kRelEvents;
  int ov = -1, os = 0, nev = 0;
  double oc = 0.0;
  const bool own = after_solve_obs(io, b, ov, os, oc);
  if (own) {  // updateAfterSolve comes first (PCBProcessor.cpp:245-248)
    if (lane == 0) {
      io.ev_var[e0] = ov;
      io.ev_side[e0] = (int8_t)os;
      io.ev_cost[e0] = oc;
    }
    nev = 1;
  }
  int dec = io.decision[b];
  if (dec == 0) {
    const double *x = io.x + (size_t)b * io.n;
    const long long calls = calls_of(io, b);
    const double objval = io.obj[b];
    // reliable candidates, ascending index (:84-96): the largest score, the
    // lowest index on ties (a NaN score never wins a strict comparison)
    double rs = -INFINITY, ru = 0.0;
    int rj = INT_MAX;
    for (int j = lane; j < io.n; j += 64) {
      if (!is_int(io.vtype[j])) continue;
      const double v = x[j];
      if (!fractional(v)) continue;
      const PcView pv = pc_view(io, j, own, ov, os, oc);
      if (!reliable(io, j, calls, pv)) continue;
      const double cd = (v - floor(v)) * pv.pd, cu = (ceil(v) - v) * pv.pu;
      const double sc = rel_score(cu, cd);
      if (sc > rs) {   // lanes visit ascending j: the first maximum
        rs = sc;
        rj = j;
      }
    }
    wave_max_key(rs, ru, rj);
    double best = -INFINITY;
    int bj = -1;
    bool down_first = false;
    if (rj != INT_MAX) {
      const double v = x[rj];
      const PcView pv = pc_view(io, rj, own, ov, os, oc);
      const double cd = (v - floor(v)) * pv.pd, cu = (ceil(v) - v) * pv.pu;
      best = rs;
      bj = rj;
      down_first = cu > cd;
    }
    // strong-branched candidates (:98-128), in order
    const double maxchange = io.cutoff - objval;
    const int nsb = io.nsb[b];
    const size_t off = 2 * (size_t)io.sb_off[b];
    int status = 0;   // 0 NotModified, 1 Pruned, 2 Modified
    int mvar = -1, mup = 0;
    int ran = 0;       // candidates strong-branched (the loop stops at a verdict)
    // lane k holds candidate k's column, value and verdict (loaded together,
    // not one dependent round trip per candidate)
    int lj = 0, loc = 0;
    double lv = 0.0, lcd = 0.0, lcu = 0.0;
    if (lane < nsb) {
      lj = io.sb_var[(size_t)b * kRelMaxCands + lane];
      lv = io.sb_val[(size_t)b * kRelMaxCands + lane];
      loc = sb_outcome(io, off, lane, objval, maxchange, lcd, lcu);
    }
    for (int k = 0; k < nsb; ++k) {
      const int j = rl(lj, k);
      const double v = rld(lv, k);
      const double dd = v - floor(v), ud = ceil(v) - v;
      const double cd = rld(lcd, k), cu = rld(lcu, k);
      const int oc2 = rl(loc, k);
      ran = k + 1;
      if (oc2 < 0) {
        // an unreliable side: no verdict, no observation
      } else if (oc2 == 1) {
        status = 1;
      } else if (oc2 == 2) {
        status = 2;       // the down branch's bound change
        mvar = j;
        mup = 0;
      } else if (oc2 == 3) {
        status = 2;       // the up branch's bound change
        mvar = j;
        mup = 1;
      } else if (nev + 2 <= kRelEvents) {
        if (lane == 0) {
          io.ev_var[e0 + nev] = j;
          io.ev_side[e0 + nev] = 0;
          io.ev_cost[e0 + nev] = fabs(cd) / (fabs(dd) + kRelETol);
          io.ev_var[e0 + nev + 1] = j;
          io.ev_side[e0 + nev + 1] = 1;
          io.ev_cost[e0 + nev + 1] = fabs(cu) / (fabs(ud) + kRelETol);
        }
        nev += 2;
      }
      const double sc = rel_score(cu, cd);
      // lastStrBranched_ = calls: within the round the last writer is the
      // largest call number (pc_fold stores it)
      if (lane == 0) atomicMax(&io.last_new[j], (int)calls);
      if (status != 0) break;
      if (sc > best) {
        best = sc;
        bj = j;
        down_first = cu > cd;
      }
    }
    if (status == 0) {
      // the remaining unreliable candidates by pseudocost (:129-147), in
      // CompareScore order after the first nsb (the strong-branched ones:
      // rel_prepare chose them with the same keys): the largest score, the
      // earliest key on ties; it wins only above the best so far
      double ps = -INFINITY;
      int pj = -1;
      if (nsb > 0) {
        pj = io.sb_var[(size_t)b * kRelMaxCands + nsb - 1];
        const double v = x[pj];
        ps = unrel_score(pc_view(io, pj, own, ov, os, oc), v - floor(v), ceil(v) - v);
      }
      double us = -INFINITY, uk = INFINITY;
      int uj = INT_MAX;
      for (int j = lane; j < io.n; j += 64) {
        if (!is_int(io.vtype[j])) continue;
        const double v = x[j];
        if (!fractional(v)) continue;
        const PcView pv = pc_view(io, j, own, ov, os, oc);
        if (reliable(io, j, calls, pv)) continue;
        const double key = unrel_score(pv, v - floor(v), ceil(v) - v);
        if (!(key > ps || (key == ps && j > pj))) continue;   // strong-branched, or unordered
        const double cd = (v - floor(v)) * pv.pd, cu = (ceil(v) - v) * pv.pu;
        const double sc = rel_score(cu, cd);
        if (!(sc > -INFINITY)) continue;
        if (sc > us || (sc == us && (key < uk || (key == uk && j < uj)))) {
          us = sc;
          uk = key;
          uj = j;
        }
      }
      wave_max_key(us, uk, uj);
      if (uj != INT_MAX && us > best) {
        const double v = x[uj];
        const PcView pv = pc_view(io, uj, own, ov, os, oc);
        const double cd = (v - floor(v)) * pv.pd, cu = (ceil(v) - v) * pv.pu;
        best = us;
        bj = uj;
        down_first = cu > cd;
      }
      if (lane == 0) {
        io.bvar[b] = bj;
        io.bval[b] = x[bj];
        io.bup[b] = down_first ? 0 : 1;
      }
    } else if (status == 1) {
      dec = 1;   // PrunedByBrancher -> NodeInfeasible (PCBProcessor.cpp:284-294)
      if (lane == 0) atomicAdd(&io.counters[1], 1ull);
    } else {
      // ModifiedByBrancher: the node again with the one-sided bound change
      // (PCBProcessor.cpp:295-305); the tail writes it as a single child
      dec = 5;
      if (lane == 0) {
        io.bvar[b] = mvar;
        io.bval[b] = x[mvar];
        io.bup[b] = (int8_t)mup;
        atomicAdd(&io.counters[2], 1ull);
      }
    }
    if (ran > 0) {  // the LPs the reference solves: up to the verdict
      unsigned long long piv = lane < 2 * ran ? (unsigned long long)io.c_iters[off + lane] : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) piv += __shfl_xor(piv, o, 64);
      if (lane == 0) {
        atomicAdd(&io.counters[0], (unsigned long long)(2 * ran));
        atomicAdd(&io.counters[3], piv);
      }
    }
  }
  if (lane == 0) {
    io.dec_out[b] = dec;
    io.nev[b] = nev;
  }
}

// ---- chained strong branching (ReliabilityBrancher::strongBranch_, :469-506):
// the brancher's LPs run one after the other through the node's engine, each
// resolving from the basis the previous one left (HipLPEngine / CpuLPEngine
// keep a solve's basis when it ended optimal or at the iteration limit, and
// the one it started from otherwise; the first starts from the node's optimal
// basis), and findBestCandidate_ stops strong-branching at the first verdict
// (:111-118).  One chain slot per node, solved in steps: step s is the s-th
// LP of every node still strong-branching.

__global__ __launch_bounds__(256) void rel_chain_init(RelIO io, LpWarm w, int32_t *ch_head,
                                                      int8_t *ch_st, double *ch_d,
                                                      double *ch_binv, uint8_t *stopped, int m) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  if (lane == 0) stopped[b] = 0;
  if (io.nsb[b] == 0) return;
  const int N = io.n + m;
  const size_t mm = (size_t)m * m;
  for (int k = lane; k < m; k += 64) ch_head[(size_t)b * m + k] = w.head[b * w.s_head + k];
  for (int k = lane; k < N; k += 64) {
    ch_st[(size_t)b * N + k] = w.st[b * w.s_st + k];
    ch_d[(size_t)b * N + k] = w.d[b * w.s_d + k];
  }
  for (size_t k = lane; k < mm; k += 64) ch_binv[(size_t)b * mm + k] = w.binv[b * w.s_binv + k];
}

// step s's list; at an even step s >= 2 first the verdict of candidate
// s / 2 - 1, whose pair of LPs the two previous steps ran (findBestCandidate_
// stops strong-branching there, ReliabilityBrancher.cpp:111-118).  The
// verdict after the last pair is not needed: rel_decide stops at it itself.
__global__ __launch_bounds__(256) void rel_chain_list(RelIO io, int s, uint8_t *stopped,
                                                      int32_t *list, int32_t *count) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= io.nb) return;
  bool stop = stopped[b] != 0;
  const int c = (s >> 1) - 1;
  if (!stop && s >= 2 && (s & 1) == 0 && c < io.nsb[b]) {
    const double objval = io.obj[b];
    double cd, cu;
    if (sb_outcome(io, 2 * (size_t)io.sb_off[b], c, objval, io.cutoff - objval, cd, cu) > 0) {
      stopped[b] = 1;
      stop = true;
    }
  }
  if (stop || s >= 2 * io.nsb[b]) return;
  list[atomicAdd(count, 1)] = 2 * io.sb_off[b] + s;
}

// the round's observations packed in node order (offsets: excl_scan of nev)
__global__ __launch_bounds__(256) void rel_compact(RelIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= io.nb) return;
  const int k = io.nev[b];
  const size_t o = (size_t)io.ev_off[b];
  for (int e = 0; e < k; ++e) {
    const size_t i = (size_t)b * kRelEvents + e;
    io.cv_var[o + e] = io.ev_var[i];
    io.cv_side[o + e] = io.ev_side[i];
    io.cv_cost[o + e] = io.ev_cost[i];
  }
}

// updatePCost_ over the round's observations, per variable in node order:
// one wave per variable walks the packed list 64 at a time (one coalesced
// load, a ballot of this variable's entries, then their costs in order)
__global__ __launch_bounds__(64) void pc_fold(RelIO io) {
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  double pu = io.pc_up[j], pd = io.pc_dn[j];
  int cu = io.cnt_up[j], cd = io.cnt_dn[j];
  const int E = *io.ev_total;
  for (int c0 = 0; c0 < E; c0 += 64) {
    const int i = c0 + lane;
    const int v = i < E ? io.cv_var[i] : -1;
    const double c = i < E ? io.cv_cost[i] : 0.0;
    const int sd = i < E ? io.cv_side[i] : 0;
    uint64_t mine = __ballot(v == j);
    while (mine) {
      const int k = __builtin_ctzll(mine);
      mine &= mine - 1;
      const double x = __shfl(c, k, 64);
      if (__shfl(sd, k, 64) == 0) {
        pd = (pd * cd + x) / (cd + 1);
        cd += 1;
      } else {
        pu = (pu * cu + x) / (cu + 1);
        cu += 1;
      }
    }
  }
  if (lane == 0) {
    if (io.last_new[j] >= 0) io.last[j] = io.last_new[j];
    io.pc_up[j] = pu;
    io.pc_dn[j] = pd;
    io.cnt_up[j] = cu;
    io.cnt_dn[j] = cd;
  }
}

}  // namespace

hipError_t launch_rel_rank(const RelIO &io, int32_t *flag, int32_t *rank, int32_t *total,
                           hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_flags, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io, flag);
  hipLaunchKernelGGL(excl_scan, dim3(1), dim3(1024), 0, stream, flag, rank, io.nb, total);
  return hipGetLastError();
}

hipError_t launch_rel_prepare(const RelIO &io, int32_t *sb_off, int32_t *total,
                              hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_prepare, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  hipLaunchKernelGGL(excl_scan, dim3(1), dim3(1024), 0, stream, io.nsb, sb_off, io.nb, total);
  return hipGetLastError();
}

hipError_t launch_rel_children(const RelIO &io, const double *wlb, const double *wub,
                               double *clb, double *cub, int32_t *cnode, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_children, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io, wlb, wub,
                     clb, cub, cnode);
  return hipGetLastError();
}

hipError_t launch_rel_chain_init(const RelIO &io, const LpWarm &node_ws, int32_t *ch_head,
                                 int8_t *ch_st, double *ch_d, double *ch_binv, uint8_t *stopped,
                                 int m, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_chain_init, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io, node_ws,
                     ch_head, ch_st, ch_d, ch_binv, stopped, m);
  return hipGetLastError();
}

hipError_t launch_rel_chain_list(const RelIO &io, int s, uint8_t *stopped, int32_t *list,
                                 int32_t *count, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_chain_list, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io, s,
                     stopped, list, count);
  return hipGetLastError();
}

hipError_t launch_rel_decide(const RelIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_decide, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  hipLaunchKernelGGL(excl_scan, dim3(1), dim3(1024), 0, stream, io.nev, io.ev_off, io.nb,
                     io.ev_total);
  hipLaunchKernelGGL(rel_compact, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io);
  hipLaunchKernelGGL(pc_fold, dim3(io.n), dim3(64), 0, stream, io);
  return hipGetLastError();
}

}  // namespace mgpu

namespace mgpu {
namespace {
// per-batch parent data of the popped nodes: node bound, parent branching
// variable and value (stack: slot base + i; best-first: the selected slots)
__global__ __launch_bounds__(256) void rel_gather(int nb, int base, const uint32_t *slots,
                                                  const double *pnlb, const int32_t *ppvar,
                                                  const double *ppval, double *bnlb,
                                                  int32_t *bpvar, double *bpval) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nb) return;
  const size_t s = slots != nullptr ? (size_t)slots[i] : (size_t)base + i;
  bnlb[i] = pnlb[s];
  bpvar[i] = ppvar[s];
  bpval[i] = ppval[s];
}
}  // namespace

hipError_t launch_rel_gather(int nb, int base, const uint32_t *slots, const double *pnlb,
                             const int32_t *ppvar, const double *ppval, double *bnlb,
                             int32_t *bpvar, double *bpval, hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(rel_gather, dim3((nb + 255) / 256), dim3(256), 0, stream, nb, base, slots,
                     pnlb, ppvar, ppval, bnlb, bpvar, bpval);
  return hipGetLastError();
}
}  // namespace mgpu
