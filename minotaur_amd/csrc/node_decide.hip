// Node decision after the relaxation solve, batched: the engine-status
// switch of PCBProcessor::shouldPrune_ (src/base/PCBProcessor.cpp:400-523)
// and the integrality test of IntVarHandler::isFeasible
// (src/base/IntVarHandler.cpp:54-84), one wave per node.
//
// decision codes (mgpu.h): 0 continue/branch, 1 infeasible (FBBT, LP or
// engine error), 2 pruned by bound (NodeHitUb), 3 integer feasible (new
// incumbent candidate), 4 engine problem (unbounded / unknown status).
// Pinned against the reference's own shouldPrune_ + isFeasible
// (tests/golden/decide_*.npz, oracle/ref/ref_decide.cpp).
#include "mgpu_internal.h"
#include "wave.h"

#include <climits>

namespace mgpu {
namespace {

constexpr int kNodesPerBlock = 4;

__global__ __launch_bounds__(64 * kNodesPerBlock) void node_decide_kernel(DevLP lp,
                                                                           DecideIO io) {
  const int lane = threadIdx.x & 63;
  const int nn = io.node_list != nullptr ? *io.node_count : io.batch;
  for (int t = blockIdx.x * kNodesPerBlock + (threadIdx.x >> 6); t < nn;
       t += gridDim.x * kNodesPerBlock) {
  const int b = io.node_list != nullptr ? io.node_list[t] : t;
  const int st = io.status[b];
  const double solval = io.obj[b];
  int dec;
  double inf_meas = 0.0;
  // EngineStatus numerics (Types.h:152-166)
  const bool optimal = st == 0 || st == 1 || st == 6;   // Proven(Local)Optimal, IterationLimit
  const bool cont = st == 7 || st == 9;                 // ProvenFailedCQFeas, FailedFeas
  if (io.fbbt_infeas != nullptr && io.fbbt_infeas[b] != 0) {
    dec = 1;  // presolveNode reported infeasible: pruned before the solve
  } else if (st == 2 || st == 3 || st == 8 || st == 10 || st == 11) {
    // Proven(Local)Infeasible, ProvenFailedCQInfeas, FailedInfeas, and
    // EngineError (contOnErr_ is false in PCBProcessor, :39, :497-515)
    dec = 1;
  } else if (st == 5) {
    dec = 2;  // ProvenObjectiveCutOff -> NodeHitUb (:431-435)
  } else {
    // ProvenUnbounded (the reference asserts, :437-442) and
    // EngineUnknownStatus (no case) keep the node (shouldPrune_ false) and
    // still reach isFeasible (its inf_meas is reported), decision 4
    const bool engine = !(optimal || cont);
    const double cut = io.incumbent;
    if (optimal && (solval >= cut - io.abs_tol || solval >= cut - fabs(cut) * io.rel_tol ||
                    solval >= io.cutoff)) {
      dec = 2;  // :486-491
    } else {
      // IntVarHandler::isFeasible over Binary/Integer columns.  inf_meas is
      // accumulated in column order as the reference's loop does (:64-79):
      // each lane holds one column's violation (0 when integral), the wave
      // adds them lane by lane through v_readlane, so the sum is the
      // reference's sequential sum bit for bit (adding +0.0 is exact).
      const double *x = io.x + (size_t)b * lp.n;
      bool frac = false;
      for (int j0 = 0; j0 < lp.n; j0 += 64) {
        const int j = j0 + lane;
        double f = 0.0;
        if (j < lp.n) {
          const uint8_t t = lp.vtype[j];
          if (t == kBinary || t == kInteger) {
            const double v = x[j];
            const double g = fabs(v - floor(v + 0.5));
            if (g > io.int_tol) f = g;
          }
        }
        frac |= f > 0.0;
        const int cnt = lp.n - j0 < 64 ? lp.n - j0 : 64;
        for (int k = 0; k < cnt; ++k) inf_meas += rld(f, k);
      }
      dec = engine ? 4 : __any(frac) ? 0 : 3;
      if (dec == 0 && io.bvar != nullptr) {
        // MaxVioBrancher::findBestCandidate_ (MaxVioBrancher.cpp) over the
        // IntVarHandler candidates (IntVarHandler.cpp:86-108): score
        // 0.1 * (0.8 min(dd, ud) + 0.2 max(dd, ud)) (VarOrig), largest
        // wins, ties -> lowest index (candidate set ordered by index);
        // up branch first when dd > ud.
        double best = -INFINITY;
        int bj = INT_MAX;
        for (int j = lane; j < lp.n; j += 64) {
          const uint8_t t = lp.vtype[j];
          if (t != kBinary && t != kInteger) continue;
          const double v = x[j];
          if (!(fabs(floor(v + 0.5) - v) > io.int_tol)) continue;
          const double dd = v - floor(v), ud = ceil(v) - v;
          const double lo = (ud < dd) ? ud : dd, hi = (dd < ud) ? ud : dd;
          const double sc = 0.1 * (0.8 * lo + 0.2 * hi);
          if (sc > best) {
            best = sc;
            bj = j;
          }
        }
        wave_argmax(best, bj);
        if (lane == 0) {
          const double v = x[bj];
          io.bvar[b] = bj;
          io.bval[b] = v;
          io.bup[b] = (v - floor(v)) > (ceil(v) - v) ? 1 : 0;
        }
      }
    }
  }
  if (lane == 0) {
    io.decision[b] = dec;
    if (io.inf_meas != nullptr) io.inf_meas[b] = inf_meas;
    if (io.cand_obj != nullptr) io.cand_obj[b] = dec == 3 ? solval : INFINITY;
  }
  }
}

}  // namespace

hipError_t launch_node_decide(const DevLP &lp, const DecideIO &io, hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  int blocks = (io.batch + kNodesPerBlock - 1) / kNodesPerBlock;
  // list mode: the count is on the device; a grid-stride loop over it
  if (io.node_list != nullptr && blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(node_decide_kernel, dim3(blocks), dim3(64 * kNodesPerBlock), 0, stream,
                     lp, io);
  return hipGetLastError();
}

}  // namespace mgpu
