// Device-side structures of the batched spatial B&B (glob_tree.hip).
#pragma once

#include "mgpu_internal.h"

namespace mgpu {

struct GlobOut {                // per round, device -> host
  long long ndec[6];            // mgpu_glob_stats decision codes
  long long lps, pivots;        // LPs solved (not pruned by K2) and their pivots
  long long br_int;             // branchings at floor / ceil (IntVarHandler)
  int nchild;                   // children written
  int best_idx;                 // batch index of the best feasible node, -1 none
  double best;
};

struct GlobIO {
  int nb, base, nv, R;
  // problem: variable types, registries, original functions (function ncon
  // is the objective when it has one; nfun = ncon + has_obj)
  const uint8_t *vtype;         // [nv]
  int nsq, nbil, ncon, nfun;
  const int32_t *sq;            // [nsq][2] x, y
  const int32_t *bil;           // [nbil][3] x0, x1, y
  const int32_t *lptr, *lvar, *qptr, *qv1, *qv2;
  const double *lval, *qval, *clb, *cub;
  double obj_const;
  double inc, abs_tol, rel_tol;
  // the round: K2 verdicts, tightened boxes and rows, LP results
  const int32_t *kinf;          // [nb] K2 infeasible (1) / failure (2, 3)
  const double *wlb, *wub;      // [nb][nv]
  const double *wrows;          // [nb][R]
  int32_t *status, *iters;      // (the separation loop merges re-solves in)
  double *obj, *x;              // [nb], [nb][nv]
  double *cand;                 // [nb][4][nv] scratch
  int32_t *dec, *bvar, *pos, *depth_in;
  double *bval;
  int8_t *bup, *bint;
  GlobOut *out;
  // the pool (stack): children go to base + pos
  double *plb, *pub, *prows, *pnlb;
  int32_t *pdepth;
  // tangent cuts of the squares (QuadHandler::separate): S slots per square,
  // T = 2 nsq S record values [2 xl, xl^2] (inactive [0, +inf]) after the R
  // row-state values of the node record wvals [nb][R + T]; pool copy ptan
  // [cap][T].  The separation loop re-solves the flagged nodes into st2 /
  // obj2 / it2 / x2 and merges them back.
  int S, T;
  double *wvals, *ptan;
  int32_t *flag, *skip2;
  const int32_t *st2, *it2;
  const double *obj2, *x2;
  unsigned long long *acc;      // [2] tangent cuts, re-solved nodes (this pass)
  const int32_t *only;          // glob_decide: only the nodes with only[b] != 0
  // the round's input nodes: depth [nb] and tangent slots [nb][T] (stack
  // order: the pool at base; reference order: gathered from pool slots)
  const int32_t *in_depth;
  const double *in_tan;
  // reference order (mgpu_glob_config order 2): the pool slots of the round
  // (gather) and of the children (2 per branched node at pos: down, up)
  const int32_t *sel, *child_slots;
  double *glb, *gub, *grows, *gtan;   // gathered boxes, rows, tangent slots
  int32_t *gdepth;
  // parent-basis warm starts (warm 1): per pool slot the parent's optimal
  // basis (head [m], statuses [n+m], has-basis flag); gathered per node;
  // the round's optimal bases (wo) go to the children
  int m, N;
  int32_t *pws_head, *ghead;
  int8_t *pws_st, *gst;
  uint8_t *pws_ok, *gok;
  const int32_t *wo_head;
  const int8_t *wo_st;
  int32_t *skip_a;              // kinf or no basis: the warm call skips the node
  // LinearHandler::presolveNode on the node's relaxation (mgpu_glob_config
  // lin 1; glob_linear): the M rows of the relaxation as a term table, rows
  // ascending, each row's terms ascending by variable.  A term's weight is
  // ltval (ltsrc < 0) or the node record's value ltsrc (< R: the rows frows,
  // else the tangent slots ftan); a row's upper side likewise (lrhsrc).
  // Column incidence lcptr / lcterm (term indices).  Objective loidx /
  // loval; has_inc: the incumbent bound inc_ub = incumbent - constant.
  int M, nobj, cons_bad, has_inc;
  double inc_ub;
  const int32_t *lrptr, *ltvar, *ltsrc, *ltrow, *lrhsrc, *lcptr, *lcterm, *loidx;
  const double *ltval, *lrlo, *lrhi, *loval;
  const double *flb_in, *fub_in, *frows, *ftan;   // the round's nodes as they come
  double *flb, *fub;            // [nb][nv] the presolved boxes (K2's input)
  int32_t *finf;                // [nb] checkBounds_ found the node infeasible
  uint8_t *fflag;               // [nb][M] the rows' BFlag
};

hipError_t launch_glob_round_tail(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_decide(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_pack(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_separate(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_merge(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_gather(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_skips(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_summary(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_children(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_linear(const GlobIO &io, hipStream_t stream);
hipError_t launch_glob_linear_verdict(const GlobIO &io, hipStream_t stream);

}  // namespace mgpu
