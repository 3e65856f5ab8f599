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
  const int32_t *status, *iters;
  const double *obj, *x;        // [nb], [nb][nv]
  double *cand;                 // [nb][4][nv] scratch
  int32_t *dec, *bvar, *pos, *depth_in;
  double *bval;
  int8_t *bup, *bint;
  GlobOut *out;
  // the pool (stack): children go to base + pos
  double *plb, *pub, *prows, *pnlb;
  int32_t *pdepth;
};

hipError_t launch_glob_round_tail(const GlobIO &io, hipStream_t stream);

}  // namespace mgpu
