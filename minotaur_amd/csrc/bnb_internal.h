// Device-side structures of the batched branch-and-bound step (bnb.hip).
#pragma once

#include "mgpu_internal.h"

namespace mgpu {

struct BnbOut {                 // per round, device -> host
  long long ndec[5];            // decision counts (mgpu.h decision codes)
  int nbranched;                // nodes with decision 0 (2 children each)
  int best_idx;                 // batch index of the best integer-feasible node, -1 none
  double best;                  // its objective (+inf none)
};

struct BnbIO {
  int nb;                       // nodes popped this round
  int base;                     // pool slot of the first popped node
  const int32_t *decision;      // [nb]
  const double *cand_obj;       // [nb]
  const double *obj;            // [nb] relaxation values (children's bound)
  const int32_t *bvar;          // [nb]
  const double *bval;
  const int8_t *bup;
  const double *wlb, *wub;      // [nb][n] FBBT-tightened boxes of the popped nodes
  int32_t *depth_in;            // [nb] depth of the popped nodes (copied first)
  double *plb, *pub;            // pool [cap][n]
  double *pnlb;                 // pool lower bounds [cap]
  int32_t *pdepth;              // pool depths [cap]
  int32_t *pos;                 // [nb] in-block exclusive prefix
  int32_t *bsum, *bidx, *boff;  // [nblk]
  double *bmin;                 // [nblk]
  int32_t *bcnt;                // [nblk][5]
  BnbOut *out;
};

hipError_t launch_bnb_tail(const BnbIO &io, int n, hipStream_t stream);
hipError_t launch_sb_boxes(const double *plb, const double *pub, const int32_t *var,
                           const double *val, int ncand, int n, double *clb, double *cub,
                           hipStream_t stream);
hipError_t launch_bnb_shard(double *plb, double *pub, double *pnlb, int32_t *pdep, double *tlb,
                            double *tub, double *tnlb, int32_t *tdep, int count, int n,
                            int rank, int world, int *kept, hipStream_t stream);

}  // namespace mgpu
