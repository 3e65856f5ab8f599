// Device-side structures of the batched branch-and-bound step (bnb.hip).
#pragma once

#include "mgpu_internal.h"

namespace mgpu {

struct BnbOut {                 // per round, device -> host
  long long ndec[5];            // decision counts (mgpu.h decision codes)
  long long lps, pivots;        // LPs solved (not pruned by FBBT) and their pivots
  int nbranched;                // nodes with decision 0 (2 children each)
  int best_idx;                 // batch index of the best integer-feasible node, -1 none
  double best;                  // its objective (+inf none)
};

struct BnbIO {
  int nb;                       // nodes popped this round
  int base;                     // pool slot of the first popped node (stack mode)
  // best-first mode (slots != null): the pool is a slot array with free
  // slots; child c of the round goes to free slot F(c): the slots just
  // selected (slots[0, nb), in selection order), then the earlier holes
  // (slots[live, hw) of the sorted array: ascending), then new slots hw, ...
  const uint32_t *slots;        // [hw] slot ids sorted by (bound, slot)
  int live, hw;                 // live nodes before the selection, high-water mark
  uint8_t *plive;               // [cap] slot holds an open node
  // parent warm starts (ws_head != null): the node's optimal basis (the LP's
  // warm start out, batch-indexed) is copied to both children's slots
  int m, N;
  const int32_t *wo_head;
  const int8_t *wo_st;
  const double *wo_d, *wo_binv;
  int32_t *ws_head;             // [cap][m]
  int8_t *ws_st;                // [cap][N]
  double *ws_d, *ws_binv;       // [cap][N], [cap][m][m]
  const int32_t *decision;      // [nb]
  const int32_t *status;        // [nb] LP status (12 = not solved: FBBT-infeasible)
  const int32_t *iters;         // [nb] LP pivots
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

// Best-first selection (bnb_select.hip): gather of the selected nodes.
struct BnbSelIO {
  int nb, n, m, N;
  const uint32_t *slots;        // [nb] selected pool slots
  const double *plb, *pub;      // pool boxes [cap][n]
  const int32_t *pdepth;
  uint8_t *plive;
  double *wlb, *wub;            // [nb][n] batch boxes
  int32_t *depth_in;            // [nb]
  const int32_t *ws_head;       // pool bases (null: root warm start)
  const int8_t *ws_st;
  const double *ws_d, *ws_binv;
  int32_t *bws_head;            // [nb] batch bases
  int8_t *bws_st;
  double *bws_d, *bws_binv;
};

hipError_t launch_bnb_tail(const BnbIO &io, int n, hipStream_t stream);
hipError_t launch_bnb_keys(const double *pnlb, uint8_t *plive, int hw, double cutoff, double ub,
                           uint64_t *keys, uint32_t *vals, int32_t *counts, hipStream_t stream);
hipError_t bnb_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *keys_in,
                          uint64_t *keys_out, const uint32_t *vals_in, uint32_t *vals_out,
                          int count, hipStream_t stream);
hipError_t launch_bnb_gather(const BnbSelIO &io, hipStream_t stream);
hipError_t launch_sb_boxes(const double *plb, const double *pub, const int32_t *var,
                           const double *val, int ncand, int n, double *clb, double *cub,
                           hipStream_t stream);
hipError_t launch_bnb_shard(double *plb, double *pub, double *pnlb, int32_t *pdep, double *tlb,
                            double *tub, double *tnlb, int32_t *tdep, int count, int n,
                            int rank, int world, int *kept, hipStream_t stream);

}  // namespace mgpu
