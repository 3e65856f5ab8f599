// Device-side structures of the batched branch-and-bound step (bnb.hip).
#pragma once

#include "mgpu_internal.h"

namespace mgpu {

struct BnbOut {                 // per round, device -> host
  long long ndec[5];            // decision counts (mgpu.h decision codes)
  long long lps, pivots;        // LPs solved (not pruned by FBBT) and their pivots
  long long pfi_pivots;         // of those, run by the product-form kernel (<= pfi_cap per LP)
  int nchild;                   // children written (2 per decision 0, 1 per decision 5)
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
  // reference-heap mode: the slot of child c is child_slots[c] (assigned on
  // the host); defer_children: the tail runs the scans only, the children
  // writer follows once the host has assigned the slots
  const int32_t *child_slots;
  int defer_children;
  uint8_t *plive;               // [cap] slot holds an open node
  // parent warm starts (ws_head != null): the node's optimal basis (the LP's
  // warm start out, batch-indexed) is copied to both children's slots
  int m, N;
  const int32_t *wo_head;
  const int8_t *wo_st;
  const double *wo_d, *wo_binv;
  // a node modified by the brancher (decision 5) is solved again from the
  // basis its strong branching left (the chain slot, batch-indexed; null:
  // wo_*)
  const int32_t *mo_head;
  const int8_t *mo_st;
  const double *mo_d, *mo_binv;
  int32_t *ws_head;             // [cap][m]
  int8_t *ws_st;                // [cap][N]
  double *ws_d, *ws_binv;       // [cap][N], [cap][m][m]
  // path warm starts (opk != null): the node's final path (batch-indexed)
  // is copied to both children's slots
  const int32_t *opk;           // [nb]
  const uint32_t *oppath;       // [nb][kPathMax]
  const int8_t *opst;           // [nb][N]
  int32_t *ppk;                 // [cap]
  uint32_t *ppath;              // [cap][kPathMax]
  int8_t *ppst;                 // [cap][N]
  const int32_t *decision;      // [nb] (5: one child with the bound change bvar/bval/bup)
  int32_t *ppvar;               // [cap] or null: the children's parent branching variable
  double *ppval;                //   and its value (reliability branching's pseudocosts)
  const int32_t *status;        // [nb] LP status (12 = not solved: FBBT-infeasible)
  const int32_t *iters;         // [nb] LP pivots
  int pfi_cap;                  // product-form eta cap of the round's LP call (0: dense)
  const unsigned long long *pfi_piv;   // K3P's pivot counter of that call (null: none)
  const int32_t *kin;           // warm 2: each node's warm-start eta count (batch-indexed)
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
  int32_t *bcnt;                // [nblk][8]
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
  const int32_t *pk;            // pool paths (null: none)
  const uint32_t *ppath;
  const int8_t *pst;
  int32_t *bpk;                 // [nb] batch paths
  uint32_t *bppath;
  int8_t *bpst;
};

// Batched reliability branching (bnb_rel.hip).  ReliabilityBrancher
// defaults (ReliabilityBrancher.cpp:43-58): maxStrongCands_ 20,
// maxIterations_ 25, thresh_ 4, minNodeDist_ 50, eTol_ 1e-6, trustCutoff_.
constexpr int kRelMaxCands = 20;
constexpr int kRelIterLimit = 25;
constexpr int kRelThresh = 4;
constexpr int kRelMinDist = 50;
constexpr double kRelETol = 1e-6;
constexpr int kRelMaxDepth = 1000;   // maxDepth_: deeper nodes are not strong-branched (:105)
constexpr int kRelEvents = 1 + 2 * kRelMaxCands;   // pseudocost observations per node
static_assert(2 * kRelMaxCands <= 64, "rel_decide: one lane per strong-branching LP");
struct RelIO {
  int nb, n;
  const uint8_t *vtype;         // [n]
  const int32_t *decision;      // [nb] node_decide's decisions
  const double *x, *obj;        // [nb][n], [nb] node LP solution
  const double *nlb;            // [nb] node bound (the parent's LP value)
  const int32_t *depth;         // [nb] node depth (Node::getDepth)
  const int32_t *pvar;          // [nb] parent's branching variable (-1: none)
  const double *pval;           // [nb] its value in the parent's LP solution
  double *pc_up, *pc_dn;        // [n] pseudocosts (pseudoUp_ / pseudoDown_)
  int32_t *cnt_up, *cnt_dn;     // [n] timesUp_ / timesDown_
  int32_t *last;                // [n] lastStrBranched_
  int32_t *last_new;            // [n] this round's last writer (-1 none): the largest
                                //   call number that strong-branched the variable
  long long calls0;             // findBranches calls before this round
  int32_t *rank;                // [nb] rank among the round's branching nodes
  double cutoff;                // incumbent value (s_pool best, +inf none)
  int32_t *nsb;                 // [nb] strong-branched candidates
  int32_t *sb_var;              // [nb][kRelMaxCands]
  double *sb_val;
  int32_t *sb_off;              // [nb] exclusive prefix of nsb
  const int32_t *c_status;      // strong-branching LPs [2 * total]: down, up per candidate
  const double *c_obj;
  const int32_t *c_iters;
  int32_t *dec_out;             // [nb] 0 branch, 1 pruned by brancher, 5 modified, else as in
  int32_t *bvar;                // [nb] choice (decision 0) / bound change (decision 5)
  double *bval;
  int8_t *bup;                  // 1: up branch first / the up branch's bound change
  int32_t *nev;                 // [nb] observations
  int32_t *ev_var;              // [nb][kRelEvents]
  int8_t *ev_side;              // 0 down, 1 up
  double *ev_cost;
  int32_t *ev_off;              // [nb] packed offsets of the nodes' observations
  int32_t *ev_total;            // device: number of observations
  int32_t *cv_var;              // packed observations [nb * kRelEvents] in node order
  int8_t *cv_side;
  double *cv_cost;
  unsigned long long *counters; // [4] strong-branching LPs, pruned, modified, their pivots
  int32_t *nsb_max;             // device: the round's largest nsb (rel_prepare)
};
// Chained strong branching: the nodes' chain slots (one warm start per node)
// start as the node's optimal basis; step s solves the s-th strong-branching
// LP of every node still strong-branching, from and back into its slot.
hipError_t launch_rel_chain_init(const RelIO &io, const LpWarm &node_ws, int32_t *ch_head,
                                 int8_t *ch_st, double *ch_d, double *ch_binv, uint8_t *stopped,
                                 int m, hipStream_t stream);
hipError_t launch_rel_chain_list(const RelIO &io, int s, uint8_t *stopped, int32_t *list,
                                 int32_t *count, hipStream_t stream);
hipError_t launch_rel_rank(const RelIO &io, int32_t *flag, int32_t *rank, int32_t *total,
                           hipStream_t stream);
hipError_t launch_rel_prepare(const RelIO &io, int32_t *sb_off, int32_t *total,
                              hipStream_t stream);
hipError_t launch_rel_children(const RelIO &io, const double *wlb, const double *wub,
                               double *clb, double *cub, int32_t *cnode, hipStream_t stream);
hipError_t launch_rel_decide(const RelIO &io, hipStream_t stream);
hipError_t launch_rel_gather(int nb, int base, const uint32_t *slots, const double *pnlb,
                             const int32_t *ppvar, const double *ppval, double *bnlb,
                             int32_t *bpvar, double *bpval, hipStream_t stream);

hipError_t launch_bnb_tail(const BnbIO &io, int n, hipStream_t stream);
hipError_t launch_bnb_children(const BnbIO &io, int n, hipStream_t stream);
hipError_t launch_bnb_keys(const double *pnlb, uint8_t *plive, int hw, double cutoff, double ub,
                           uint64_t *keys, uint32_t *vals, int32_t *counts, hipStream_t stream);
hipError_t bnb_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *keys_in,
                          uint64_t *keys_out, const uint32_t *vals_in, uint32_t *vals_out,
                          int count, hipStream_t stream);
hipError_t launch_bnb_gather(const BnbSelIO &io, hipStream_t stream);
hipError_t launch_sb_boxes(const double *plb, const double *pub, const int32_t *var,
                           const double *val, int ncand, int n, double *clb, double *cub,
                           hipStream_t stream);
hipError_t launch_bnb_shard_rows(unsigned char *rows, unsigned char *tmp, size_t row_bytes,
                                 int kept, int rank, int world, hipStream_t stream);
hipError_t launch_bnb_shard(double *plb, double *pub, double *pnlb, int32_t *pdep, double *tlb,
                            double *tub, double *tnlb, int32_t *tdep, int count, int n,
                            int rank, int world, int *kept, hipStream_t stream);

// Node migration (bnb_migrate.hip): packed rows [lb n | ub n | bound | depth]
// into pool slots, per-node state reset for a migrated node.
struct MigratePack {            // pool slots -> rows (bnb_pack)
  int k, n, N, W;               // W: row width in doubles (mig_width)
  const int32_t *slots;         // [k] source pool slots
  const double *plb, *pub, *pnlb;
  const int32_t *pdepth;
  uint8_t *plive;               // best-first: the slot is freed (null: stack)
  const int32_t *ppk;           // warm mode 2 (null: rows without a basis)
  const uint32_t *ppath;
  const int8_t *ppst;
  double *buf;                  // [k][W]
};
struct MigrateIO {
  int k, n, m, N, W;
  const int32_t *slots;         // [k] destination pool slots
  const double *buf;            // [k][W]
  double *plb, *pub, *pnlb;
  int32_t *pdepth;
  uint8_t *plive;               // best-first pool flags (null: stack)
  int32_t *ppvar;               // reliability: parent branching variable (null: none)
  int32_t *ppk;                 // warm mode 2: the rows' bases (null: none)
  uint32_t *ppath;
  int8_t *ppst;
  int32_t *ws_head;             // parent warm starts (null: none) <- the root basis r_*
  int8_t *ws_st;
  double *ws_d, *ws_binv;
  const int32_t *r_head;
  const int8_t *r_st;
  const double *r_d, *r_binv;
};
hipError_t launch_bnb_pack(const MigratePack &io, hipStream_t stream);
hipError_t launch_bnb_unpack(const MigrateIO &io, hipStream_t stream);
hipError_t launch_bnb_move_rows(unsigned char *rows, unsigned char *tmp, size_t row_bytes,
                                const int32_t *from, const int32_t *to, int k,
                                hipStream_t stream);
// dst row t = src row from[t] (device index array), rows of row_bytes
hipError_t launch_bnb_gather_rows(const unsigned char *src, unsigned char *dst, size_t row_bytes,
                                  const int32_t *from, int k, hipStream_t stream);

}  // namespace mgpu
