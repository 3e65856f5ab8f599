// Internal device-side data layout of the engine (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgpu {

// Tolerances of LinearHandler (LinearHandler.cpp:56-58): intTol_, eTol_,
// infty_.  Bit-identical constants in every kernel.
constexpr double kIntTol = 1e-6;
constexpr double kETol = 1e-8;
constexpr double kInfty = 1e20;

// Reference VariableType numerics (Types.h:83-89).
constexpr int kBinary = 0;
constexpr int kInteger = 1;

// One row term: coefficient + column, packed to 16 B so a wave-uniform term
// is one scalar dwordx4 load.
struct alignas(16) Term {
  double a;
  int32_t j;
  int32_t pad;
};

// Wave-uniform row/term records for the FBBT kernel.  A wave loads up to 64
// of them with ONE coalesced vector load (lane t holds record t) and
// broadcasts record k with v_readlane into SGPRs: no scalar-memory loads in
// the inner loops (SMEM and LDS share lgkmcnt, so mixing them serialises).
struct alignas(16) RowRec {   // 32 B
  double lo, hi;              // row bounds
  int32_t k0, nt;             // first term, term count
  int32_t pad0, pad1;
};
struct alignas(16) TermRec {  // 32 B; a, j, isint in the first 16 B (one read in a row visit)
  double a;                   // coefficient (0 for the integer-column list)
  int32_t j;                  // column
  int32_t isint;              // column is Binary/Integer
  uint64_t cmask;             // rows holding column j (bitmask, m <= 64)
  int32_t cs, ce;             // CSC range of column j (m > 64)
};

// Batch-shared linear relaxation, resident in HBM after mgpu_load_lp.
struct DevLP {
  int n, m, nnz, nobj;
  int cons_bad;                 // checkBounds_ row test (LinearHandler.cpp:350-357)
  const int32_t *rowptr;        // [m+1]
  const Term *terms;            // [nnz] row-major, columns ascending
  const double *rlo, *rhi;      // [m]
  const int32_t *colptr;        // [n+1]  column -> rows (changeBFlag_)
  const int32_t *rowidx;        // [nnz]
  const uint8_t *vtype;         // [n]
  const Term *obj;              // [nobj] nonzero objective terms, ascending
  const double *collb, *colub;  // [n] root box
  const double *objd;           // [n] dense objective
  double objoff;
  const RowRec *rows;           // [m]
  const TermRec *trec;          // [nnz] row terms
  const TermRec *orec;          // [nobj] objective terms
  const TermRec *irec;          // [nint] integer columns (tightenInts_)
  int nint;
  const int32_t *ccont;         // [ncont] the other columns, ascending
  int ncont;
  const double *cval;           // [nnz] CSC values (column order of colptr/rowidx)
  const int32_t *ccol;          // [nnz] CSR column indices
  const double *rval;           // [nnz] CSR values
};

// Warm start of the LP kernel (one basis per node, or one shared basis when
// the strides are 0): basic column per row, status of every column
// (0 at lb, 1 at ub, 2 free, 3 basic), reduced costs, dense basis inverse.
struct LpWarm {
  const int32_t *head;
  const int8_t *st;
  const double *d;
  const double *binv;
  long s_head, s_st, s_d, s_binv;   // per-node strides in elements (0 = shared)
};

// Per-node rows (the glob path: QuadHandler::upSqCon_/upBilCon_ rewrite the
// secant and McCormick rows at every node, QuadHandler.cpp:3322-3419, and
// OsiLPEngine::changeConstraint hands them to the LP, OsiLPEngine.cpp:
// 206-243).  The sparsity pattern is the loaded one; node b overrides the
// values of `ncoef` matrix entries and the bounds of `nrow` rows from its
// value record vals[b * stride ...] (e.g. K2's row state, zero-copy).
struct NodeRowsIO {
  const double *vals;           // [B][stride]; null = no per-node rows
  long stride;
  int ncoef;
  const int32_t *csc_pos;       // [ncoef] entry position in the CSC arrays
  const int32_t *csr_pos;       // [ncoef] entry position in the CSR arrays
  const int32_t *coef_src;      // [ncoef] offset in a node record
  int nrow;
  const int32_t *row;           // [nrow] row index
  const int32_t *lo_src;        // [nrow] offset of the row's lower bound, -1 = loaded
  const int32_t *hi_src;        // [nrow] offset of the row's upper bound, -1 = loaded
  // K3L (m > 64): per-workgroup scratch in HBM for the node's matrix values
  // and row bounds and, for a warm start given without an inverse, the
  // basis matrix of the in-kernel refactorisation: wg + blockIdx.x * wg_stride
  double *wg;
  long wg_stride;               // doubles per workgroup: 2 nnz + 2 m + m m
  const double *binv0;          // K3L: the warm basis' inverse for the loaded
                                // matrix ([m][m] column-major, shared) or null
};
// LinearFunction::addTerm keeps only |a| > 1e-9 (LinearFunction.cpp:22,
// 89-95): a smaller node coefficient is the term's absence, i.e. 0.
constexpr double kLfTol = 1e-9;

struct LpIO {
  int batch;
  NodeRowsIO nr;                // K3 only: per-node matrix values / row bounds
  const double *lb, *ub;        // [B][n] node boxes
  long box_stride;              // elements between boxes (n; 0 = one shared box)
  const int32_t *obj_col;       // [B] or null: LP b minimises obj_sign[b] * x[obj_col[b]]
  const double *obj_sign;       //   (bound LPs, QuadHandler::tightenLP_)
  const int32_t *skip;          // [B] nonzero = node already infeasible (FBBT)
  LpWarm ws;                    // ws.head == nullptr: slack basis
  const int32_t *ws_index;      // [B] or null: LP b starts from warm start ws_index[b]
                                //   (strong-branching children -> their node's basis)
  int iter_limit;
  int32_t *status;              // [B] EngineStatus numerics
  double *obj;                  // [B] objective incl. constant
  int32_t *iters;               // [B]
  double *x;                    // [B][n] primal (optional)
  int32_t *wo_head;             // [B][m]  warm start out (optional)
  int8_t *wo_st;                // [B][n+m]
  double *wo_d;                 // [B][n+m]
  double *wo_binv;              // [B][m][m]
  double *rc;                   // [B][n+m] reduced costs out, 0 for basic columns (optional)
  const int32_t *wo_index;      // [B] or null: LP b's warm start out goes to row wo_index[b]
                                //   (chained strong branching: in place, the node's slot)
  // K3 and K3L: solve just the nodes node_list[list_lo .. min(*node_count,
  // list_hi)) (device memory; the overflow list of K3P / K3PW), null = every node
  // of the batch.  list_ws: the per-node warm start is indexed by list
  // position (K3P's continuation slots), not by node.  iter_base is added to
  // the reported iteration counts (the pivots K3P already made).
  const int32_t *node_list;
  const int32_t *node_count;
  int list_lo, list_hi, list_ws, iter_base;
  // per list position: the pivots already made (K3P's continuation slots;
  // null = iter_base); the iteration limit and the Bland switch count them
  const int32_t *iter_base_list;
  int32_t *next;                // K3L: zeroed device node counter (dynamic schedule) or null
  // K3 only: next[1] counts exited waves; the last one zeroes next[0..1],
  // so the counter needs no fill before the next launch (null: not used)
  int32_t *next_exit;
  // Path warm starts (K3P only; path.k == null: none).  Node b starts from
  // the shared warm start (the root basis) after its k[b] pivots path[b]
  // (entering column | row << 16, stride kPathMax) with column statuses
  // st[b][n+m]; k[b] <= 0 = the shared warm start itself.  Out (optional):
  // the node's final path for its children, k_out 0 = restart from the root
  // (not optimal in the product form, or longer than `inherit` pivots).
  struct {
    const int32_t *k;
    const uint32_t *path;
    const int8_t *st;
    int32_t *k_out;
    uint32_t *path_out;
    int8_t *st_out;
    int inherit;
  } path;
  // Chained LPs (K3 only; chain_n == null: none), ReliabilityBrancher::
  // strongBranch_ through one engine (:469-506): unit u of the batch is node
  // u, whose LPs 2 chain_off[u] .. 2 (chain_off[u] + chain_n[u]) - 1 (down,
  // up per candidate) run one after the other in ONE wave, each from the
  // warm start the previous optimal / iteration-limited one left (ws_index /
  // wo_index: the node's chain slot); after each pair the verdict of
  // sb_verdict against the node's value chain_nobj[u] and the incumbent
  // chain_cutoff ends the chain (findBestCandidate_, :111-118).
  const int32_t *chain_off, *chain_n;
  const double *chain_nobj;
  double chain_cutoff;
};
constexpr int kPathMax = 32;    // pivots per path warm start (MGPU_PATH_MAX)
constexpr int kPathInherit = 32; // longest basis difference the batched tree hands to children (= the eta cap: profiles/r04q)

// K1: waves per CU a batch too small for one node per lane is spread over
// (tuned on config 2's complete tree, tools/tree_probe.py)
constexpr int kFbbtSmallWaves = 8;
// K1G is the auto choice up to this many nodes (mgpu_fbbt_dev), with
// kFbbtGroupG lanes per node
constexpr int kFbbtGroupMax = 65536;
constexpr int kFbbtGroupG = 16;
constexpr int kLpWaves = 4;     // nodes (waves) per workgroup
constexpr int kLpMaxM = 64;     // basis rows held one per lane in VGPRs
constexpr int kLpDefaultIterLimit = 10000;  // OsiLPEngine maxIterLimit_ (OsiLPEngine.cpp:99)
// Anti-cycling: a solve that has made this many pivots (counted across the
// product-form / dense continuation split) switches to Bland's rule — the
// infeasible row with the lowest basic column, the exact minimum ratio with
// the lowest column on ties (oracle/lp_dual.c STALL_PIVOTS).  Degenerate
// deep-tree node LPs otherwise cycle to the iteration limit.
constexpr int kStallPivots = 128;

// K3P (lp_pfi.hip): product-form dual simplex for a batch that shares its
// warm start.  At most kPfiMax eta columns per node, n + m <= 64*kPfiSlots.
constexpr int kPfiMax = 32;   // the default cap (the headline's 32-eta build)
constexpr int kPfiBig = 48;   // the largest cap: the 48-eta build (narrow tree rounds)
static_assert(kPfiBig < kStallPivots, "K3P never reaches the Bland switch");
constexpr int kPfiSlots = 4;
struct DecideIO {
  int batch;
  const int32_t *fbbt_infeas;   // [B] or null
  const int32_t *status;        // [B] LP status
  const double *obj;            // [B]
  const double *x;              // [B][n]
  double incumbent;             // best known objective (+inf if none)
  double abs_tol, rel_tol;      // solAbs_tol / solRel_tol (1e-6)
  double cutoff;                // obj_cut_off (+inf)
  double int_tol;               // int_tol (1e-6)
  int32_t *decision;            // [B]
  double *inf_meas;             // [B] or null
  double *cand_obj;             // [B] or null: obj if integer feasible else +inf
  int32_t *bvar;                // [B] or null: branching variable when decision 0
  double *bval;                 // [B] its LP value
  int8_t *bup;                  // [B] 1: up branch preferred (dd > ud)
  // list mode (node_list != null): decide only nodes node_list[i], i <
  // *node_count (device count), e.g. the product form's overflow list
  const int32_t *node_list;
  const int32_t *node_count;
};
struct PfiIO {
  int kmax;                     // eta-file cap for this launch (1..kPfiBig)
  int32_t *ovf_list;            // [B] nodes that needed more than kmax pivots
  int32_t *ovf_count;           // device counter, zeroed before the launch
  int32_t *next;                // device node counter (dynamic schedule), zeroed
  // continuation state of overflow slot i < ovf_cap (K3 goes on from it):
  // basis head [m], column status [n+m], reduced costs [n+m], explicit
  // B^-1 = E...E B0^-1 [m][m] column-major
  int ovf_cap;
  int32_t *c_iters;             // [slot] the node's own pivots at the overflow
  int32_t *c_head;
  int8_t *c_st;
  double *c_d, *c_binv;
  // B0^{-1} a_q of every column q of [A -I], column-major [N][m]: computed
  // once per launch by launch_pfi_t0 with ftran_b0's arithmetic, so every
  // FTRAN through B0^{-1} (the warm start's column replacements, each
  // pivot's entering column) is one coalesced load (null: computed in place)
  const double *t0;
  // pivots the product-form kernel ran itself, summed over the launch (K3P;
  // null: not counted): the dense continuation's pivots are not in it
  unsigned long long *pivots;
  // decide != 0 (K3P): the node decision of node_decide (shouldPrune_ +
  // isFeasible + MaxVio) in the kernel's epilogue, on the primal values in
  // LDS, for every node that does not overflow; x is then written only for
  // integer-feasible nodes (the incumbent candidates).  The overflow list is
  // decided after its dense continuation (launch_node_decide, list mode).
  int decide;
  DecideIO dec;
};
// B0^{-1} a_q for every column into t0 [N][m] (K3P's ftran_b0, bit for bit)
hipError_t launch_pfi_t0(const DevLP &lp, const double *binv, double *t0, hipStream_t stream);
// continuation slots per LP call: one per LP of the batch, up to this many
// bytes of HBM (K3P overflow beyond the slots restarts in K3 from the shared
// warm start)
constexpr size_t kPfiOvfBytes = 24ull << 30;
size_t lp_pfi_lds_bytes(int n, int m, int nnz, int kmax);
bool lp_pfi_fits(int n, int m, int nnz);
hipError_t launch_lp_pfi(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                         hipStream_t stream);
// K3PW (lp_pfi_wide.hip): K3P for 64 < m <= 128 (two basis rows per lane),
// n + m <= 256, at most kPfiWideMax etas; its overflow list goes to K3L.
constexpr int kPfiWideMax = 32;
static_assert(kPfiWideMax < kStallPivots, "K3PW never reaches the Bland switch");
size_t lp_pfiw_lds_bytes(int n, int m, int nnz);
bool lp_pfiw_fits(int n, int m, int nnz);
hipError_t launch_lp_pfiw(const DevLP &lp, const LpIO &io, const PfiIO &px, int num_cus,
                          hipStream_t stream);



hipError_t launch_node_decide(const DevLP &lp, const DecideIO &io, hipStream_t stream);

size_t lp_lds_bytes(int n, int m, int nnz);
// K3 with per-node rows: each wave also keeps its node's matrix values and
// row bounds in LDS
size_t lp_lds_bytes_rows(int n, int m, int nnz);

// K3R (lp_rows.hip): the warm basis refactored for each node's own matrix
// (OsiLPEngine::changeConstraint then Clp's factorisation of the kept
// basis): the oracle's invert_basis (Gauss-Jordan, partial pivoting, a
// pivot below 1e-12 = singular -> slack basis) and compute_duals, bit for
// bit.  Writes a per-node warm start (head, st, d, binv column-major).
struct RefacIO {
  int batch;
  NodeRowsIO nr;
  const int32_t *skip;          // [B] or null
  const int32_t *head;          // warm basis in: [m] (s_head 0) or [B][m]
  const int8_t *st;             // [n+m] or [B][n+m]
  long s_head, s_st;
  int32_t *o_head;              // [B][m]
  int8_t *o_st;                 // [B][n+m]
  double *o_d;                  // [B][n+m]
  double *o_binv;               // [B][m][m] column-major
  int32_t *o_sing;              // [B] 1: singular, slack basis (or null)
  // the warm basis' inverse for the LOADED matrix ([m][m] column-major,
  // shared) or null: with it, a node's basis is refactored by replacing only
  // the basic columns its rows changed (Gauss-Jordan when a pivot is tiny)
  const double *binv0;
};
size_t lp_refactor_lds_bytes(int n, int m, int nnz);
hipError_t launch_lp_refactor(const DevLP &lp, const RefacIO &io, hipStream_t stream);

hipError_t launch_lp_dual(const DevLP &lp, const LpIO &io, int num_cus, hipStream_t stream);
// K3L (lp_large.hip): one node per 256-thread workgroup, B^-1 in HBM slots
size_t lp_large_lds_bytes(int n, int m);
constexpr int kLargeLdsMax = 160 * 1024 - 64;  // dynamic LDS cap (K3L has a static word too)
int lp_large_grid(int batch, int n, int m, int num_cus);
hipError_t lp_large_prepare();
hipError_t launch_lp_large(const DevLP &lp, const LpIO &io, double *binv_slots, int grid,
                           hipStream_t stream);

// Output/optional mod-log arguments of one FBBT launch.
struct FbbtIO {
  const double *lb_in, *ub_in;  // [B][n]
  double *lb_out, *ub_out;      // [B][n]
  int32_t *infeas, *nmods;      // [B]
  int32_t *mod_var, *mod_lu;    // [B][mod_cap] or null
  double *mod_val;
  int mod_cap;
  int batch;
  int has_inc;
  double inc_ub;                // incumbent - objective constant
  int npw;                      // nodes per wave (64, or fewer for more waves)
  double *scratch;              // global-bounds variant: [waves][2][n][kLanes]
  uint8_t *flag_scratch;        // global-bounds variant: [waves][m][kLanes]
  int32_t *next;                // persistent variant: zeroed node counter (queue head)
  int refill_min;               // persistent variant: idle lanes before a refill (1 = any)
};

constexpr int kLanes = 64;      // wave64: one node per lane
constexpr int kLdsStride = 65;  // padded [var][lane] stride (bank spread)

hipError_t launch_fbbt_linear(const DevLP &lp, const FbbtIO &io, int variant,
                              hipStream_t stream);
// K1G (fbbt_group.hip): g = 16, 8 or 4 lanes per node, bounds in LDS;
// m <= 64, no mod log.  Waves per workgroup the LDS allows (0: not
// applicable).
int fbbt_group_waves(const DevLP &lp, int g);
hipError_t launch_fbbt_group(const DevLP &lp, const FbbtIO &io, int g, int num_cus,
                             hipStream_t stream);
size_t fbbt_lds_bytes(int n, int m);
size_t fbbt_persist_lds(const DevLP &lp);   // records staged by K1's persistent kernel

// ---- quadratic node FBBT (K2) ---------------------------------------------
// One tightenQuad_ term, pre-classified on the host (QuadHandler.cpp:
// 2361-2427): kind 0 univariate a x^2 + b x (x also linear), 1 product /
// square coef * v1 * v2, 2 linear coef * v1.
struct alignas(16) QTermRec {  // 32 B
  double a, b;
  int32_t kind, v1, v2, pad;
};
// One tightenQuad_ function: terms [t0, t0 + nt) in forward order.
struct alignas(16) QFunRec {   // 32 B
  double clb, cub;
  int32_t t0, nt, is_obj, pad;
};
struct DevQuad {
  int nv, nsq, nbil, maxt;
  const uint8_t *vtype;          // [nv] Types.h numerics
  const int32_t *sq;             // [nsq][2]  x, y
  const int32_t *bil;            // [nbil][3] x0, x1, y
  // tightenQuad_ programs: [0] without the objective, [1] with it
  const QFunRec *fun[2];
  int nfun[2];
  const QTermRec *term[2];
  double obj_const;
};
struct QuadIO {
  int batch;
  const double *lb_in, *ub_in;   // [B][nv]
  double *lb_out, *ub_out;       // [B][nv]
  const double *rows_in;         // [B][R] or shared (rows_stride 0)
  long rows_stride;
  double *rows_out;              // [B][R]
  int32_t *infeas, *nmods;       // [B]; infeas 2 = propagation cap hit
  int32_t *mod_kind, *mod_idx;   // [B][mod_cap] or null
  double *mod_v1, *mod_v2;
  int mod_cap;
  int qt;                        // run tightenQuad_
  int prog;                      // which program (objective processed or not)
  double best;                   // incumbent objective value (+inf if none)
  double *scratch;               // [waves][2 nv + 2 maxt][kLanes]
};
hipError_t launch_quad_fbbt(const DevQuad &q, const QuadIO &io, bool use_lds,
                            hipStream_t stream);
size_t quad_lds_bytes(const DevQuad &q);

}  // namespace mgpu
