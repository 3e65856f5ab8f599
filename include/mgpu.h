/*
 * mgpu.h — C ABI of the MI355X (gfx950) relaxation-solving and
 * bound-tightening engine for Minotaur's branch-and-bound.
 *
 * This is the drop-in boundary.  A host C++ plugin that keeps
 * Minotaur's src/base plugin surface unchanged calls only these entry points:
 *
 *   HipLPEngine : LPEngine   (replaces OsiLPEngine, src/interfaces/OsiLPEngine.cpp)
 *   batched FBBT handler     (replaces LinearHandler::presolveNode,
 *                             src/base/LinearHandler.cpp:1592-1603)
 *
 * (INTEGRATION.md shows both subclasses and the EngineFactory registration.)
 *
 * Conventions
 *   - Plain pointers and sizes only; no exceptions cross the ABI; every
 *     function returns MGPU_OK (0) or a negative MGPU_ERR_* code and records
 *     a message retrievable with mgpu_last_error().
 *   - Variable types use the reference's VariableType numerics
 *     (src/base/Types.h:83-89): 0 Binary, 1 Integer, 2 ImplBin, 3 ImplInt,
 *     4 Continuous.
 *   - LP status values ARE the reference's EngineStatus numerics
 *     (src/base/Types.h:152-166).
 *   - Missing bounds are IEEE +-infinity; |b| >= 1e20 counts as infinite in
 *     FBBT exactly as in LinearHandler.cpp:58,71.
 *   - Node boxes are row-major [batch][n] f64.
 *   - Functions suffixed _dev take DEVICE pointers (hipMalloc'ed or torch
 *     CUDA tensors) and are asynchronous on the context's stream; the others
 *     take host pointers and return after the results are in host memory.
 *   - One context per host thread (the reference engine is not thread-safe
 *     either: OsiLPEngine, and QGPar.cpp:712-715 clones one per thread).
 */
#ifndef MGPU_H
#define MGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGPU_OK 0
#define MGPU_ERR_ARG (-1)     /* bad argument (null pointer, size) */
#define MGPU_ERR_HIP (-2)     /* HIP runtime error (maps to EngineError) */
#define MGPU_ERR_STATE (-3)   /* call out of order (e.g. no problem loaded) */
#define MGPU_ERR_NOMEM (-4)   /* device allocation failed */
#define MGPU_ERR_ENGINE (-5)  /* a relaxation ended unbounded / unknown (tree search) */

/* EngineStatus numerics (src/base/Types.h:152-166). */
#define MGPU_PROVEN_OPTIMAL 0
#define MGPU_PROVEN_INFEASIBLE 2
#define MGPU_PROVEN_UNBOUNDED 4
#define MGPU_PROVEN_OBJECTIVE_CUTOFF 5
#define MGPU_ENGINE_ITERATION_LIMIT 6
#define MGPU_ENGINE_ERROR 11
#define MGPU_ENGINE_UNKNOWN_STATUS 12

typedef struct mgpu_ctx mgpu_ctx;

/* Context lifetime.  `device` is the HIP device ordinal (one process per
 * GPU: pass LOCAL_RANK).  Replaces the OsiLPEngine constructor
 * (OsiLPEngine.cpp:95-137) and emptyCopy() (:289-291). */
int mgpu_create(int device, mgpu_ctx **out);
int mgpu_destroy(mgpu_ctx *ctx);
const char *mgpu_last_error(const mgpu_ctx *ctx);
/* Use an existing hipStream_t (e.g. torch.cuda.current_stream()); NULL =
 * the context's own stream. */
int mgpu_set_stream(mgpu_ctx *ctx, void *hip_stream);
void *mgpu_get_stream(mgpu_ctx *ctx);
int mgpu_sync(mgpu_ctx *ctx);
/* Device allocations the engine has made in this process (count and bytes,
 * every context, pinned host staging included; buffers grow on demand and
 * are then reused).  A host that
 * times a region checks that the count did not move inside it. */
int mgpu_alloc_stats(long long *count, long long *bytes);

/* Load the batch-shared relaxation: row-major CSR, row bounds, root column
 * bounds and types, and a linear objective to MINIMISE plus constant.
 * Terms inside a row must be given in the order the reference iterates them
 * (the LinearFunction's VariableGroup, ascending variable id: Types.cpp:30-34)
 * — FBBT sums in that order; each column at most once per row.
 * A failed (re)load leaves the context without a problem: every call that
 * needs one returns MGPU_ERR_STATE until a load succeeds.
 * Replaces OsiLPEngine::load (OsiLPEngine.cpp:390-498). */
int mgpu_load_lp(mgpu_ctx *ctx, int n, int m, const int32_t *rowptr,
                 const int32_t *colidx, const double *val,
                 const double *rowlb, const double *rowub,
                 const double *collb, const double *colub,
                 const int32_t *coltype, const double *obj, double objoff);

/* Batched node FBBT over linear rows: for every node box b, the exact
 * result of LinearHandler::presolveNode (LinearHandler.cpp:1592-1653) on the
 * loaded rows with that box.
 *   incumbent   : best known objective value, +INFINITY if none (the
 *                 reference then skips varBndsFromObj_, :1636-1640).
 *   lb/ub_out   : tightened boxes [batch][n] (may alias lb/ub_in).
 *   infeasible  : [batch] presolveNode's return value (1 = infeasible).
 *   nmods       : [batch] number of VarBoundMods the reference appends to
 *                 r_mods.
 *   mod_cap>0   : also write the mod log in push order, [batch][mod_cap]
 *                 (var index, 0 Lower / 1 Upper, new value); entries past
 *                 mod_cap are dropped but still counted in nmods. */
int mgpu_fbbt(mgpu_ctx *ctx, int batch, const double *lb_in,
              const double *ub_in, double incumbent, double *lb_out,
              double *ub_out, int32_t *infeasible, int32_t *nmods,
              int mod_cap, int32_t *mod_var, int32_t *mod_lu,
              double *mod_val);
int mgpu_fbbt_dev(mgpu_ctx *ctx, int batch, const double *d_lb_in,
                  const double *d_ub_in, double incumbent, double *d_lb_out,
                  double *d_ub_out, int32_t *d_infeasible, int32_t *d_nmods,
                  int mod_cap, int32_t *d_mod_var, int32_t *d_mod_lu,
                  double *d_mod_val);

/* Batched LP relaxation solves: for every node box b, what
 * OsiLPEngine::solve (OsiLPEngine.cpp:571-652) returns for the loaded rows
 * with that box — a bounded dual simplex from the warm basis.
 *   skip        : [batch] or NULL; nonzero = node already pruned (e.g. by
 *                 FBBT): not solved, status 12 (EngineUnknownStatus).
 *   ws_*        : warm start (basic column per row [m], column status
 *                 [n+m] 0 lb/1 ub/2 free/3 basic, reduced costs [n+m], basis
 *                 inverse [m][m] COLUMN-major, i.e. binv[k*m+i] = (B^-1)_ik,
 *                 so lane i's row loads coalesce); ws_shared=1: one basis for
 *                 all nodes (e.g. the root optimum), else [batch] of each.
 *                 ws_head == NULL: slack basis.  ws_d == NULL with a
 *                 warm basis: the reduced costs are rebuilt in the kernel for
 *                 the loaded objective (y = c_B' B^-1, d = c - A'y; a basis
 *                 saved under another objective, e.g. the OBBT loop; runs on
 *                 K3 / K3L).  Replaces
 *                 getWarmStartCopy/loadFromWarmStart (:375-384, :500-505).
 *   iter_limit  : pivots per LP; 0 = the reference default 10000
 *                 (OsiLPEngine maxIterLimit_, OsiLPEngine.cpp:99), < 0 = no
 *                 limit; hitting it gives status 6 (EngineIterationLimit,
 *                 :561-569).
 *   status/obj/iters : [batch]; obj includes the objective constant and is
 *                 +INF for infeasible nodes.
 *   x           : [batch][n] primal solution, or NULL.
 *   wo_*        : [batch] warm starts out (children's warm start), or NULL.
 * Kernels: K3P when the batch shares one warm start and wants none back
 * (product form against the shared inverse, m <= 64, n + m <= 256; an LP
 * needing more than the eta-file cap is re-solved by K3), else K3
 * (basis-inverse rows one per lane, m <= 64) or, for more rows, K3L (one
 * node per workgroup, B^-1 in HBM; n + m up to ~3000). */
int mgpu_lp_solve(mgpu_ctx *ctx, int batch, const double *lb, const double *ub,
                  const int32_t *skip, const int32_t *ws_head, const int8_t *ws_st,
                  const double *ws_d, const double *ws_binv, int ws_shared,
                  int iter_limit, int32_t *status, double *obj, int32_t *iters,
                  double *x, int32_t *wo_head, int8_t *wo_st, double *wo_d,
                  double *wo_binv);
int mgpu_lp_solve_dev(mgpu_ctx *ctx, int batch, const double *d_lb, const double *d_ub,
                      const int32_t *d_skip, const int32_t *d_ws_head,
                      const int8_t *d_ws_st, const double *d_ws_d,
                      const double *d_ws_binv, int ws_shared, int iter_limit,
                      int32_t *d_status, double *d_obj, int32_t *d_iters, double *d_x,
                      int32_t *d_wo_head, int8_t *d_wo_st, double *d_wo_d,
                      double *d_wo_binv);

/* ---- basis warm starts (the batched tree's warm mode 2) -------------------
 * NodeIncRelaxer::createNodeRelaxation loads each child with its parent's
 * optimal basis (NodeIncRelaxer.cpp:146-150; TreeManager::branch hands both
 * children the parent's warm start, TreeManager.cpp:97-136; the basis itself
 * is Clp's CoinWarmStartBasis, OsiLPEngine.cpp:375-384, 500-505).  A dense
 * basis inverse per open node (32 KB at m = 64) is too much to keep and move
 * for millions of nodes; a node keeps its basis as the column statuses (n+m
 * bytes) plus the list of its basic columns that are NOT basic in the shared
 * root basis (ascending column index, at most MGPU_PATH_MAX).  K3P rebuilds
 * the inverse from the shared one by column replacement: each listed column
 * takes, through FTRAN, the free row (a root basic column that is nonbasic in
 * the node) with the largest |alpha| (lowest row on ties) and becomes an eta
 * column; a replacement with |alpha| < 1e-9 falls back to the shared basis.
 * Then the reduced costs of that basis are recomputed and the solve
 * continues with its own pivots in the same eta file.  The eta count is the
 * basis difference, not the length of the pivot history.
 *   k_in[b] <= 0      : node b starts from the shared warm start itself;
 *   path_in [batch][MGPU_PATH_MAX] (the listed columns), st_in [batch][n+m]
 *                       (0 lb, 1 ub, 2 free, 3 basic);
 *   k_out / path_out / st_out (optional): node b's final basis for its
 *                       children in the same form, when it is optimal in the
 *                       product form with at most `inherit` basic columns
 *                       outside the shared basis, else k_out[b] = 0 (children
 *                       restart from the shared warm start);
 *   iters             : the node's own pivots.
 * Runs K3P only (m <= 64, n + m <= 256, eta cap <= MGPU_PATH_MAX; an LP that
 * fills the eta file is continued by K3).  oracle/lp_dual.c
 * orc_dual_simplex_path_batch restates it. */
#define MGPU_PATH_MAX 32
int mgpu_lp_solve_path(mgpu_ctx *ctx, int batch, const double *lb, const double *ub,
                       const int32_t *ws_head, const int8_t *ws_st, const double *ws_d,
                       const double *ws_binv, const int32_t *k_in, const uint32_t *path_in,
                       const int8_t *st_in, int inherit, int iter_limit, int32_t *status,
                       double *obj, int32_t *iters, double *x, int32_t *k_out,
                       uint32_t *path_out, int8_t *st_out);
int mgpu_lp_solve_path_dev(mgpu_ctx *ctx, int batch, const double *d_lb, const double *d_ub,
                           const int32_t *d_skip, const int32_t *d_ws_head,
                           const int8_t *d_ws_st, const double *d_ws_d,
                           const double *d_ws_binv, const int32_t *d_k_in,
                           const uint32_t *d_path_in, const int8_t *d_st_in, int inherit,
                           int iter_limit, int32_t *d_status, double *d_obj,
                           int32_t *d_iters, double *d_x, int32_t *d_k_out,
                           uint32_t *d_path_out, int8_t *d_st_out);

/* ---- per-node rows (the glob path) ---------------------------------------
 * QuadHandler rewrites the secant / McCormick rows of the relaxation at
 * every node (upSqCon_ / upBilCon_, QuadHandler.cpp:3322-3419) and hands
 * them to the engine through OsiLPEngine::changeConstraint (OsiLPEngine.cpp:
 * 206-243), after which Clp refactors the kept basis.  Batched: the loaded
 * relaxation fixes the sparsity pattern; node b brings a value record
 * vals[b][stride] (e.g. mgpu_quad_fbbt's rows_out, zero-copy) from which
 *   coef_pos[k] : an entry of the loaded CSR (index into colidx/val) whose
 *                 value is vals[b][coef_src[k]]; |value| <= 1e-9 counts as
 *                 the term's absence (LinearFunction::addTerm,
 *                 LinearFunction.cpp:89-95);
 *   row_idx[q]  : a row whose bounds are vals[b][lo_src[q]] / vals[b][hi_src[q]]
 *                 (-1 keeps the loaded bound).
 * mgpu_set_node_rows validates and uploads the map (cleared by mgpu_load_lp;
 * ncoef = nrow = 0 clears it).  mgpu_lp_solve_rows[_dev] then solves every
 * node's own LP: with a warm basis (head [m] + st [n+m], shared or per node)
 * the basis is refactored for each node's matrix on the device (K3R: the
 * oracle's Gauss-Jordan with partial pivoting; singular -> slack basis) and
 * its reduced costs recomputed, then the dense dual simplex K3 runs from it
 * (m <= 64).  Outputs as mgpu_lp_solve.  ws_binv (optional, shared warm start,
 * m <= 64): B^-1 of the warm basis for the LOADED matrix, [m][m]
 * column-major; K3R then replaces only the basic columns a node's rows
 * changed (one product-form update each) instead of refactoring from
 * scratch; beyond 64 rows K3L does the same inside the kernel. */
int mgpu_set_node_rows(mgpu_ctx *ctx, int stride, int ncoef, const int32_t *coef_pos,
                       const int32_t *coef_src, int nrow, const int32_t *row_idx,
                       const int32_t *lo_src, const int32_t *hi_src);
int mgpu_lp_solve_rows(mgpu_ctx *ctx, int batch, const double *lb, const double *ub,
                       const int32_t *skip, const double *vals, const int32_t *ws_head,
                       const int8_t *ws_st, int ws_shared, int iter_limit, int32_t *status,
                       double *obj, int32_t *iters, double *x, const double *ws_binv);
int mgpu_lp_solve_rows_dev(mgpu_ctx *ctx, int batch, const double *d_lb, const double *d_ub,
                           const int32_t *d_skip, const double *d_vals,
                           const int32_t *d_ws_head, const int8_t *d_ws_st, int ws_shared,
                           int iter_limit, int32_t *d_status, double *d_obj, int32_t *d_iters,
                           double *d_x, const double *d_ws_binv);

/* The warm basis refactored for the LOADED matrix (host pointers, one
 * basis): what Clp does with the kept basis after OsiLPEngine::
 * changeConstraint / addConstraint / removeCons (OsiLPEngine.cpp:152-262).
 * K3R on the device: the oracle's Gauss-Jordan with partial pivoting and
 * compute_duals.  In: head [m], st [n+m]; out: head, st, reduced costs d
 * [n+m], B^-1 [m][m] column-major; *singular = 1 when the basis was
 * singular and the slack basis was returned instead.  m <= 64. */
int mgpu_lp_refactor(mgpu_ctx *ctx, const int32_t *head, const int8_t *st, int32_t *o_head,
                     int8_t *o_st, double *o_d, double *o_binv, int *singular);

/* Node decision after the relaxation solve (device pointers, async): the
 * EngineStatus switch of PCBProcessor::shouldPrune_ (PCBProcessor.cpp:400-523)
 * plus IntVarHandler::isFeasible (IntVarHandler.cpp:54-84).
 *   decision[b]: 0 branch, 1 infeasible (FBBT or LP), 2 pruned by bound,
 *                3 integer feasible (incumbent candidate), 4 engine problem.
 *   cand_obj[b]: objective when decision 3, else +INF (min = new incumbent).
 * Tolerances are the reference options solAbs_tol, solRel_tol,
 * obj_cut_off, int_tol (Environment.cpp:486,509-528: 1e-6, 1e-6, +INF, 1e-6). */
int mgpu_node_decide_dev(mgpu_ctx *ctx, int batch, const int32_t *d_fbbt_infeas,
                         const int32_t *d_status, const double *d_obj, const double *d_x,
                         double incumbent, double abs_tol, double rel_tol, double cutoff,
                         double int_tol, int32_t *d_decision, double *d_inf_meas,
                         double *d_cand_obj);

/* Which FBBT kernel variant the next calls use (linear K1 and quadratic
 * K2): 0 auto, 1 node state in LDS, 2 node state in a global scratch
 * (large n), 3 (K1) persistent lanes refilled from a node queue, 4 / 5 / 6
 * (K1) K1G with 16 / 8 / 4 lanes per node, bounds in LDS (m <= 64, no mod
 * log).  For tests/benchmarks. */
int mgpu_set_fbbt_variant(mgpu_ctx *ctx, int variant);

/* Which LP kernel the next LP calls use: 0 auto, 1 K3, 2 K3L, 3 product
 * form (K3P / K3PW).  Auto: K3P (product form against the shared inverse)
 * for a batch that shares one warm start and wants no warm start back, when
 * m <= 64 and n + m <= 256, K3PW for such a batch when 64 < m <= 128 and
 * B0^{-1} fits LDS; else K3 when m <= 64 and the matrix fits LDS; else K3L.
 * K3 and K3L restate oracle/lp_dual.c pivot for pivot, K3P its product-form
 * mode (oracle dual_simplex(..., pfi=k)).  For tests/benchmarks. */
int mgpu_set_lp_variant(mgpu_ctx *ctx, int variant);

/* K3P eta-file cap: a node that needs more pivots is continued by K3 from
 * its basis and explicit inverse (one continuation slot per LP of the batch,
 * up to 24 GB; past that it restarts in K3 from the shared warm start).  The
 * eta file lives in VGPRs: caps <= 16 run the 16-eta build (4 waves per
 * SIMD), larger caps the 32-eta build (3 waves per SIMD).  0 keeps auto mode
 * off K3P; 1..MGPU_LP_PFI_BIG (default MGPU_LP_PFI_MAX; caps above it run
 * the 48-eta build at two waves per SIMD, for narrow tree rounds). */
#define MGPU_LP_PFI_MAX 32
#define MGPU_LP_PFI_BIG 48   /* the largest cap mgpu_set_lp_pfi accepts */
int mgpu_set_lp_pfi(mgpu_ctx *ctx, int kmax);

/* K3PW (64 < m <= 128 rows, two basis rows per lane) eta-file cap: a node
 * that needs more pivots is continued by K3L from its basis and explicit
 * inverse.  0 keeps auto mode off K3PW; 1..MGPU_LP_PFI_WIDE_MAX (default
 * MGPU_LP_PFI_WIDE_MAX). */
#define MGPU_LP_PFI_WIDE_MAX 32
int mgpu_set_lp_pfi_wide(mgpu_ctx *ctx, int kmax);

/* The eta-file cap the LP calls use for a batch that shares one warm start
 * and wants no warm start back (K3P or K3PW, the oracle's dual_simplex(...,
 * pfi=k)); 0 when such a batch runs a dense kernel (K3 / K3L). */
int mgpu_lp_pfi_cap(mgpu_ctx *ctx);

/* ---- the single-LP route (an LPEngine solving one LP at a time) ----
 * Replaces the per-solve traffic of OsiLPEngine::solve / getWarmStartCopy /
 * loadFromWarmStart (src/interfaces/OsiLPEngine.cpp:571-652, :375-384,
 * :500-505) for HipLPEngine: warm starts stay in DEVICE slots (basic column
 * per row, column status, reduced costs, basis inverse of the loaded
 * problem's n, m), the host only passes slot ids, and one call is one K3 /
 * K3L launch that reads the box from and writes its results to a pinned host
 * block (no copy-engine transfers).
 *   mgpu_ws_alloc : a free slot sized for the loaded problem (slots of other
 *                   sizes stay valid for their problem);
 *   mgpu_ws_free  : return it (no device work);
 *   mgpu_ws_read / mgpu_ws_write : host copies (head [m], st [n+m], d [n+m],
 *                   binv [m][m] column-major; NULL skips an array on read, d
 *                   may be NULL on write) -- synchronous, for rare host edits
 *                   (rows added / removed, refactor);
 *   mgpu_lp_solve1: one LP on box lb/ub [n] from slot ws_in (-1: slack
 *                   basis; ws_d = 0: the slot's reduced costs are for another
 *                   objective and are rebuilt), final basis into slot ws_out
 *                   (-1: none; written when status is 0 or 6), status / obj
 *                   (incl. the objective constant) / iters as mgpu_lp_solve,
 *                   x [n] and rc [n+m] (reduced costs of the structurals,
 *                   then of the logicals = the row duals y; 0 for basic
 *                   columns) when status is 0 or 6.  Synchronous. */
int mgpu_ws_alloc(mgpu_ctx *ctx, int *slot);
int mgpu_ws_free(mgpu_ctx *ctx, int slot);
int mgpu_ws_read(mgpu_ctx *ctx, int slot, int32_t *head, int8_t *st, double *d, double *binv);
int mgpu_ws_write(mgpu_ctx *ctx, int slot, const int32_t *head, const int8_t *st,
                  const double *d, const double *binv);
int mgpu_lp_solve1(mgpu_ctx *ctx, const double *lb, const double *ub, int ws_in, int ws_d,
                   int ws_out, int iter_limit, int32_t *status, double *obj, int32_t *iters,
                   double *x, double *rc);

/* Batched bound LPs: LP b minimises obj_sign[b] * x[obj_col[b]] over the
 * loaded relaxation on ONE box lb/ub [n] (the relaxation's), warm-started
 * from one shared basis (head [m], st [n+m], binv [m][m] column-major, as
 * mgpu_lp_solve; reduced costs are rebuilt for each objective).  This is
 * the LP work of root OBBT, QuadHandler::tightenLP_ / getBndByLP_
 * (src/base/QuadHandler.cpp:2218-2297, :2080-2109): the caller loads the
 * relaxation plus the objective cutoff row (:2236-2246) with mgpu_load_lp.
 *   obj[b] = obj_sign[b] * x[obj_col[b]] at the optimum (no constant);
 *   status/iters/x as mgpu_lp_solve. */
int mgpu_lp_bound(mgpu_ctx *ctx, int batch, const double *lb, const double *ub,
                  const int32_t *obj_col, const double *obj_sign, const int32_t *ws_head,
                  const int8_t *ws_st, const double *ws_binv, int iter_limit, int32_t *status,
                  double *obj, int32_t *iters, double *x);
int mgpu_lp_bound_dev(mgpu_ctx *ctx, int batch, const double *d_lb, const double *d_ub,
                      const int32_t *d_obj_col, const double *d_obj_sign,
                      const int32_t *d_ws_head, const int8_t *d_ws_st, const double *d_ws_binv,
                      int iter_limit, int32_t *d_status, double *d_obj, int32_t *d_iters,
                      double *d_x);

/* ---- batched branch-and-bound (the caller of the path) -----------------
 * Replaces BranchAndBound::solve's node loop (src/base/BranchAndBound.cpp:
 * 355-526) for the loaded linear relaxation: rounds of up to `batch` open
 * nodes, each FBBT (LinearHandler::presolveNode) -> LP (warm-started from
 * the root optimum) -> PCBProcessor::shouldPrune_ / IntVarHandler::
 * isFeasible -> MaxVioBrancher choice -> IntVarHandler::getBranches, with an
 * HBM-resident pool of open nodes (depth-first stack or best-first, see
 * mgpu_bnb_config).
 *   mgpu_bnb_init  : starts a tree at the root box (pool of `capacity`
 *                    nodes) with a known incumbent value (+INF if none).
 *   mgpu_bnb_round : one round; `incumbent` may lower the incumbent (e.g.
 *                    the all-reduced value of other ranks).  stats are
 *                    cumulative; open == 0 after a round = tree finished.
 *                    MGPU_ERR_ENGINE (stats still filled) when a node LP
 *                    ended unbounded or unknown (decision 4): the reference
 *                    asserts there (PCBProcessor.cpp:437-442).
 *   mgpu_bnb_best  : incumbent value and solution (x NaN when none found).
 * decision codes in ndec[] are those of mgpu_node_decide_dev. */
typedef struct {
  long long rounds, nodes;      /* rounds run, nodes evaluated            */
  long long ndec[5];            /* branch, infeasible, pruned, feasible, error */
  int open;                     /* open nodes after the last round        */
  int last_batch;               /* nodes evaluated in the last round      */
  double incumbent;             /* best objective value (+INF if none)    */
  long long pruned;             /* best-first: open nodes pruned by the
                                   incumbent before evaluation
                                   (TreeManager::getCandidate)            */
  long long lps, pivots;        /* node LPs solved (OsiLPStats::calls) and
                                   their simplex pivots                   */
  long long sb_lps, sb_pivots;  /* reliability branching: strong-branching
                                   LPs (also OsiLPStats::calls) and pivots */
  long long sb_pruned;          /* nodes PrunedByBrancher                 */
  long long sb_modified;        /* nodes ModifiedByBrancher (solved again
                                   with the one-sided bound change from the
                                   last strong-branching basis; counted in
                                   nodes and ndec[0] once more)           */
  long long pfi_pivots;         /* node-LP pivots run by K3P itself (its
                                   own counter: warm-start column
                                   replacements are not pivots; 0 for K3PW
                                   and the dense kernels)                 */
} mgpu_bnb_stats;

/* Search options of the next mgpu_bnb_init (default 0, 0):
 *   order 0: depth-first over batches (the pool is a stack; the preferred
 *            child is popped first, TreeManager's dive);
 *   order 1: best-first (TreeManager tree_search "bfs", NodeHeap.cpp:24-47):
 *            each round takes the `batch` open nodes with the lowest
 *            (bound, pool slot), after pruning the open nodes whose bound
 *            cannot beat the incumbent (TreeManager::getCandidate /
 *            shouldPrune_, TreeManager.cpp:162-186, :403-413);
 *   warm 0:  every node LP starts from the root optimum (one shared basis:
 *            K3P for m <= 64);
 *   warm 1:  every node LP starts from its parent's optimal basis
 *            (NodeIncRelaxer::createNodeRelaxation, NodeIncRelaxer.cpp:
 *            146-150); the basis lives with the node in HBM, m*4 + (n+m)*9 +
 *            m*m*8 bytes per pool slot (K3 / K3L per-node warm starts). */
int mgpu_bnb_config(mgpu_ctx *ctx, int order, int warm);
/* Relaxation of the next mgpu_bnb_init's tree (default 0):
 *   0: the loaded LP (K3P / K3 / K3L);
 *   1: the loaded QP (mgpu_load_qp, same columns as the loaded rows): node
 *      QPs by K5 on the FBBT-tightened boxes — QPDRelaxer + BqpdEngine
 *      (examples/QPDRelaxer.cpp:56-126, BqpdEngine.cpp:449-534) batched.
 *      The loaded LP supplies the rows for K1 (LinearHandler::presolveNode,
 *      without objective propagation: the objective is quadratic) and the
 *      column types; root warm starts (warm 0), MaxVio branching.  A node QP
 *      the interior point does not solve within its iteration limit gets a
 *      phase-1 LP over its box (min 0 s.t. the rows, K3 / K3L): infeasible
 *      rows make it ProvenInfeasible; a feasible one it could not solve ends
 *      the round with MGPU_ERR_ENGINE (decision 4). */
int mgpu_bnb_relaxation(mgpu_ctx *ctx, int kind);
/* order 2: the reference's own node order — TreeManager's "bfs" NodeHeap
 *          (NodeHeap.cpp:24-47: lowest bound within 1e-6, then shallower,
 *          then the larger node id) kept on the host with std::push_heap /
 *          std::pop_heap, node ids as TreeManager assigns them (children in
 *          IntVarHandler::getBranches order, guided dive included), open
 *          nodes pruned lazily at the heap top (TreeManager::getCandidate);
 *          with warm 1 the root LP runs from the slack basis after the
 *          root's presolve (BranchAndBound::processRoot_).  At batch 1 this
 *          is BranchAndBound::solve's sequence (tests/test_ref_tree_gpu.py);
 *          larger batches pop `batch` nodes per round.  Not shardable.
 * warm 2:  every node LP starts from its parent's optimal basis kept as its
 *          column statuses + basic columns outside the root basis, rebuilt by
 *          column replacement (mgpu_lp_solve_path; K3P, MaxVio). */
/* Guided dive (IntVarHandler option guided_dive, default on,
 * Environment.cpp:160-163): with an incumbent, the child whose bound moves
 * the variable toward the incumbent's value comes first.  Order 2 only (the
 * other orders place children by slot). */
int mgpu_bnb_guided_dive(mgpu_ctx *ctx, int on);

/* Brancher of the next mgpu_bnb_init: 0 MaxVioBrancher (default), 1
 * ReliabilityBrancher (the reference's default, ReliabilityBrancher.cpp) with
 * its defaults: pseudocosts, reliability threshold 4 observations per side,
 * node distance 50, at most 20 unreliable candidates strong-branched per
 * node with an iteration limit of 25, pruning / one-sided bound changes
 * from strong branching (trustCutoff).  Batched semantics: the nodes of a
 * round see the pseudocost state of the round's start (plus each node's own
 * updateAfterSolve observation); the round's observations are folded in
 * node order after it, so batch 1 is the reference's sequence.  All the
 * round's strong-branching LPs run in one K3 / K3L batch, each from its
 * node's optimal basis.  Pseudocosts stay with the rank (MpiBranchAndBound
 * keeps one brancher per process). */
int mgpu_bnb_brancher(mgpu_ctx *ctx, int kind);

/* Batch growth of the next mgpu_bnb_init's tree (default 0: off).  With
 * div > 0 a round evaluates at most max(1, nodes evaluated so far / div)
 * nodes (and at most its `batch`): the tree starts narrow and widens as it
 * grows, so every round's decisions rest mostly on what earlier rounds
 * learned -- the batched reliability brancher's pseudocosts come from
 * earlier rounds only (ReliabilityBrancher.cpp:98-132), and a round of
 * 1/div of the tree so far keeps its decisions close to the sequential
 * reference's.  tls4-OA with reliability branching: 12 977 nodes at a fixed
 * batch, 3 371 with div 2 (the reference's own tree: 2 626). */
int mgpu_bnb_growth(mgpu_ctx *ctx, int div);
/* How the reliability brancher runs a round's strong-branching LPs (default
 * 1): 1 every node's chain in one K3 launch, one wave per node, each LP from
 * the basis the previous optimal / iteration-limited one left and the chain
 * ended after the first candidate with a verdict (ReliabilityBrancher::
 * strongBranch_ / findBestCandidate_, :469-506, :111-118); 0 one launch per
 * chain position over every node still strong-branching.  The same LPs, the
 * same results; K3L problems (m > 64) always take the per-position launches. */
int mgpu_set_sb_chain(mgpu_ctx *ctx, int on);

int mgpu_bnb_init(mgpu_ctx *ctx, int capacity, const double *root_lb, const double *root_ub,
                  double incumbent);
int mgpu_bnb_round(mgpu_ctx *ctx, int batch, double incumbent, mgpu_bnb_stats *stats);
int mgpu_bnb_best(mgpu_ctx *ctx, double *obj, double *x);
/* Strong branching (ReliabilityBrancher::strongBranch_, ReliabilityBrancher.cpp:
 * 469-506, with the iteration cap of :101): for ncand candidates (variable,
 * LP value) of one node, 2*ncand child LPs in ONE batch — child 2c = down
 * (ub = floor(val)), 2c+1 = up (lb = ceil(val)) of the node box lb/ub [n] —
 * all warm-started from the node's optimal basis (shared; head/st/d/binv as
 * mgpu_lp_solve, d may be the parent's reduced costs), iter_limit pivots
 * each (status 6 when hit).  The _dev form also returns the child boxes. */
int mgpu_strong_branch(mgpu_ctx *ctx, const double *lb, const double *ub, int ncand,
                       const int32_t *cand_var, const double *cand_val, const int32_t *ws_head,
                       const int8_t *ws_st, const double *ws_d, const double *ws_binv,
                       int iter_limit, int32_t *status, double *obj, int32_t *iters);
int mgpu_strong_branch_dev(mgpu_ctx *ctx, const double *d_lb, const double *d_ub, int ncand,
                           const int32_t *d_cand_var, const double *d_cand_val,
                           const int32_t *d_ws_head, const int8_t *d_ws_st,
                           const double *d_ws_d, const double *d_ws_binv, int iter_limit,
                           double *d_child_lb, double *d_child_ub, int32_t *d_status,
                           double *d_obj, int32_t *d_iters);

/* Node-sharded multi-GPU search (MpiBranchAndBound's round-robin deal,
 * src/base/MpiBranchAndBound.cpp:142-188): keeps open nodes i with
 * i = rank (mod world), packed in order; *kept = nodes left. */
int mgpu_bnb_shard(mgpu_ctx *ctx, int rank, int world, int *kept);

/* Node migration between ranks (MpiBranchAndBound::LoadBalance_'s node
 * send / receive, src/base/MpiBranchAndBound.cpp:78-195; Serializer.cpp:
 * 26-112 carries the same content: the node's bound changes, lower bound and
 * depth).  Host buffers, boxes [k][n].
 *   mgpu_bnb_export: removes up to k open nodes (the stack's top k; in
 *                    best-first order the first k live pool slots) and
 *                    returns their boxes, bounds and depths; *got = count.
 *   mgpu_bnb_import: adds k open nodes (with parent warm starts they start
 *                    from the root basis; best-first: the lowest free slots
 *                    first, as mgpu_bnb_import_dev). */
int mgpu_bnb_export(mgpu_ctx *ctx, int k, double *lb, double *ub, double *nlb, int32_t *depth,
                    int *got);
int mgpu_bnb_import(mgpu_ctx *ctx, int k, const double *lb, const double *ub, const double *nlb,
                    const int32_t *depth);

/* Open nodes in Minotaur's Serializer wire format (Serializer::writeNode /
 * writeMods, src/base/Serializer.cpp:26-112; DeSerializer::readNode /
 * readMods / readVarBoundMod, :130-191), the format MpiBranchAndBound moves
 * nodes in: a node exported by mgpu_bnb_export can go to a reference rank or
 * into a checkpoint the reference's DeSerializer reads, and back through
 * mgpu_bnb_import.  Host only (no context, no device work).
 *   bytes: [uint32 id][double lb][size_t k], then k entries
 *          [int var][short lu][double old][double new], packed, host byte
 *          order, ascending (var, lu) (lu 0 Lower, 1 Upper: BoundType).
 *   mgpu_node_serialize: the node's box against the root box: one entry per
 *          bound that differs (old = the root's, new = the node's), which is
 *          writeMods' merge of the path's relaxation mods (first old, last
 *          new).  *len = the byte count; out NULL: the count only;
 *          MGPU_ERR_ARG if cap < *len.
 *   mgpu_node_deserialize: one node from buf[0, len): its id, lower bound
 *          and box (the root box with each entry's new value); *used = the
 *          bytes read.  MGPU_ERR_ARG on a short buffer, a variable outside
 *          [0, n) or lu not 0 / 1. */
int mgpu_node_serialize(uint32_t id, double lb, int n, const double *root_lb,
                        const double *root_ub, const double *lb_box, const double *ub_box,
                        uint8_t *out, size_t cap, size_t *len);
int mgpu_node_deserialize(const uint8_t *buf, size_t len, int n, const double *root_lb,
                          const double *root_ub, uint32_t *id, double *lb, double *lb_box,
                          double *ub_box, size_t *used);

/* Bound-aware load balancing on device rows (MpiBranchAndBound::LoadBalance_,
 * src/base/MpiBranchAndBound.cpp:78-195).  LoadBalance_ pops each rank's
 * next 50 P candidates (TreeManager::getCandidate, :93-105), all-gathers
 * their lower bounds (:107), sorts them (:111-135) and deals the i-th best to
 * rank i mod P (:142-188), one MPI_Send of a serialised node per move.
 *   mgpu_bnb_pick:       this rank's next S candidates in its search order
 *                        (depth-first: the stack top, topmost first;
 *                        best-first: pruned by the incumbent, then ascending
 *                        (bound, slot)); their bounds into lbs[0, *got) (host).
 *                        The nodes stay in the pool.
 *   mgpu_bnb_export_dev: removes the picked nodes idx[0, k) (indices into the
 *                        last pick, host array) and packs them, in that
 *                        order, into device rows buf[k][W] =
 *                        [lb | ub | bound | depth] (Serializer.cpp:26-112's
 *                        content), in warm mode 2 followed by the node's
 *                        warm start [k | path (MGPU_PATH_MAX) | column
 *                        statuses, 16 two-bit codes per f64]: the basis
 *                        relative to the root basis every rank shares;
 *                        the depth-first stack closes its gaps.
 *   mgpu_bnb_import_dev: adds k nodes from device rows buf (best-first: the
 *                        lowest free pool slots, then past the high-water
 *                        mark; depth-first: on top), in row order; in warm
 *                        mode 2 they start from the basis their row
 *                        carries, otherwise from the root basis.
 *   mgpu_bnb_row_width:  W, the row width in f64 (2n + 2, or 2n + 3 +
 *                        MGPU_PATH_MAX + ceil((n + m) / 16) in warm mode 2).
 *   mgpu_bnb_count:      open nodes and pool slots left for imports. */
int mgpu_bnb_pick(mgpu_ctx *ctx, int S, double *lbs, int *got);
int mgpu_bnb_export_dev(mgpu_ctx *ctx, int k, const int32_t *idx, double *d_rows);
int mgpu_bnb_import_dev(mgpu_ctx *ctx, int k, const double *d_rows);
int mgpu_bnb_row_width(mgpu_ctx *ctx);
int mgpu_bnb_count(mgpu_ctx *ctx, int *open, int *spare);

/* ---- the round collectives of the node-sharded tree (multi-GPU) ---------
 * MpiBranchAndBound (src/base/MpiBranchAndBound.cpp) runs one B&B per MPI
 * rank and couples them with a few small collectives; here they live in the
 * engine so that a C++ host shaped like MpiBranchAndBound shards the batched
 * tree with the C ABI alone (one process per GPU, one context per process).
 * A context without a communicator is a world of one: every collective is
 * the identity there.
 *   mgpu_comm_unique_id : an RCCL unique id (MGPU_COMM_ID_BYTES), made by one
 *                         rank and handed to the others by the host's own
 *                         launcher (MPI_Bcast, a file, a TCP store);
 *   mgpu_comm_init      : an RCCL communicator over the contexts' devices
 *                         (xGMI between the GPUs of a node);
 *   mgpu_comm_init_host : the host's own transport instead (e.g. MPI calls on
 *                         host buffers; device rows are staged through host
 *                         memory); the callbacks return 0 on success;
 *   mgpu_comm_info      : this context's rank and world size.
 * Collectives (blocking unless _dev; every rank calls them in the same order):
 *   mgpu_allreduce_f64  : v[count] in place, op MGPU_OP_SUM / MIN / MAX (the
 *                         MPI_Gather of statistics :417, :442 as a SUM);
 *   mgpu_allreduce_min  : one f64 MIN: the incumbent (MPI_Allreduce MIN,
 *                         :387-389, and the eager pushes of :197-208);
 *   mgpu_round_reduce   : the per-round exchange in ONE all-reduce MIN of
 *                         [incumbent, -open, open, -err] -> out[4] = global
 *                         incumbent, max and min open count over the ranks,
 *                         1 when some rank reported err != 0 (the LOR stop
 *                         flag of :85 and the idle-rank test of the balancer);
 *   mgpu_allgather_f64  : recv[world][count] = every rank's send[count]
 *                         (MPI_Allgather of the candidates' bounds, :107);
 *   mgpu_alltoall_rows_dev : rows of `width` f64 in device memory,
 *                         send_counts[r] rows to rank r (grouped by receiver,
 *                         ascending), recv_counts[r] rows from rank r
 *                         (grouped by sender); asynchronous on the context's
 *                         stream with RCCL (the per-node MPI_Send / MPI_Recv
 *                         of :159-185 as one grouped exchange).
 * Load balancing:
 *   mgpu_lb_deal        : LoadBalance_'s deal (:111-188), host only, no
 *                         context: the rank-major bounds lbs[world][S] (+INF
 *                         padding) sorted ascending by (bound, rank, index)
 *                         (a stable sort; the reference's std::sort leaves
 *                         ties unordered), the i-th dealt to rank i mod world,
 *                         stopping at the first +INF; owner / local / recv[i]
 *                         for i < the returned count;
 *   mgpu_bnb_rebalance  : one whole LoadBalance_ on the tree pool: pick this
 *                         rank's next S candidates (mgpu_bnb_pick), all-gather
 *                         their bounds and every rank's free pool room, deal,
 *                         refuse on every rank a deal that would overflow some
 *                         pool (MGPU_ERR_STATE), export the nodes that change
 *                         rank as device rows, exchange them in one all-to-all
 *                         and import the received rows in deal order.
 *                         picked[S] (optional): the bounds this rank offered,
 *                         *npicked of them; received[world*S] (optional): the
 *                         bounds of the nodes it received, in deal order;
 *                         *moved: nodes that changed rank (all ranks);
 *                         *open_after: this rank's open nodes afterwards. */
#define MGPU_COMM_ID_BYTES 128
#define MGPU_ERR_COMM (-6)   /* a collective failed (RCCL or the host transport) */
#define MGPU_OP_SUM 0
#define MGPU_OP_MIN 1
#define MGPU_OP_MAX 2
typedef struct {
  void *user;
  int (*allreduce)(void *user, double *v, int count, int op);
  int (*allgather)(void *user, const double *send, int count, double *recv);
  int (*alltoallv)(void *user, const double *send, const int32_t *send_counts, double *recv,
                   const int32_t *recv_counts, int width);
} mgpu_host_transport;
int mgpu_comm_unique_id(void *id);
int mgpu_comm_init(mgpu_ctx *ctx, int rank, int world, const void *id);
int mgpu_comm_init_host(mgpu_ctx *ctx, int rank, int world, const mgpu_host_transport *t);
int mgpu_comm_info(mgpu_ctx *ctx, int *rank, int *world);
int mgpu_allreduce_f64(mgpu_ctx *ctx, double *v, int count, int op);
int mgpu_allreduce_min(mgpu_ctx *ctx, double *v);
int mgpu_round_reduce(mgpu_ctx *ctx, double incumbent, double open, int err, double *out);
int mgpu_allgather_f64(mgpu_ctx *ctx, const double *send, int count, double *recv);
int mgpu_alltoall_rows_dev(mgpu_ctx *ctx, int width, const double *d_send,
                           const int32_t *send_counts, double *d_recv,
                           const int32_t *recv_counts);
int mgpu_lb_deal(int world, int S, const double *lbs, int32_t *owner, int32_t *local,
                 int32_t *recv);
int mgpu_bnb_rebalance(mgpu_ctx *ctx, int S, double *picked, int *npicked, double *received,
                       int *nreceived, long long *moved, int *open_after);

/* ---- Batched spatial branch-and-bound (the glob path) --------------------
 * The node loop of the reference's glob solver (Glob::createBab_,
 * src/solvers/Glob.cpp:134-220: BranchAndBound + NodeIncRelaxer +
 * PCBProcessor, handlers IntVarHandler / LinearHandler / QuadHandler,
 * brancher=maxvio) for a QCQP after SimpleTransformer.  Prerequisites: the
 * relaxation LP loaded (mgpu_load_lp: the original rows with products
 * replaced, then QuadHandler::relax_'s secant / McCormick rows at the root
 * box; columns = the quadratic problem's variables), the quadratic problem
 * (mgpu_load_quad) and the node-rows map of the rewritten entries
 * (mgpu_set_node_rows, record stride = its row-state length R, plus 2 S
 * values per square when the LP carries S tangent-cut rows per square:
 * minotaur_amd/quad.py relaxation_lp(tan_slots=S)).
 *   mgpu_glob_init:  the root (the loaded column bounds, its rows from
 *                    mgpu_quad_rows) on an HBM stack of `capacity` nodes; the
 *                    root LP from the slack basis gives the basis every node
 *                    LP starts from (refactored for the node's rows).
 *   mgpu_glob_round: pops the top `batch` nodes: K2 (QuadHandler::
 *                    presolveNode from the parent's rows, tightenQuad_ on),
 *                    K3R + K3 on each node's own rows, then shouldPrune_,
 *                    IntVarHandler / QuadHandler isFeasible and MaxVio
 *                    branching over both handlers' candidates (spatial
 *                    branching at the LP value on a continuous variable,
 *                    floor / ceil on an integer one), two children per
 *                    branched node (the preferred one on top).
 *                    With tangent slots (S > 0): the squares' separation of
 *                    QuadHandler::separate (QuadHandler.cpp:1658-1689) for
 *                    the nodes that would branch -- a tangent of y = x^2 at
 *                    findLinPt_'s point into the square's next free slot,
 *                    the node re-solved and decided again, until no node
 *                    adds a cut (PCBProcessor.cpp:267-280); children inherit
 *                    the node's cuts.
 *   mgpu_glob_best:  the incumbent value and point (NaN: none).
 * Decision codes of ndec: 0 branched, 1 infeasible (K2 or LP), 2 pruned by
 * bound, 3 feasible (incumbent candidate), 4 engine problem (the round
 * returns MGPU_ERR_ENGINE), 5 not feasible without a branching candidate
 * (the reference hands such a node to an NLP engine, PCBProcessor.cpp:
 * 311-330; here it is closed and counted). */
typedef struct {
  long long rounds, nodes;
  long long ndec[6];
  long long lps, pivots;       /* LPs solved (nodes not K2-infeasible, and the
                                  re-solves of the separation loop), their pivots */
  long long br_int, br_cont;   /* branchings at floor / ceil, at the LP value */
  int open, last_batch;
  double incumbent;
  long long cuts, resolves;    /* tangent cuts added, node LPs re-solved for them */
  long long obbt_lps;          /* root OBBT's bound LPs (its root re-solve counts in lps) */
  long long sb_lps;            /* relstronger's strong-branching LPs (counted in lps too) */
} mgpu_glob_stats;
/* Search order, warm starts, the tightenQuad_ rule, the linear node
 * presolve and root OBBT of the next mgpu_glob_init (defaults 0, 0, 1, 0, 0):
 *   order 0  depth-first over batches (an HBM stack, the preferred child on top);
 *         2  the reference's node order: TreeManager's "bfs" NodeHeap
 *            (NodeHeap.cpp:24-47), node ids as TreeManager assigns them, the
 *            children in QuadHandler / IntVarHandler::getBranches order;
 *   warm  0  every node LP from the root basis refactored for its rows;
 *         1  from its parent's optimal basis refactored for its rows, as
 *            HipLPEngine / OsiLPEngine refactor the kept basis after
 *            NodeIncRelaxer replays the node's rows; the root from the slack
 *            basis;
 *   qt    1  tightenQuad_ at every node (doQT_ set, as Glob's presolve sets
 *            it on QCQPs it can tighten); 0 only at the first presolveNode
 *            call (QuadHandler.cpp:1215, 1241; doQT_ false);
 *   lin   1  LinearHandler::presolveNode before QuadHandler's at every node
 *            (PCBProcessor::presolveNode_, PCBProcessor.cpp:134-175; Glob sets
 *            pres_freq 1, Glob.cpp:404): simplePresolve in node mode
 *            (LinearHandler.cpp:1592-1653) over the node's relaxation rows --
 *            the linear rows, the secant / McCormick rows as the node
 *            inherited them, the tangent cuts -- with the incumbent's
 *            objective bound once one is known; a node it proves infeasible
 *            is pruned before its LP (decision 1, no LP counted); 0 none;
 *   obbt  1  root OBBT (OBBT option, Environment.cpp:325-326, on in Glob):
 *            QuadHandler::postSolveRootNode (QuadHandler.cpp:1397-1547) when
 *            the root's first LP neither prunes nor is feasible
 *            (PCBProcessor.cpp:256-262) -- the variables of violated products
 *            marked, tightenLP_'s bound LPs chained one after the other on a
 *            bound-tightening context of the round's own (bte_: each from the
 *            previous optimal basis, the first from the slack basis),
 *            setItmpFromSol_ after each, updatePBounds_, then the secant /
 *            McCormick rows rewritten for the new box; the root is re-solved
 *            when its point violates the tightened relaxation (SepaResolve)
 *            and decided again either way; 0 none.
 * At batch 1 with order 2, warm 1 the tree is the reference's own glob tree
 * node for node, with or without the linear presolve and root OBBT
 * (tests/test_glob_pin_{cpu,gpu}.py). */
int mgpu_glob_config(mgpu_ctx *ctx, int order, int warm, int qt, int lin, int obbt);
/* The glob tree's brancher for the next mgpu_glob_init (default 0):
 *   0  MaxVioBrancher (device decision, any batch);
 *   1  Glob's default, relstronger: StrongBrancher with reliabilitySetup(20,
 *      50, 5) (Glob.cpp:171-181, 308; StrongBrancher.cpp) -- pseudocosts with
 *      reliability threshold 5, up to 20 unreliable candidates strong-
 *      branched in the order of their violation score, each child built with
 *      the handler's getBrMod (QuadHandler's rows for the branch's box) and
 *      every handler's node presolve (getStrongerMods), its LP chained through
 *      the engine with 50 pivots at most, stopping at a verdict (the node
 *      pruned, or modified and re-solved), updateAfterSolve's pseudocost per
 *      node.  One node per round (the reference's sequence; the host runs the
 *      node's loop, the device every presolve, LP and decision); needs order
 *      2, warm 1 and lin 1. */
int mgpu_glob_brancher(mgpu_ctx *ctx, int kind);
int mgpu_glob_init(mgpu_ctx *ctx, int capacity, double incumbent);
int mgpu_glob_round(mgpu_ctx *ctx, int batch, double incumbent, mgpu_glob_stats *stats);
int mgpu_glob_best(mgpu_ctx *ctx, double *obj, double *x);
/* relstronger trees (mgpu_glob_brancher 1): the main engine's solves since
 * mgpu_glob_init in order -- node LPs, re-solves and strong-branching LPs --
 * as (status, value incl. constant, pivots); at most cap written (any array
 * may be NULL); returns the count. */
int mgpu_glob_lp_log(mgpu_ctx *ctx, int cap, int32_t *status, double *value, int32_t *iters);

/* ---- QP relaxation with an MFMA KKT block (K5) ---------------
 * Replaces BqpdEngine::solve (src/interfaces/BqpdEngine.cpp:449-534) on the
 * QP relaxation QPDRelaxer builds (examples/QPDRelaxer.cpp:56-126):
 *     min 1/2 x'Qx + c'x + k  s.t.  A x = b,  lb <= x <= ub   (node box)
 * Q dense symmetric PSD [n][n] (row-major), A dense [m][n] (m <= 64).
 * mgpu_qp_solve[_dev]: one primal-dual interior point solve per node box
 * ([batch][n] lb/ub, finite), Mehrotra predictor-corrector, Newton systems
 * through K = Q + D = L L' (MFMA blocked Cholesky) and M = A K^-1 A'.
 *   status[b]: 0 optimal (residuals <= 1e-9 (1 + |b|, |c|), mu <= 1e-10),
 *              6 iteration limit (maxit, default 80);
 *   obj[b] = 1/2 x'Qx + c'x + k;  iters[b];  x [batch][n] optional. */
int mgpu_load_qp(mgpu_ctx *ctx, int n, int m, const double *Q, const double *c, double k,
                 const double *A, const double *b);
int mgpu_qp_solve(mgpu_ctx *ctx, int batch, const double *lb, const double *ub, int maxit,
                  int32_t *status, double *obj, int32_t *iters, double *x);
int mgpu_qp_solve_dev(mgpu_ctx *ctx, int batch, const double *d_lb, const double *d_ub,
                      int maxit, int32_t *d_status, double *d_obj, int32_t *d_iters,
                      double *d_x);

/* ---- quadratic node FBBT (K2) ------------------------------------------
 * Replaces QuadHandler::presolveNode (src/base/QuadHandler.cpp:1204-1269)
 * for a batch of node boxes over the transformed problem p_ of mglob.
 *
 * mgpu_load_quad: the handler's registries and the original quadratic
 * functions, as QuadHandler::addConstraint (QuadHandler.cpp:127-179) and
 * tightenQuad_ (:2683-2924) see them.
 *   nv, vtype[nv]        variables of p_ (original 0..nv0-1, then aux y's)
 *   sq_x/sq_y[nsq]       y = x^2, strictly ascending x (LinSqrMap order)
 *   bil_x0/x1/y[nbil]    y = x0*x1, x0 < x1, strictly ascending (x0, x1)
 *                        (CompareLinBil, LinBil.cpp:51-62)
 *   ncon, lptr/lvar/lval, qptr/qv1/qv2/qval, clb/cub: the original problem's
 *     constraints in index order; function c has linear terms
 *     [lptr[c], lptr[c+1]) (strictly ascending var, |a| > 1e-9) and
 *     quadratic terms [qptr[c], qptr[c+1]) (v1 <= v2, strictly ascending
 *     (v1, v2), |a| >= 1e-8), all variables < nv0.  When has_obj, function
 *     ncon is the objective (constant obj_const, minimised).
 * A problem is loaded once per context; it may coexist with mgpu_load_lp. */
int mgpu_load_quad(mgpu_ctx *ctx, int nv0, int nv, const int32_t *vtype, int nsq,
                   const int32_t *sq_x, const int32_t *sq_y, int nbil, const int32_t *bil_x0,
                   const int32_t *bil_x1, const int32_t *bil_y, int ncon, const int32_t *lptr,
                   const int32_t *lvar, const double *lval, const int32_t *qptr,
                   const int32_t *qv1, const int32_t *qv2, const double *qval,
                   const double *clb, const double *cub, int has_obj, double obj_const);

/* Secant / McCormick row state of QuadHandler::relax_ (QuadHandler.cpp:
 * 1549-1592) at box lb/ub [nv] (host pointers).  rows[R], R = 2 nsq +
 * 12 nbil: per square [a_x, rhs] of  y + a_x x <= rhs, then per bilinear
 * [a0, a1, rhs] for its four rows  -y + a0 x0 + a1 x1 <= rhs (types 0, 1)
 * and  y + a0 x0 + a1 x1 <= rhs (types 2, 3).  Returns R in *nrows. */
int mgpu_quad_rows(mgpu_ctx *ctx, const double *lb, const double *ub, double *rows, int *nrows);

/* One QuadHandler::presolveNode per node box.
 *   incumbent  best solution value (+INF if none; s_pool->getBestSolutionValue)
 *   qt         1 when tightenQuad_ runs (first call or doQT_, :1241)
 *   rows_in    [batch][R], or [R] shared by all nodes when rows_shared
 *   rows_out   [batch][R] row state after upSqCon_/upBilCon_
 *   infeas[b]  0 feasible, 1 infeasible (presolveNode returned true),
 *              2 propagation loop exceeded 100000 passes, 3 a row rebuild
 *              needed a default bound (|x bound| > 1e12, addDefaultBounds_)
 *   mod log    r_mods in order: kind 0/1 VarBoundMod lower/upper (v1 = new
 *              value), 2 VarBoundMod2 (v1 = lb, v2 = ub), 3 LinConMod (idx =
 *              row: squares 0..nsq-1, then nsq + 4 k + type; v1 = new rhs). */
int mgpu_quad_fbbt(mgpu_ctx *ctx, int batch, const double *lb_in, const double *ub_in,
                   double incumbent, int qt, const double *rows_in, int rows_shared,
                   double *lb_out, double *ub_out, double *rows_out, int32_t *infeas,
                   int32_t *nmods, int mod_cap, int32_t *mod_kind, int32_t *mod_idx,
                   double *mod_v1, double *mod_v2);
int mgpu_quad_fbbt_dev(mgpu_ctx *ctx, int batch, const double *d_lb_in, const double *d_ub_in,
                       double incumbent, int qt, const double *d_rows_in, int rows_shared,
                       double *d_lb_out, double *d_ub_out, double *d_rows_out,
                       int32_t *d_infeas, int32_t *d_nmods, int mod_cap, int32_t *d_mod_kind,
                       int32_t *d_mod_idx, double *d_mod_v1, double *d_mod_v2);

/* Device-side timing of the last launch of the named kernel family
 * ("fbbt", "lp", "quad", "qp", "refactor" = K3R of the last
 * mgpu_lp_solve_rows), measured with hipEvents on the context stream.
 * "lp" is the whole LP call; "lp_main" its first kernel (K3P, or the only
 * one) and "lp_tail" the dense K3 re-solve of K3P's overflow list (0 when
 * K3P did not run).  With mgpu_set_qp_ktime on, "qp_potrf", "qp_trsm" and
 * "qp_step" are the summed times of those K5 kernels over the last QP
 * solve's interior-point iterations. */
double mgpu_last_kernel_ms(mgpu_ctx *ctx, const char *which);

/* Per-kernel event timing of K5's iteration kernels (the KKT factor, the
 * W / Schur products, the Newton steps): on = 1 records events around each
 * of them in every iteration (a measurement mode; the solve itself is
 * unchanged).  Not a reference interface: the bench's per-kernel roofline. */
int mgpu_set_qp_ktime(mgpu_ctx *ctx, int on);

#ifdef __cplusplus
}
#endif
#endif /* MGPU_H */
