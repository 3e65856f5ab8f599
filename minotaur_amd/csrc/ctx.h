// Host-side context of the C ABI (shared by the runtime translation units).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/mgpu.h"
#include "mgpu_internal.h"

using namespace mgpu;

struct QuadState;  // quad_runtime.cpp
struct BnbState;   // bnb.cpp
struct QpState;    // qp_runtime.cpp
struct GlobState;  // glob_runtime.cpp
struct CommState;  // comm_runtime.cpp

// every device allocation the engine makes (mgpu_alloc_stats: a timed
// region must not contain one)
void note_dev_alloc(size_t bytes);  // mgpu_runtime.cpp

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  hipError_t ensure(size_t want) {
    if (want <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) {
      bytes = want;
      note_dev_alloc(want);
    }
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

struct mgpu_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  bool loaded = false;
  DevLP lp{};
  // problem storage
  DevBuf rowptr, terms, rlo, rhi, colptr, rowidx, vtype, obj, collb, colub, objd;
  DevBuf rows, trec, orec, irec, ccont, cval, ccol, rval;
  // LP workspaces (host-pointer path)
  DevBuf lp_lb, lp_ub, lp_skip, lp_wh, lp_wst, lp_wd, lp_wb, lp_st, lp_obj, lp_it, lp_x,
      lp_oh, lp_ost, lp_od, lp_ob;
  std::vector<Term> h_terms;
  // workspaces
  DevBuf io_lb_in, io_ub_in, io_lb_out, io_ub_out, io_inf, io_nmods, io_mv, io_ml, io_mval;
  DevBuf scratch, flag_scratch;
  DevBuf fbbt_next;            // K1 persistent variant: node queue head
  DevBuf lp_next3;             // K3's self-resetting node counter [next, exited waves]
  int fbbt_variant = 0;
  int bnb_relax = 0;          // mgpu_bnb_relaxation: 0 LP (K3P/K3/K3L), 1 QP (K5)
  int lp_variant = 0;          // 0 auto, 1 K3 (m <= 64), 2 K3L, 3 K3P
  int lp_pfi = kPfiMax;        // K3P eta-file cap (0: auto never picks K3P)
  int lp_pfi_wide = kPfiWideMax;  // K3PW eta-file cap (0: auto never picks K3PW)
  int bnb_order = 0;           // mgpu_bnb_config: 0 depth-first stack, 1 best-first
  int bnb_warm = 0;            // mgpu_bnb_config: 0 root basis, 1 parent basis
  int bnb_brancher = 0;        // mgpu_bnb_brancher: 0 MaxVio, 1 reliability
  int bnb_guided = 1;          // mgpu_bnb_guided_dive (order 2: child order by the incumbent)
  int bnb_grow = 0;            // mgpu_bnb_growth: batch <= nodes so far / div (0: off)
  bool sb_chain = true;        // mgpu_set_sb_chain: strong-branching chains in one K3 launch
  DevBuf lp_slots;             // K3L: one B^-1 [m][m] per resident workgroup
  DevBuf lp_next;              // K3L: node counter of the dynamic schedule
  DevBuf pfi_ovf;              // K3P: overflow counter + node list
  DevBuf pfi_cont;             // K3P: continuation state of overflowing LPs
  DevBuf pfi_t0;               // K3P: B0^{-1} a_q of every column [N][m]
  DevBuf pfi_piv;              // K3P: pivots of the last product-form call (u64)
  int num_cus = 256;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr,
            ev5 = nullptr, ev6 = nullptr, ev7 = nullptr;
  hipEvent_t ev8 = nullptr;    // between K3P and its dense overflow re-solve
  bool last_lp_pfi = false;    // the last LP call ran K3P or K3PW
  // the batched tree's node decision for K3P to fuse into its epilogue (set
  // around one LP call by bnb.cpp); lp_decided: that call did decide
  const DecideIO *pfi_decide = nullptr;
  bool lp_decided = false;
  double last_fbbt_ms = 0.0, last_lp_ms = 0.0, last_quad_ms = 0.0, last_qp_ms = 0.0;
  bool qp_ktime = false;          // mgpu_set_qp_ktime
  double last_qp_kms[3] = {0.0, 0.0, 0.0};   // K5 factor / W+Schur / step, summed
  // per-node rows (mgpu_set_node_rows): device maps csc_pos, csr_pos,
  // coef_src, row, lo_src, hi_src; K3R's per-node warm starts; host-path
  // staging of the node records
  bool nr_set = false;
  int nr_stride = 0, nr_ncoef = 0, nr_nrow = 0;
  DevBuf nr_map, nr_ws, nr_vals;
  hipEvent_t ev9 = nullptr, ev10 = nullptr;  // around K3R
  double last_refac_ms = 0.0;
  // device warm-start slots (mgpu_ws_*): chunks of equal-size slots per (n, m)
  struct WsChunk {
    char *base = nullptr;
    int n = 0, m = 0, cap = 0;
    size_t bytes = 0;          // one slot
    std::vector<int> free;
  };
  std::vector<WsChunk> ws_chunks;
  // single-LP route (mgpu_lp_solve1): pinned host block the kernel reads the
  // box from and writes its results to (zero copy)
  char *lp1_pin = nullptr;
  size_t lp1_pin_bytes = 0;
  char *fb1_pin = nullptr;     // the same for mgpu_fbbt at batch 1
  size_t fb1_pin_bytes = 0;
  QuadState *quad = nullptr;   // K2 problem (mgpu_load_quad)
  BnbState *bnb = nullptr;     // batched B&B tree (mgpu_bnb_init)
  QpState *qp = nullptr;       // QP relaxation (mgpu_load_qp)
  GlobState *glob = nullptr;   // batched spatial B&B (mgpu_glob_init)
  int glob_order = 0, glob_warm = 0, glob_qt = 1, glob_lin = 0, glob_obbt = 0;  // mgpu_glob_config
  int glob_brancher = 0;                                                        // mgpu_glob_brancher
  CommState *comm = nullptr;   // round collectives (mgpu_comm_init[_host])
};

namespace {

int fail(mgpu_ctx *c, int code, const char *fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(c, expr)                                                          \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess)                                                        \
      return fail((c), e_ == hipErrorOutOfMemory ? MGPU_ERR_NOMEM : MGPU_ERR_HIP, \
                  "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,      \
                  __LINE__);                                                     \
  } while (0)

inline size_t al16h(size_t b) { return (b + 15) & ~(size_t)15; }

template <class T>
hipError_t upload(DevBuf &b, const T *src, size_t count) {
  hipError_t e = b.ensure(count * sizeof(T) > 0 ? count * sizeof(T) : 16);
  if (e != hipSuccess || count == 0) return e;
  return hipMemcpy(b.p, src, count * sizeof(T), hipMemcpyHostToDevice);
}

}  // namespace

void quad_state_free(mgpu_ctx *c);  // quad_runtime.cpp
void bnb_state_free(mgpu_ctx *c);   // bnb.cpp
void qp_state_free(mgpu_ctx *c);    // qp_runtime.cpp
// K5 over a batch of node boxes; skip[b] != 0 = not solved (qp_runtime.cpp)
int qp_solve_nodes(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                   const int32_t *skip, int maxit, int32_t *status, double *obj, int32_t *iters,
                   double *x);
void glob_state_free(mgpu_ctx *c);  // glob_runtime.cpp
void comm_state_free(mgpu_ctx *c);  // comm_runtime.cpp
// the pool's migration workspaces for exchanges of up to S rows (bnb.cpp)
int bnb_reserve_migration(mgpu_ctx *c, int S);
// a solve's optimal basis out (rows_runtime.cpp lp_solve_rows_wo)
struct LpWarmOut {
  int32_t *head;
  int8_t *st;
  double *d, *binv;
};
int lp_solve_rows_wo(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                     const int32_t *skip, const double *vals, const int32_t *ws_head,
                     const int8_t *ws_st, int ws_shared, int iter_limit, int32_t *status,
                     double *obj, int32_t *iters, double *x, const double *ws_binv,
                     const LpWarmOut *wo);
// an LP batch with per-node warm starts through the K3 / K3L selection of
// mgpu_lp_solve (mgpu_runtime.cpp); io.next is set here
int launch_lp_nodes(mgpu_ctx *c, const LpIO &io);
bool lp_chain_ok(const mgpu_ctx *c);
