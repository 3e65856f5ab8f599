// Host runtime of the per-node rows path (include/mgpu.h "per-node rows"):
// the node-row map of mgpu_set_node_rows, and mgpu_lp_solve_rows[_dev] =
// K3R (per-node basis refactorisation, lp_rows.hip) then K3 (lp_dual.hip)
// with each node's matrix values and row bounds.
//
// Reference: QuadHandler::upSqCon_ / upBilCon_ (src/base/QuadHandler.cpp:
// 3322-3419) produce the rewritten rows, OsiLPEngine::changeConstraint
// (src/interfaces/OsiLPEngine.cpp:206-243) loads them, OsiLPEngine::solve
// (:571-652) resolves from the kept basis.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.h"

namespace {

// device layout of the map: csc_pos, csr_pos, coef_src [ncoef], then row,
// lo_src, hi_src [nrow]
struct MapView {
  const int32_t *csc_pos, *csr_pos, *coef_src, *row, *lo_src, *hi_src;
};

MapView map_view(const mgpu_ctx *c) {
  const int32_t *b = c->nr_map.as<int32_t>();
  const size_t k = (size_t)c->nr_ncoef, r = (size_t)c->nr_nrow;
  return MapView{b, b + k, b + 2 * k, b + 3 * k, b + 3 * k + r, b + 3 * k + 2 * r};
}

}  // namespace

extern "C" {

int mgpu_set_node_rows(mgpu_ctx *c, int stride, int ncoef, const int32_t *coef_pos,
                       const int32_t *coef_src, int nrow, const int32_t *row_idx,
                       const int32_t *lo_src, const int32_t *hi_src) {
  if (!c) return MGPU_ERR_ARG;
  c->nr_set = false;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_set_node_rows: no problem loaded");
  if (ncoef < 0 || nrow < 0) return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: bad count");
  if (ncoef == 0 && nrow == 0) return MGPU_OK;  // cleared
  const int n = c->lp.n, m = c->lp.m, nnz = c->lp.nnz;
  if (stride <= 0 || (ncoef > 0 && (!coef_pos || !coef_src)) ||
      (nrow > 0 && (!row_idx || !lo_src || !hi_src)))
    return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: bad argument");
  // CSR entry -> CSC position, as mgpu_load_lp filled the CSC (CSR order)
  std::vector<int32_t> csc_of(nnz > 0 ? nnz : 1);
  {
    std::vector<int32_t> fill(n + 1, 0);
    for (int k = 0; k < nnz; ++k) fill[c->h_terms[k].j + 1]++;
    for (int j = 0; j < n; ++j) fill[j + 1] += fill[j];
    for (int k = 0; k < nnz; ++k) csc_of[k] = fill[c->h_terms[k].j]++;
  }
  std::vector<int32_t> h((size_t)3 * ncoef + (size_t)3 * nrow + 1);
  std::vector<char> seen(nnz > 0 ? nnz : 1, 0), rseen(m > 0 ? m : 1, 0);
  for (int k = 0; k < ncoef; ++k) {
    const int pos = coef_pos[k], src = coef_src[k];
    if (pos < 0 || pos >= nnz || seen[pos])
      return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: coef_pos[%d] = %d out of range or repeated",
                  k, pos);
    if (src < 0 || src >= stride)
      return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: coef_src[%d] = %d not in [0, %d)", k,
                  src, stride);
    seen[pos] = 1;
    h[k] = csc_of[pos];
    h[ncoef + k] = pos;
    h[2 * ncoef + k] = src;
  }
  int32_t *hr = h.data() + 3 * (size_t)ncoef;
  for (int q = 0; q < nrow; ++q) {
    const int r = row_idx[q];
    if (r < 0 || r >= m || rseen[r])
      return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: row_idx[%d] = %d out of range or repeated",
                  q, r);
    if (lo_src[q] < -1 || lo_src[q] >= stride || hi_src[q] < -1 || hi_src[q] >= stride)
      return fail(c, MGPU_ERR_ARG, "mgpu_set_node_rows: row %d bound source out of range", r);
    rseen[r] = 1;
    hr[q] = r;
    hr[nrow + q] = lo_src[q];
    hr[2 * nrow + q] = hi_src[q];
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the old map may be in use
  HIPCHK(c, upload(c->nr_map, h.data(), h.size()));
  c->nr_stride = stride;
  c->nr_ncoef = ncoef;
  c->nr_nrow = nrow;
  c->nr_set = true;
  return MGPU_OK;
}

int mgpu_lp_solve_rows_dev(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                           const int32_t *skip, const double *vals, const int32_t *ws_head,
                           const int8_t *ws_st, int ws_shared, int iter_limit, int32_t *status,
                           double *obj, int32_t *iters, double *x, const double *ws_binv) {
  return lp_solve_rows_wo(c, batch, lb, ub, skip, vals, ws_head, ws_st, ws_shared, iter_limit,
                          status, obj, iters, x, ws_binv, nullptr);
}

}  // extern "C"

// mgpu_lp_solve_rows_dev plus the optimal basis of every solved node written
// out (wo: head [B][m], st [B][n+m], d [B][n+m], B^-1 [B][m][m]; null: none):
// the glob tree's parent-basis warm starts (glob_runtime.cpp)
int lp_solve_rows_wo(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                     const int32_t *skip, const double *vals, const int32_t *ws_head,
                     const int8_t *ws_st, int ws_shared, int iter_limit, int32_t *status,
                     double *obj, int32_t *iters, double *x, const double *ws_binv,
                     const LpWarmOut *wo) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_rows: no problem loaded");
  if (!c->nr_set) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_rows: no node rows set");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !vals || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: bad argument");
  if (ws_head && !ws_st)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: warm start needs head and st");
  if (ws_binv && (!ws_head || !ws_shared))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: ws_binv needs a shared warm start");
  const int n = c->lp.n, m = c->lp.m, N = n + m, nnz = c->lp.nnz;
  if (m == 0) return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: m = 0");
  // K3R + K3 while the node matrix and the refactorisation fit one wave's
  // LDS (m <= 64); beyond, K3L with the node rows in a per-workgroup HBM
  // slot and the warm basis refactored inside the kernel
  const bool large = m > kLpMaxM || lp_lds_bytes_rows(n, m, nnz) > 160 * 1024 ||
                     lp_refactor_lds_bytes(n, m, nnz) > 160 * 1024;
  if (large && lp_large_lds_bytes(n, m) > (size_t)kLargeLdsMax)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: n+m=%d too large for K3L's LDS state",
                N);
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const MapView mv = map_view(c);
  NodeRowsIO nr{};
  nr.vals = vals;
  nr.stride = c->nr_stride;
  nr.ncoef = c->nr_ncoef;
  nr.csc_pos = mv.csc_pos;
  nr.csr_pos = mv.csr_pos;
  nr.coef_src = mv.coef_src;
  nr.nrow = c->nr_nrow;
  nr.row = mv.row;
  nr.lo_src = mv.lo_src;
  nr.hi_src = mv.hi_src;

  LpIO io{};
  io.batch = batch;
  io.nr = nr;
  io.lb = lb;
  io.ub = ub;
  io.box_stride = n;
  io.skip = skip;
  io.iter_limit = iter_limit > 0 ? iter_limit : iter_limit == 0 ? kLpDefaultIterLimit : 0x7fffffff;
  io.status = status;
  io.obj = obj;
  io.iters = iters;
  io.x = x;
  if (wo != nullptr) {
    io.wo_head = wo->head;
    io.wo_st = wo->st;
    io.wo_d = wo->d;
    io.wo_binv = wo->binv;
  }
  HIPCHK(c, hipEventRecord(c->ev9, c->stream));
  if (large) {
    const int grid = lp_large_grid(batch, n, m, c->num_cus);
    const long wgs = 2L * nnz + 2L * m + (long)m * m;
    HIPCHK(c, c->lp_slots.ensure((size_t)grid * m * m * sizeof(double) + 8));
    HIPCHK(c, c->nr_ws.ensure((size_t)grid * wgs * sizeof(double) + 8));
    io.nr.wg = c->nr_ws.as<double>();
    io.nr.wg_stride = wgs;
    io.nr.binv0 = ws_binv;
    if (ws_head)  // head + statuses only: K3L refactors them for each node's matrix
      io.ws = LpWarm{ws_head, ws_st, nullptr, nullptr, ws_shared ? 0 : m, ws_shared ? 0 : N,
                     0, 0};
    HIPCHK(c, hipEventRecord(c->ev10, c->stream));
    c->last_lp_pfi = false;
    HIPCHK(c, c->lp_next.ensure(sizeof(int32_t)));
    HIPCHK(c, hipMemsetAsync(c->lp_next.p, 0, sizeof(int32_t), c->stream));
    io.next = c->lp_next.as<int32_t>();
    HIPCHK(c, lp_large_prepare());
    (void)hipGetLastError();
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    HIPCHK(c, launch_lp_large(c->lp, io, c->lp_slots.as<double>(), grid, c->stream));
    HIPCHK(c, hipEventRecord(c->ev3, c->stream));
    return MGPU_OK;
  }
  if (ws_head) {
    // K3R: every node's warm start for its own matrix
    const size_t B = (size_t)batch;
    const size_t s_head = al16h(B * m * 4), s_st = al16h(B * N), s_d = al16h(B * N * 8),
                 s_binv = B * m * m * 8;
    HIPCHK(c, c->nr_ws.ensure(s_head + s_st + s_d + s_binv));
    char *w = c->nr_ws.as<char>();
    RefacIO rf{};
    rf.batch = batch;
    rf.nr = nr;
    rf.skip = skip;
    rf.head = ws_head;
    rf.st = ws_st;
    rf.s_head = ws_shared ? 0 : m;
    rf.s_st = ws_shared ? 0 : N;
    rf.o_head = (int32_t *)w;
    rf.o_st = (int8_t *)(w + s_head);
    rf.o_d = (double *)(w + s_head + s_st);
    rf.o_binv = (double *)(w + s_head + s_st + s_d);
    rf.binv0 = ws_binv;
    HIPCHK(c, launch_lp_refactor(c->lp, rf, c->stream));
    io.ws = LpWarm{rf.o_head, rf.o_st, rf.o_d, rf.o_binv, m, N, N, (long)m * m};
  }
  HIPCHK(c, hipEventRecord(c->ev10, c->stream));
  c->last_lp_pfi = false;
  HIPCHK(c, c->lp_next.ensure(sizeof(int32_t)));  // K3's dynamic node schedule
  HIPCHK(c, hipMemsetAsync(c->lp_next.p, 0, sizeof(int32_t), c->stream));
  io.next = c->lp_next.as<int32_t>();
  HIPCHK(c, hipEventRecord(c->ev2, c->stream));
  HIPCHK(c, launch_lp_dual(c->lp, io, c->num_cus, c->stream));
  HIPCHK(c, hipEventRecord(c->ev3, c->stream));
  return MGPU_OK;
}

extern "C" {

int mgpu_lp_solve_rows(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                       const int32_t *skip, const double *vals, const int32_t *ws_head,
                       const int8_t *ws_st, int ws_shared, int iter_limit, int32_t *status,
                       double *obj, int32_t *iters, double *x, const double *ws_binv) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_rows: no problem loaded");
  if (!c->nr_set) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_rows: no node rows set");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !vals || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: bad argument");
  if (ws_head && !ws_st)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_rows: warm start needs head and st");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  const size_t B = (size_t)batch, wsB = ws_shared ? 1 : B;
  hipStream_t s = c->stream;
  auto h2d = [&](DevBuf &d, const void *src, size_t bytes) -> hipError_t {
    hipError_t e = d.ensure(bytes > 0 ? bytes : 16);
    if (e != hipSuccess || !src) return e;
    return hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, s);
  };
  HIPCHK(c, h2d(c->lp_lb, lb, B * n * 8));
  HIPCHK(c, h2d(c->lp_ub, ub, B * n * 8));
  HIPCHK(c, h2d(c->nr_vals, vals, B * c->nr_stride * 8));
  if (skip) HIPCHK(c, h2d(c->lp_skip, skip, B * 4));
  if (ws_head) {
    HIPCHK(c, h2d(c->lp_wh, ws_head, wsB * m * 4));
    HIPCHK(c, h2d(c->lp_wst, ws_st, wsB * N));
  }
  if (ws_binv) HIPCHK(c, h2d(c->lp_wb, ws_binv, (size_t)m * m * 8));
  HIPCHK(c, c->lp_st.ensure(B * 4));
  HIPCHK(c, c->lp_obj.ensure(B * 8));
  HIPCHK(c, c->lp_it.ensure(B * 4));
  if (x) HIPCHK(c, c->lp_x.ensure(B * n * 8));
  int rc = mgpu_lp_solve_rows_dev(
      c, batch, c->lp_lb.as<double>(), c->lp_ub.as<double>(),
      skip ? c->lp_skip.as<int32_t>() : nullptr, c->nr_vals.as<double>(),
      ws_head ? c->lp_wh.as<int32_t>() : nullptr, ws_head ? c->lp_wst.as<int8_t>() : nullptr,
      ws_shared, iter_limit, c->lp_st.as<int32_t>(), c->lp_obj.as<double>(),
      c->lp_it.as<int32_t>(), x ? c->lp_x.as<double>() : nullptr,
      ws_binv ? c->lp_wb.as<double>() : nullptr);
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(status, c->lp_st.p, B * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(obj, c->lp_obj.p, B * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(iters, c->lp_it.p, B * 4, hipMemcpyDeviceToHost, s));
  if (x) HIPCHK(c, hipMemcpyAsync(x, c->lp_x.p, B * n * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return MGPU_OK;
}

int mgpu_lp_refactor(mgpu_ctx *c, const int32_t *head, const int8_t *st, int32_t *o_head,
                     int8_t *o_st, double *o_d, double *o_binv, int *singular) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_refactor: no problem loaded");
  if (!head || !st || !o_head || !o_st || !o_d || !o_binv)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_refactor: bad argument");
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  if (m > kLpMaxM || m == 0 || lp_refactor_lds_bytes(n, m, c->lp.nnz) > 160 * 1024)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_refactor: needs 0 < m <= %d (m=%d)", kLpMaxM, m);
  HIPCHK(c, hipSetDevice(c->device));
  const size_t s_h = al16h((size_t)m * 4), s_s = al16h((size_t)N), s_d = al16h((size_t)N * 8),
               s_b = al16h((size_t)m * m * 8);
  // in: head, st; out: head, st, d, binv, singular flag
  HIPCHK(c, c->nr_vals.ensure(2 * s_h + 2 * s_s + s_d + s_b + 16));
  char *w = c->nr_vals.as<char>();
  int32_t *d_head = (int32_t *)w;
  int8_t *d_st = (int8_t *)(w + s_h);
  RefacIO rf{};
  rf.batch = 1;
  rf.head = d_head;
  rf.st = d_st;
  rf.o_head = (int32_t *)(w + s_h + s_s);
  rf.o_st = (int8_t *)(w + 2 * s_h + s_s);
  rf.o_d = (double *)(w + 2 * s_h + 2 * s_s);
  rf.o_binv = (double *)(w + 2 * s_h + 2 * s_s + s_d);
  rf.o_sing = (int32_t *)(w + 2 * s_h + 2 * s_s + s_d + s_b);
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_head, head, (size_t)m * 4, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(d_st, st, (size_t)N, hipMemcpyHostToDevice, s));
  HIPCHK(c, launch_lp_refactor(c->lp, rf, s));
  int32_t sing = 0;
  HIPCHK(c, hipMemcpyAsync(o_head, rf.o_head, (size_t)m * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(o_st, rf.o_st, (size_t)N, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(o_d, rf.o_d, (size_t)N * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(o_binv, rf.o_binv, (size_t)m * m * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(&sing, rf.o_sing, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  if (singular) *singular = sing;
  return MGPU_OK;
}

}  // extern "C"
