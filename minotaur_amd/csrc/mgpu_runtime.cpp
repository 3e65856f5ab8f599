// Host runtime behind the C ABI (include/mgpu.h): one context per host
// thread and device, the batch-shared relaxation resident in HBM, grow-only
// device workspaces, and synchronous host-pointer wrappers around the
// asynchronous device-pointer entry points.
//
// Reference counterparts: OsiLPEngine (src/interfaces/OsiLPEngine.cpp) for
// the context/problem lifetime (load :390-498, clear :264-275), and
// LinearHandler::presolveNode (src/base/LinearHandler.cpp:1592-1603) for
// mgpu_fbbt.  No exception crosses the ABI; HIP failures become
// MGPU_ERR_HIP, which the engine adapter maps to EngineError.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <atomic>

#include "ctx.h"


extern "C" {

int mgpu_create(int device, mgpu_ctx **out) {
  if (!out) return MGPU_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MGPU_ERR_HIP;
  if (device < 0 || device >= ndev) return MGPU_ERR_ARG;
  mgpu_ctx *c = new mgpu_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->ev2) != hipSuccess || hipEventCreate(&c->ev3) != hipSuccess ||
      hipEventCreate(&c->ev4) != hipSuccess || hipEventCreate(&c->ev5) != hipSuccess ||
      hipEventCreate(&c->ev6) != hipSuccess || hipEventCreate(&c->ev7) != hipSuccess ||
      hipEventCreate(&c->ev8) != hipSuccess || hipEventCreate(&c->ev9) != hipSuccess ||
      hipEventCreate(&c->ev10) != hipSuccess) {
    delete c;
    return MGPU_ERR_HIP;
  }
  c->stream = c->own_stream;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cus = prop.multiProcessorCount;
  *out = c;
  return MGPU_OK;
}

int mgpu_destroy(mgpu_ctx *c) {
  if (!c) return MGPU_ERR_ARG;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf *b : {&c->rowptr, &c->terms, &c->rlo, &c->rhi, &c->colptr, &c->rowidx,
                    &c->vtype, &c->obj, &c->collb, &c->colub, &c->objd, &c->rows,
                    &c->trec, &c->orec, &c->irec, &c->ccont, &c->cval, &c->ccol, &c->rval,
                    &c->lp_lb, &c->lp_ub, &c->lp_skip, &c->lp_wh, &c->lp_wst, &c->lp_wd,
                    &c->lp_wb, &c->lp_st, &c->lp_obj, &c->lp_it, &c->lp_x, &c->lp_oh,
                    &c->lp_ost, &c->lp_od, &c->lp_ob, &c->lp_slots, &c->io_lb_in,
                    &c->io_ub_in, &c->io_lb_out, &c->io_ub_out, &c->io_inf, &c->io_nmods,
                    &c->io_mv, &c->io_ml, &c->io_mval, &c->scratch, &c->flag_scratch,
                    &c->fbbt_next, &c->lp_next3, &c->nr_map, &c->nr_ws, &c->nr_vals, &c->pfi_piv})
    b->release();
  for (auto &ch : c->ws_chunks)
    if (ch.base) (void)hipFree(ch.base);
  c->ws_chunks.clear();
  if (c->lp1_pin) (void)hipHostFree(c->lp1_pin);
  c->lp1_pin = nullptr;
  if (c->fb1_pin) (void)hipHostFree(c->fb1_pin);
  c->fb1_pin = nullptr;
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->ev3) (void)hipEventDestroy(c->ev3);
  if (c->ev4) (void)hipEventDestroy(c->ev4);
  if (c->ev5) (void)hipEventDestroy(c->ev5);
  if (c->ev6) (void)hipEventDestroy(c->ev6);
  if (c->ev7) (void)hipEventDestroy(c->ev7);
  if (c->ev8) (void)hipEventDestroy(c->ev8);
  if (c->ev9) (void)hipEventDestroy(c->ev9);
  if (c->ev10) (void)hipEventDestroy(c->ev10);
  glob_state_free(c);
  quad_state_free(c);
  bnb_state_free(c);
  qp_state_free(c);
  comm_state_free(c);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return MGPU_OK;
}

namespace {
std::atomic<long long> g_alloc_count{0}, g_alloc_bytes{0};
}  // namespace

extern "C++" void note_dev_alloc(size_t bytes) {
  g_alloc_count.fetch_add(1, std::memory_order_relaxed);
  g_alloc_bytes.fetch_add((long long)bytes, std::memory_order_relaxed);
}

int mgpu_alloc_stats(long long *count, long long *bytes) {
  if (count) *count = g_alloc_count.load(std::memory_order_relaxed);
  if (bytes) *bytes = g_alloc_bytes.load(std::memory_order_relaxed);
  return MGPU_OK;
}

const char *mgpu_last_error(const mgpu_ctx *c) { return c ? c->err.c_str() : "null context"; }

int mgpu_set_stream(mgpu_ctx *c, void *s) {
  if (!c) return MGPU_ERR_ARG;
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return MGPU_OK;
}

void *mgpu_get_stream(mgpu_ctx *c) { return c ? (void *)c->stream : nullptr; }

int mgpu_sync(mgpu_ctx *c) {
  if (!c) return MGPU_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

int mgpu_load_lp(mgpu_ctx *c, int n, int m, const int32_t *rowptr, const int32_t *colidx,
                 const double *val, const double *rowlb, const double *rowub,
                 const double *collb, const double *colub, const int32_t *coltype,
                 const double *obj, double objoff) {
  if (!c) return MGPU_ERR_ARG;
  // A (re)load replaces the problem: until it has completed, nothing may run
  // on the old one (its buffers are freed as the new ones are allocated), so
  // a failed load leaves the context with no problem (MGPU_ERR_STATE).
  c->loaded = false;
  if (n <= 0 || m < 0 || !rowptr || (m > 0 && (!rowlb || !rowub)) || !collb || !colub ||
      !coltype || !obj)
    return fail(c, MGPU_ERR_ARG, "mgpu_load_lp: bad argument");
  const int nnz = rowptr[m];
  if (rowptr[0] != 0 || nnz < 0 || (nnz > 0 && (!colidx || !val)))
    return fail(c, MGPU_ERR_ARG, "mgpu_load_lp: bad CSR");
  {
    std::vector<int> seen(n, -1);  // a column may appear once per row
    for (int i = 0; i < m; ++i) {
      if (rowptr[i + 1] < rowptr[i]) return fail(c, MGPU_ERR_ARG, "rowptr not monotone at %d", i);
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        if (colidx[k] < 0 || colidx[k] >= n)
          return fail(c, MGPU_ERR_ARG, "column index out of range in row %d", i);
        if (seen[colidx[k]] == i)
          return fail(c, MGPU_ERR_ARG, "row %d has duplicate column %d", i, colidx[k]);
        seen[colidx[k]] = i;
      }
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  bnb_state_free(c);  // a tree belongs to the problem it was started on
  glob_state_free(c);
  c->nr_set = false;  // so do per-node rows (positions in its CSR)
  c->lp = DevLP{};
  // CSR terms, packed
  c->h_terms.resize(nnz > 0 ? nnz : 1);
  for (int k = 0; k < nnz; ++k) c->h_terms[k] = Term{val[k], colidx[k], 0};
  // column -> rows pattern
  std::vector<int32_t> colptr(n + 1, 0), rowidx(nnz > 0 ? nnz : 1);
  for (int k = 0; k < nnz; ++k) colptr[colidx[k] + 1]++;
  for (int j = 0; j < n; ++j) colptr[j + 1] += colptr[j];
  std::vector<double> cvalv(nnz > 0 ? nnz : 1);
  {
    std::vector<int32_t> fill(colptr.begin(), colptr.end() - 1);
    for (int i = 0; i < m; ++i)
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        cvalv[fill[colidx[k]]] = val[k];
        rowidx[fill[colidx[k]]++] = i;
      }
  }
  std::vector<uint8_t> vt(n);
  for (int j = 0; j < n; ++j) vt[j] = (uint8_t)coltype[j];
  std::vector<Term> objt;
  for (int j = 0; j < n; ++j)
    if (obj[j] != 0.0) objt.push_back(Term{obj[j], j, 0});
  int cons_bad = 0;
  for (int i = 0; i < m; ++i)
    if (rowlb[i] > rowub[i] + kETol) cons_bad = 1;
  // wave-uniform records for the FBBT kernel
  std::vector<uint64_t> cmask(n, 0ull);
  if (m <= 64)
    for (int i = 0; i < m; ++i)
      for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) cmask[colidx[k]] |= 1ull << i;
  auto mkrec = [&](double a, int j) {
    TermRec r;
    r.a = a;
    r.cmask = cmask[j];
    r.j = j;
    r.cs = colptr[j];
    r.ce = colptr[j + 1];
    r.isint = (vt[j] == kBinary || vt[j] == kInteger) ? 1 : 0;
    return r;
  };
  std::vector<RowRec> rrec(m > 0 ? m : 1);
  for (int i = 0; i < m; ++i) rrec[i] = RowRec{rowlb[i], rowub[i], rowptr[i], rowptr[i + 1] - rowptr[i], 0, 0};
  std::vector<TermRec> trec(nnz > 0 ? nnz : 1), orec, irec;
  for (int i = 0; i < m; ++i)
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) trec[k] = mkrec(val[k], colidx[k]);
  for (const Term &t : objt) orec.push_back(mkrec(t.a, t.j));
  for (int j = 0; j < n; ++j)
    if (vt[j] == kBinary || vt[j] == kInteger) irec.push_back(mkrec(0.0, j));
  std::vector<int32_t> ccont;  // the other columns (checkBounds_ only)
  for (int j = 0; j < n; ++j)
    if (!(vt[j] == kBinary || vt[j] == kInteger)) ccont.push_back(j);
  const int ncont = (int)ccont.size();
  if (orec.empty()) orec.push_back(TermRec{});
  if (irec.empty()) irec.push_back(TermRec{});
  if (ccont.empty()) ccont.push_back(0);

  HIPCHK(c, upload(c->rowptr, rowptr, (size_t)m + 1));
  HIPCHK(c, upload(c->terms, c->h_terms.data(), (size_t)(nnz > 0 ? nnz : 1)));
  HIPCHK(c, upload(c->rlo, rowlb, (size_t)m));
  HIPCHK(c, upload(c->rhi, rowub, (size_t)m));
  HIPCHK(c, upload(c->colptr, colptr.data(), (size_t)n + 1));
  HIPCHK(c, upload(c->rowidx, rowidx.data(), rowidx.size()));
  HIPCHK(c, upload(c->vtype, vt.data(), (size_t)n));
  HIPCHK(c, upload(c->obj, objt.empty() ? c->h_terms.data() : objt.data(),
                   objt.empty() ? (size_t)0 : objt.size()));
  HIPCHK(c, upload(c->collb, collb, (size_t)n));
  HIPCHK(c, upload(c->colub, colub, (size_t)n));
  HIPCHK(c, upload(c->objd, obj, (size_t)n));
  HIPCHK(c, upload(c->rows, rrec.data(), rrec.size()));
  HIPCHK(c, upload(c->trec, trec.data(), trec.size()));
  HIPCHK(c, upload(c->orec, orec.data(), orec.size()));
  HIPCHK(c, upload(c->irec, irec.data(), irec.size()));
  HIPCHK(c, upload(c->ccont, ccont.data(), ccont.size()));
  HIPCHK(c, upload(c->cval, cvalv.data(), cvalv.size()));
  HIPCHK(c, upload(c->ccol, nnz > 0 ? colidx : rowptr, (size_t)(nnz > 0 ? nnz : 1)));
  HIPCHK(c, upload(c->rval, nnz > 0 ? val : cvalv.data(), (size_t)(nnz > 0 ? nnz : 1)));

  DevLP &lp = c->lp;
  lp.n = n;
  lp.m = m;
  lp.nnz = nnz;
  lp.nobj = (int)objt.size();
  lp.cons_bad = cons_bad;
  lp.rowptr = c->rowptr.as<int32_t>();
  lp.terms = c->terms.as<Term>();
  lp.rlo = c->rlo.as<double>();
  lp.rhi = c->rhi.as<double>();
  lp.colptr = c->colptr.as<int32_t>();
  lp.rowidx = c->rowidx.as<int32_t>();
  lp.vtype = c->vtype.as<uint8_t>();
  lp.obj = c->obj.as<Term>();
  lp.collb = c->collb.as<double>();
  lp.colub = c->colub.as<double>();
  lp.objd = c->objd.as<double>();
  lp.objoff = objoff;
  lp.rows = c->rows.as<RowRec>();
  lp.trec = c->trec.as<TermRec>();
  lp.orec = c->orec.as<TermRec>();
  lp.irec = c->irec.as<TermRec>();
  lp.ccont = c->ccont.as<int32_t>();
  lp.ncont = ncont;
  lp.cval = c->cval.as<double>();
  lp.ccol = c->ccol.as<int32_t>();
  lp.rval = c->rval.as<double>();
  lp.nint = 0;
  for (int j = 0; j < n; ++j) lp.nint += (vt[j] == kBinary || vt[j] == kInteger) ? 1 : 0;
  c->loaded = true;
  return MGPU_OK;
}

int mgpu_set_lp_variant(mgpu_ctx *c, int variant) {
  if (!c || variant < 0 || variant > 3) return MGPU_ERR_ARG;
  c->lp_variant = variant;
  return MGPU_OK;
}

int mgpu_set_lp_pfi(mgpu_ctx *c, int kmax) {
  if (!c || kmax < 0 || kmax > MGPU_LP_PFI_BIG) return MGPU_ERR_ARG;
  c->lp_pfi = kmax;
  return MGPU_OK;
}

int mgpu_set_lp_pfi_wide(mgpu_ctx *c, int kmax) {
  if (!c || kmax < 0 || kmax > MGPU_LP_PFI_WIDE_MAX) return MGPU_ERR_ARG;
  c->lp_pfi_wide = kmax;
  return MGPU_OK;
}

static_assert(MGPU_LP_PFI_MAX == kPfiMax, "ABI eta-file cap = kernel's");
static_assert(MGPU_LP_PFI_BIG == kPfiBig, "ABI largest eta-file cap = kernel's");
static_assert(MGPU_PATH_MAX == kPathMax, "ABI path cap = kernel's");
static_assert(MGPU_LP_PFI_WIDE_MAX == kPfiWideMax, "ABI eta-file cap = kernel's");

int mgpu_set_fbbt_variant(mgpu_ctx *c, int variant) {
  if (!c || variant < 0 || variant > 6) return MGPU_ERR_ARG;
  c->fbbt_variant = variant;
  return MGPU_OK;
}

int mgpu_set_qp_ktime(mgpu_ctx *c, int on) {
  if (!c) return MGPU_ERR_ARG;
  c->qp_ktime = on != 0;
  return MGPU_OK;
}

double mgpu_last_kernel_ms(mgpu_ctx *c, const char *which) {
  if (!c || !which) return -1.0;
  if (!strcmp(which, "fbbt")) {
    float ms = 0.f;
    if (hipEventSynchronize(c->ev1) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess)
      c->last_fbbt_ms = ms;
    return c->last_fbbt_ms;
  }
  if (!strcmp(which, "qp_potrf")) return c->last_qp_kms[0];
  if (!strcmp(which, "qp_trsm")) return c->last_qp_kms[1];
  if (!strcmp(which, "qp_step")) return c->last_qp_kms[2];
  if (!strcmp(which, "refactor")) {  // K3R of the last mgpu_lp_solve_rows
    float ms = 0.f;
    if (hipEventSynchronize(c->ev10) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev9, c->ev10) == hipSuccess)
      c->last_refac_ms = ms;
    return c->last_refac_ms;
  }
  if (!strcmp(which, "lp")) {
    float ms = 0.f;
    if (hipEventSynchronize(c->ev3) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev2, c->ev3) == hipSuccess)
      c->last_lp_ms = ms;
    return c->last_lp_ms;
  }
  // K3P alone / its dense overflow re-solve (lp = both); without K3P,
  // lp_main = lp and lp_tail = 0
  if (!strcmp(which, "lp_main") || !strcmp(which, "lp_tail")) {
    float a = 0.f, t = 0.f;
    if (hipEventSynchronize(c->ev3) != hipSuccess) return -1.0;
    if (!c->last_lp_pfi) {
      if (hipEventElapsedTime(&a, c->ev2, c->ev3) != hipSuccess) return -1.0;
    } else if (hipEventElapsedTime(&a, c->ev2, c->ev8) != hipSuccess ||
               hipEventElapsedTime(&t, c->ev8, c->ev3) != hipSuccess) {
      return -1.0;
    }
    return which[3] == 'm' ? a : t;
  }
  if (!strcmp(which, "qp")) {
    float ms = 0.f;
    if (hipEventSynchronize(c->ev7) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev6, c->ev7) == hipSuccess)
      c->last_qp_ms = ms;
    return c->last_qp_ms;
  }
  if (!strcmp(which, "quad")) {
    float ms = 0.f;
    if (hipEventSynchronize(c->ev5) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ev4, c->ev5) == hipSuccess)
      c->last_quad_ms = ms;
    return c->last_quad_ms;
  }
  return -1.0;
}

int mgpu_fbbt_dev(mgpu_ctx *c, int batch, const double *lb_in, const double *ub_in,
                  double incumbent, double *lb_out, double *ub_out, int32_t *infeas,
                  int32_t *nmods, int mod_cap, int32_t *mod_var, int32_t *mod_lu,
                  double *mod_val) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_fbbt: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb_in || !ub_in || !lb_out || !ub_out || !infeas || !nmods)))
    return fail(c, MGPU_ERR_ARG, "mgpu_fbbt: bad argument");
  if (mod_cap > 0 && (!mod_var || !mod_lu || !mod_val))
    return fail(c, MGPU_ERR_ARG, "mgpu_fbbt: mod_cap > 0 needs mod buffers");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  FbbtIO io{};
  io.lb_in = lb_in;
  io.ub_in = ub_in;
  io.lb_out = lb_out;
  io.ub_out = ub_out;
  io.infeas = infeas;
  io.nmods = nmods;
  io.mod_cap = mod_cap > 0 ? mod_cap : 0;
  io.mod_var = mod_cap > 0 ? mod_var : nullptr;
  io.mod_lu = mod_cap > 0 ? mod_lu : nullptr;
  io.mod_val = mod_cap > 0 ? mod_val : nullptr;
  io.batch = batch;
  // LinearHandler.cpp:1636-1640: only with an incumbent, against
  // (best value - objective constant).
  io.has_inc = std::isfinite(incumbent) ? 1 : 0;
  io.inc_ub = io.has_inc ? incumbent - c->lp.objoff : 0.0;
  // nodes per wave: one per lane fills the chip from kFbbtSmallWaves * CUs *
  // 64 nodes on; a smaller batch (the narrow rounds of a complete tree)
  // spreads its nodes over that many waves instead: a wave walks the union of
  // its nodes' flagged rows, so fewer nodes per wave shorten the round's
  // critical path (a forced variant keeps one node per lane);
  // MGPU_FBBT_NPW overrides for experiments
  int npw = kLanes;
  if (c->fbbt_variant == 0) {
    const long target = (long)c->num_cus * kFbbtSmallWaves;
    if ((long)batch < target * kLanes) {
      const int want = (int)(((long)batch + target - 1) / target);
      npw = 1;
      while (npw < want) npw <<= 1;
    }
  }
  if (const char *e = getenv("MGPU_FBBT_NPW")) {
    const int v = atoi(e);
    if (v >= 1 && v <= kLanes) npw = v;
  }
  io.npw = npw;
  const int waves = (batch + npw - 1) / npw;
  const bool fits = fbbt_lds_bytes(c->lp.n, c->lp.m) <= 160 * 1024;
  // Auto: the LDS variant holds one wave per CU when the node bounds take
  // most of the 160 KiB; beyond that, one node per lane with the bounds in a
  // global scratch while the batch needs at most 8 waves per CU (131 072
  // nodes on 256 CUs), and past that the persistent
  // variant, whose lanes take the next node as soon as theirs finishes
  // (measured on tls4-lin: 262 144 nodes 4.00 -> 3.45 ms, 524 288 nodes
  // 6.67 -> 5.58 ms; at 131 072 the one-shot kernel is faster, 1.87 vs
  // 2.17 ms; tools/fbbt_refill_probe.py).
  int variant = c->fbbt_variant;
  // K1G (variant 4): four nodes per wave, 16 lanes each, bounds in LDS.
  // Auto below kFbbtGroupMax nodes: there one node's chain is the kernel's
  // critical path and K1G shortens it (tls4-oa: 16 384 nodes 0.75 vs 2.25
  // ms, 65 536 2.7 vs 3.2 ms); wider batches fill the chip and K1's lanes
  // per node win (524 288: 7.1 vs 18.7 ms; tools/fbbt_batch_sweep.py,
  // profiles/r04i)
  const int gg = variant == 4 ? 16 : variant == 5 ? 8 : variant == 6 ? 4 : kFbbtGroupG;
  if (variant >= 4 || (variant == 0 && batch <= kFbbtGroupMax && io.mod_cap == 0 &&
                       fbbt_group_waves(c->lp, gg) > 0)) {
    if (fbbt_group_waves(c->lp, gg) <= 0 || io.mod_cap > 0)
      return fail(c, MGPU_ERR_ARG, "mgpu_fbbt: K1G needs m <= 64, no mod log and LDS room");
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_fbbt_group(c->lp, io, gg, c->num_cus, c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    return MGPU_OK;
  }
  if (variant == 0)
    variant = (fits && waves <= c->num_cus) ? 1 : (waves > 8 * c->num_cus && npw == kLanes) ? 3 : 2;
  // persistent path: bit flags (m <= 64) and records staged in 64 KiB of LDS
  if (variant == 3 && (c->lp.m > 64 || fbbt_persist_lds(c->lp) > 64 * 1024))
    variant = 2;
  int grid = waves;
  if (variant == 3) {
    // persistent waves: 12 per CU (three per SIMD at the kernel's 168
    // VGPRs: 524 288 tls4-OA nodes 8.29 -> 7.75 ms against 8 per CU at 179
    // VGPRs, profiles/r04s; four per SIMD spills 284 VGPRs and is slower),
    // fewer for small batches; MGPU_FBBT_WAVES overrides
    grid = c->num_cus * 12;
    if (const char *e = getenv("MGPU_FBBT_WAVES")) {
      const int v = atoi(e);
      if (v >= 1) grid = v;
    }
    const int need = (batch + kLanes - 1) / kLanes;
    if (grid > need) grid = need;
    io.npw = grid;   // the persistent launch reads its grid from npw
    HIPCHK(c, c->fbbt_next.ensure(sizeof(int32_t)));
    HIPCHK(c, hipMemsetAsync(c->fbbt_next.p, 0, sizeof(int32_t), c->stream));
    io.next = c->fbbt_next.as<int32_t>();
    // a wave refills once 16 of its lanes are idle (a wave-sweep with any
    // fresh node visits every row, so fresh nodes are better taken in groups;
    // measured on tls4-lin, 524 288 nodes: 1 / 8 / 16 / 32 idle lanes 4.91 /
    // 4.86 / 4.80 / 5.03 ms, tools/refill_sweep.sh); MGPU_FBBT_REFILL overrides
    io.refill_min = 16;
    if (const char *e = getenv("MGPU_FBBT_REFILL")) {
      const int v = atoi(e);
      if (v >= 1 && v <= 64) io.refill_min = v;
    }
  }
  if (variant == 2 || variant == 3) {
    HIPCHK(c, c->scratch.ensure((size_t)grid * 2 * c->lp.n * kLanes * sizeof(double)));
    HIPCHK(c, c->flag_scratch.ensure((size_t)grid * (c->lp.m > 0 ? c->lp.m : 1) * kLanes));
    // (byte flags are only used when m > 64; bit flags live in VGPRs)
    io.scratch = c->scratch.as<double>();
    io.flag_scratch = c->flag_scratch.as<uint8_t>();
  } else if (!fits) {
    return fail(c, MGPU_ERR_ARG, "LDS variant needs %zu B > 160 KiB",
                fbbt_lds_bytes(c->lp.n, c->lp.m));
  }
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, launch_fbbt_linear(c->lp, io, variant, c->stream));
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  return MGPU_OK;
}

int mgpu_fbbt(mgpu_ctx *c, int batch, const double *lb_in, const double *ub_in,
              double incumbent, double *lb_out, double *ub_out, int32_t *infeas,
              int32_t *nmods, int mod_cap, int32_t *mod_var, int32_t *mod_lu,
              double *mod_val) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_fbbt: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb_in || !ub_in || !lb_out || !ub_out || !infeas || !nmods)))
    return fail(c, MGPU_ERR_ARG, "mgpu_fbbt: bad argument");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t nb = (size_t)batch * c->lp.n * sizeof(double);
  const int cap = mod_cap > 0 ? mod_cap : 0;
  if (batch == 1) {
    // one node (HipLinearHandler::presolveNode): the kernel reads the box
    // from and writes its results to a pinned host block, no copy-engine
    // transfers (as mgpu_lp_solve1)
    const size_t o_ub = nb, o_lo = 2 * nb, o_uo = 3 * nb, o_i = 4 * nb, o_mv = o_i + 16,
                 o_ml = o_mv + al16h((size_t)cap * 4), o_mval = o_ml + al16h((size_t)cap * 4),
                 bytes = o_mval + (size_t)cap * 8 + 16;
    if (c->fb1_pin_bytes < bytes) {
      if (c->fb1_pin) (void)hipHostFree(c->fb1_pin);
      c->fb1_pin = nullptr;
      c->fb1_pin_bytes = 0;
      HIPCHK(c, hipHostMalloc((void **)&c->fb1_pin, bytes, hipHostMallocDefault));
      c->fb1_pin_bytes = bytes;
      note_dev_alloc(bytes);   // pinned host memory counts too
    }
    char *hp = c->fb1_pin, *dp = nullptr;
    HIPCHK(c, hipHostGetDevicePointer((void **)&dp, hp, 0));
    std::memcpy(hp, lb_in, nb);
    std::memcpy(hp + o_ub, ub_in, nb);
    int rc = mgpu_fbbt_dev(c, 1, (const double *)dp, (const double *)(dp + o_ub), incumbent,
                           (double *)(dp + o_lo), (double *)(dp + o_uo), (int32_t *)(dp + o_i),
                           (int32_t *)(dp + o_i + 4), cap, (int32_t *)(dp + o_mv),
                           (int32_t *)(dp + o_ml), (double *)(dp + o_mval));
    if (rc != MGPU_OK) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::memcpy(lb_out, hp + o_lo, nb);
    std::memcpy(ub_out, hp + o_uo, nb);
    *infeas = *(const int32_t *)(hp + o_i);
    *nmods = *(const int32_t *)(hp + o_i + 4);
    const int k = *nmods < cap ? *nmods : cap;
    if (k > 0 && mod_var && mod_lu && mod_val) {
      std::memcpy(mod_var, hp + o_mv, (size_t)k * 4);
      std::memcpy(mod_lu, hp + o_ml, (size_t)k * 4);
      std::memcpy(mod_val, hp + o_mval, (size_t)k * 8);
    }
    return MGPU_OK;
  }
  HIPCHK(c, c->io_lb_in.ensure(nb));
  HIPCHK(c, c->io_ub_in.ensure(nb));
  HIPCHK(c, c->io_lb_out.ensure(nb));
  HIPCHK(c, c->io_ub_out.ensure(nb));
  HIPCHK(c, c->io_inf.ensure((size_t)batch * 4));
  HIPCHK(c, c->io_nmods.ensure((size_t)batch * 4));
  if (cap) {
    HIPCHK(c, c->io_mv.ensure((size_t)batch * cap * 4));
    HIPCHK(c, c->io_ml.ensure((size_t)batch * cap * 4));
    HIPCHK(c, c->io_mval.ensure((size_t)batch * cap * 8));
  }
  HIPCHK(c, hipMemcpyAsync(c->io_lb_in.p, lb_in, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->io_ub_in.p, ub_in, nb, hipMemcpyHostToDevice, c->stream));
  int rc = mgpu_fbbt_dev(c, batch, c->io_lb_in.as<double>(), c->io_ub_in.as<double>(),
                         incumbent, c->io_lb_out.as<double>(), c->io_ub_out.as<double>(),
                         c->io_inf.as<int32_t>(), c->io_nmods.as<int32_t>(), cap,
                         c->io_mv.as<int32_t>(), c->io_ml.as<int32_t>(),
                         c->io_mval.as<double>());
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(lb_out, c->io_lb_out.p, nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(ub_out, c->io_ub_out.p, nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(infeas, c->io_inf.p, (size_t)batch * 4, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipMemcpyAsync(nmods, c->io_nmods.p, (size_t)batch * 4, hipMemcpyDeviceToHost,
                           c->stream));
  if (cap && mod_var && mod_lu && mod_val) {
    HIPCHK(c, hipMemcpyAsync(mod_var, c->io_mv.p, (size_t)batch * cap * 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mod_lu, c->io_ml.p, (size_t)batch * cap * 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mod_val, c->io_mval.p, (size_t)batch * cap * 8,
                             hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

namespace {
// OsiLPEngine caps Clp at maxIterLimit_ = 10000 pivots (OsiLPEngine.cpp:99):
// 0 selects that default, a negative value none (explicit opt-in), as
// include/mgpu.h documents.  The LP kernels have no anti-cycling rule, so the
// cap is what ends a cycling degenerate LP (status 6).
int lp_iter_limit(int iter_limit) {
  return iter_limit > 0 ? iter_limit : iter_limit == 0 ? kLpDefaultIterLimit : 0x7fffffff;
}

// K3 (B^-1 rows in VGPRs, m <= 64, LDS-staged matrix) unless the problem
// needs K3L (more rows, or a matrix that does not fit LDS) or a test forces
// one of them (mgpu_set_lp_variant).
bool use_large_lp(const mgpu_ctx *c) {
  if (c->lp_variant == 2) return true;
  if (c->lp_variant == 1) return false;
  return c->lp.m > kLpMaxM || lp_lds_bytes(c->lp.n, c->lp.m, c->lp.nnz) > 160 * 1024;
}

// Product form serves a batch that shares one warm start and asks for no
// warm start back: K3P for m <= 64 (dense continuation K3), K3PW for
// 64 < m <= 128 (continuation K3L); in auto mode whenever the problem fits,
// variant 3 insists.  Returns the eta-file cap (0: a dense kernel) and which
// kernel in *wide.
int pfi_cap(const mgpu_ctx *c, bool *wide) {
  *wide = false;
  if (!c->loaded || (c->lp_variant != 0 && c->lp_variant != 3)) return 0;
  const int n = c->lp.n, m = c->lp.m, nnz = c->lp.nnz;
  if (lp_pfi_fits(n, m, nnz) && lp_lds_bytes(n, m, nnz) <= 160 * 1024)
    return c->lp_variant == 3 && c->lp_pfi == 0 ? kPfiMax : c->lp_pfi;
  if (lp_pfiw_fits(n, m, nnz) && lp_large_lds_bytes(n, m) <= (size_t)kLargeLdsMax) {
    *wide = true;
    return c->lp_variant == 3 && c->lp_pfi_wide == 0 ? kPfiWideMax : c->lp_pfi_wide;
  }
  return 0;
}

bool use_pfi(const mgpu_ctx *c, const LpIO &io) {
  const bool shared = io.ws.head != nullptr && io.ws.s_head == 0 && io.ws.s_st == 0 &&
                      io.ws.s_d == 0 && io.ws.s_binv == 0 && io.ws_index == nullptr;
  bool wide;
  // K3P/K3PW take d from the warm start (bound LPs rebuild it from ocol); a
  // warm start without d for the loaded objective goes to K3 / K3L
  const bool has_d = io.ws.d != nullptr || io.obj_col != nullptr;
  return shared && has_d && io.wo_head == nullptr && pfi_cap(c, &wide) > 0;
}

int launch_lp(mgpu_ctx *c, const LpIO &io, const char *who) {
  if (use_pfi(c, io)) {
    // K3P / K3PW, then the dense K3 / K3L on exactly the nodes that filled
    // the eta file: it continues from the product form's basis and explicit
    // inverse (continuation slots), or restarts from the shared warm start
    // past the slot capacity
    bool wide = false;
    const int kcap = pfi_cap(c, &wide);
    const int m = c->lp.m, N = c->lp.n + c->lp.m;
    const size_t slot_bytes = (size_t)m * 4 + (size_t)N * 9 + (size_t)m * m * 8 + 48;
    // continuation slots for a quarter of the batch (at least 4096): 1-3 %
    // of the LPs fill the eta file on the hot path, so a slot per LP (35 KB
    // each at m = 64: 18 GB for 524 288 LPs) would be memory held for
    // nothing; overflows past the slots restart from the shared warm start
    // (the same optimum, more pivots)
    const size_t max_slots = kPfiOvfBytes / slot_bytes;
    size_t want = (size_t)io.batch / 4 > 4096 ? (size_t)io.batch / 4 : 4096;
    if (want > (size_t)io.batch) want = (size_t)io.batch;
    // basis warm starts (the tree's warm mode 2): an overflowing LP must go on
    // from ITS basis, as the oracle's product-form mode does.  Which
    // LPs overflow first is decided by the device's atomic order, so a
    // restart from the shared basis past the slots could not be restated:
    // one slot per LP, or the call fails
    if (io.path.k != nullptr) {
      if ((size_t)io.batch > max_slots)
        return fail(c, MGPU_ERR_NOMEM, "%s: %d basis-warm-started LPs need one continuation "
                    "slot each (%zu bytes), more than the %zu-byte budget", who, io.batch,
                    slot_bytes, (size_t)kPfiOvfBytes);
      want = (size_t)io.batch;
    }
    const int cap = want < max_slots ? (int)want : (int)max_slots;
    HIPCHK(c, c->pfi_ovf.ensure(((size_t)io.batch + 4) * sizeof(int32_t)));
    // (a node's basis difference handed on never exceeds the inherit cap,
    // <= kPathMax, whatever the eta cap)
    if (io.path.k != nullptr && (wide || kcap > kPfiBig))
      return fail(c, MGPU_ERR_ARG, "%s: path warm starts run on K3P (m <= 64) with an eta cap "
                  "<= %d", who, kPfiBig);
    const size_t sb_head = al16h((size_t)cap * m * 4), sb_st = al16h((size_t)cap * N),
                 sb_d = al16h((size_t)cap * N * 8), sb_binv = al16h((size_t)cap * m * m * 8),
                 sb_it = (size_t)cap * 4;
    HIPCHK(c, c->pfi_cont.ensure(sb_head + sb_st + sb_d + sb_binv + sb_it));
    // [0] overflow count, [1] K3P's next node, [2]/[3] the K3 follow-ups'
    int32_t *cnt = c->pfi_ovf.as<int32_t>();
    HIPCHK(c, hipMemsetAsync(cnt, 0, 4 * sizeof(int32_t), c->stream));
    PfiIO px{};
    px.kmax = kcap;
    HIPCHK(c, c->pfi_piv.ensure(sizeof(unsigned long long)));
    HIPCHK(c, hipMemsetAsync(c->pfi_piv.p, 0, sizeof(unsigned long long), c->stream));
    px.pivots = wide ? nullptr : c->pfi_piv.as<unsigned long long>();
    if (!wide && c->pfi_decide != nullptr) {   // the tree's decision in K3P's epilogue
      px.decide = 1;
      px.dec = *c->pfi_decide;
    }
    px.ovf_count = cnt;
    px.next = cnt + 1;
    px.ovf_list = cnt + 4;
    px.ovf_cap = cap;
    char *cp = c->pfi_cont.as<char>();
    px.c_head = (int32_t *)cp;
    px.c_st = (int8_t *)(cp + sb_head);
    px.c_d = (double *)(cp + sb_head + sb_st);
    px.c_binv = (double *)(cp + sb_head + sb_st + sb_d);
    px.c_iters = (int32_t *)(cp + sb_head + sb_st + sb_d + sb_binv);
    if (wide) {
      HIPCHK(c, launch_lp_pfiw(c->lp, io, px, c->num_cus, c->stream));
    } else {
      // every column's B0^{-1} a_q once per launch: headline K3P 13.8 ->
      // 13.4 ms (profiles/r04g)
      if (io.ws.binv != nullptr) {
        HIPCHK(c, c->pfi_t0.ensure((size_t)N * m * 8));
        HIPCHK(c, launch_pfi_t0(c->lp, io.ws.binv, c->pfi_t0.as<double>(), c->stream));
        px.t0 = c->pfi_t0.as<double>();
      }
      HIPCHK(c, launch_lp_pfi(c->lp, io, px, c->num_cus, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev8, c->stream));
    // K3L continuation: one HBM inverse slot per resident workgroup
    int lgrid = 0;
    if (wide) {
      lgrid = lp_large_grid(io.batch < cap ? io.batch : cap, c->lp.n, m, c->num_cus);
      HIPCHK(c, c->lp_slots.ensure((size_t)lgrid * m * m * sizeof(double) + 8));
      HIPCHK(c, lp_large_prepare());
    }
    auto dense = [&](const LpIO &d) -> hipError_t {
      return wide ? launch_lp_large(c->lp, d, c->lp_slots.as<double>(), lgrid, c->stream)
                  : launch_lp_dual(c->lp, d, c->num_cus, c->stream);
    };
    c->last_lp_pfi = true;
    LpIO io2 = io;
    io2.node_list = px.ovf_list;
    io2.node_count = px.ovf_count;
    io2.list_lo = 0;
    io2.list_hi = cap;
    io2.list_ws = 1;
    // the pivots each node already made: kmax for K3PW; K3P's own pivots per
    // slot (a path warm start's replayed pivots fill part of the eta file)
    io2.iter_base = px.kmax;
    io2.iter_base_list = wide ? nullptr : px.c_iters;
    io2.iter_limit = io.iter_limit;
    io2.ws = LpWarm{px.c_head, px.c_st, px.c_d, px.c_binv, m, N, N, (long)m * m};
    io2.next = cnt + 2;
    HIPCHK(c, dense(io2));
    if (io.batch > cap) {  // overflow beyond the slots: restart from the shared warm start
      LpIO io3 = io;
      io3.node_list = px.ovf_list;
      io3.node_count = px.ovf_count;
      io3.list_lo = cap;
      io3.list_hi = 0x7fffffff;
      io3.next = cnt + 3;
      HIPCHK(c, dense(io3));
    }
    if (px.decide) {   // the overflow list, after its dense continuation
      DecideIO d2 = px.dec;
      d2.node_list = px.ovf_list;
      d2.node_count = px.ovf_count;
      HIPCHK(c, launch_node_decide(c->lp, d2, c->stream));
      c->lp_decided = true;
    }
    return MGPU_OK;
  }
  c->last_lp_pfi = false;
  if (c->lp_variant == 3)
    return fail(c, MGPU_ERR_ARG, "%s: K3P/K3PW need a shared warm start, no warm-start "
                "output, m <= 128 and n + m <= %d", who, 64 * kPfiSlots);
  if (!use_large_lp(c)) {
    if (c->lp.m > kLpMaxM || lp_lds_bytes(c->lp.n, c->lp.m, c->lp.nnz) > 160 * 1024)
      return fail(c, MGPU_ERR_ARG, "%s: problem too large for K3 (m=%d)", who, c->lp.m);
    // dynamic node schedule: a counter of its own that the kernel leaves
    // zeroed (filled once, when allocated)
    if (c->lp_next3.p == nullptr) {
      HIPCHK(c, c->lp_next3.ensure(2 * sizeof(int32_t)));
      HIPCHK(c, hipMemsetAsync(c->lp_next3.p, 0, 2 * sizeof(int32_t), c->stream));
    }
    LpIO iod = io;
    iod.next = c->lp_next3.as<int32_t>();
    iod.next_exit = c->lp_next3.as<int32_t>() + 1;
    HIPCHK(c, launch_lp_dual(c->lp, iod, c->num_cus, c->stream));
    return MGPU_OK;
  }
  if (lp_large_lds_bytes(c->lp.n, c->lp.m) > (size_t)kLargeLdsMax)
    return fail(c, MGPU_ERR_ARG, "%s: n+m=%d too large for K3L's LDS state", who,
                c->lp.n + c->lp.m);
  const int grid = lp_large_grid(io.batch, c->lp.n, c->lp.m, c->num_cus);
  HIPCHK(c, c->lp_slots.ensure((size_t)grid * c->lp.m * c->lp.m * sizeof(double) + 8));
  HIPCHK(c, c->lp_next.ensure(sizeof(int32_t)));
  HIPCHK(c, hipMemsetAsync(c->lp_next.p, 0, sizeof(int32_t), c->stream));
  LpIO iod = io;
  iod.next = c->lp_next.as<int32_t>();
  HIPCHK(c, lp_large_prepare());
  (void)hipGetLastError();  // clear a stale error so the launch check is its own
  HIPCHK(c, launch_lp_large(c->lp, iod, c->lp_slots.as<double>(), grid, c->stream));
  return MGPU_OK;
}
}  // namespace

extern "C++" int launch_lp_nodes(mgpu_ctx *c, const LpIO &io) {
  return launch_lp(c, io, "lp batch");
}

// chained LPs (LpIO::chain_*) run on K3 only
extern "C++" bool lp_chain_ok(const mgpu_ctx *c) { return !use_large_lp(c); }

int mgpu_set_sb_chain(mgpu_ctx *c, int on) {
  if (!c) return MGPU_ERR_ARG;
  c->sb_chain = on != 0;
  return MGPU_OK;
}

int mgpu_lp_pfi_cap(mgpu_ctx *c) {
  if (!c) return MGPU_ERR_ARG;
  bool wide;
  return pfi_cap(c, &wide);
}

int mgpu_lp_solve_dev(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                      const int32_t *skip, const int32_t *ws_head, const int8_t *ws_st,
                      const double *ws_d, const double *ws_binv, int ws_shared, int iter_limit,
                      int32_t *status, double *obj, int32_t *iters, double *x,
                      int32_t *wo_head, int8_t *wo_st, double *wo_d, double *wo_binv) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve: bad argument");
  // ws_d may be null: the kernel then rebuilds the reduced costs of the warm
  // basis for the loaded objective (a basis saved under another objective)
  if (ws_head && (!ws_st || !ws_binv))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve: warm start needs head, st and binv");
  if (wo_head && (!wo_st || !wo_d || !wo_binv))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve: warm-start output needs all four arrays");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  LpIO io{};
  io.batch = batch;
  io.lb = lb;
  io.ub = ub;
  io.box_stride = n;
  io.skip = skip;
  io.ws.head = ws_head;
  io.ws.st = ws_st;
  io.ws.d = ws_d;
  io.ws.binv = ws_binv;
  io.ws.s_head = ws_shared ? 0 : m;
  io.ws.s_st = ws_shared ? 0 : N;
  io.ws.s_d = ws_shared ? 0 : N;
  io.ws.s_binv = ws_shared ? 0 : (long)m * m;
  io.iter_limit = lp_iter_limit(iter_limit);
  io.status = status;
  io.obj = obj;
  io.iters = iters;
  io.x = x;
  io.wo_head = wo_head;
  io.wo_st = wo_st;
  io.wo_d = wo_d;
  io.wo_binv = wo_binv;
  HIPCHK(c, hipEventRecord(c->ev2, c->stream));
  const int rc = launch_lp(c, io, "mgpu_lp_solve");
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipEventRecord(c->ev3, c->stream));
  return MGPU_OK;
}

// ---- device warm-start slots and the single-LP route ----------------------
// An LPEngine solves one LP at a time and keeps one warm start per tree node
// (HipLPEngine: getWarmStartCopy / loadFromWarmStart).  The warm starts live
// in device slots [head m | st n+m | d n+m | binv m*m] that K3 / K3L read and
// write in place; the host only moves slot ids.  The box goes in and the
// results come out through one pinned host block the kernel reads and writes
// directly (no copy engine round trips).
namespace {
constexpr int kWsChunkSlots = 256;
struct WsLayout {
  size_t st, d, binv, bytes;
};
WsLayout ws_layout(int n, int m) {
  const size_t N = (size_t)n + m;
  WsLayout L;
  L.st = al16h((size_t)m * 4);
  L.d = L.st + al16h(N);
  L.binv = L.d + al16h(N * 8);
  L.bytes = (L.binv + (size_t)m * m * 8 + 255) & ~(size_t)255;
  return L;
}
char *ws_slot(mgpu_ctx *c, int slot, int *n, int *m) {
  if (slot < 0) return nullptr;
  const size_t k = (size_t)slot / kWsChunkSlots, i = (size_t)slot % kWsChunkSlots;
  if (k >= c->ws_chunks.size() || !c->ws_chunks[k].base) return nullptr;
  const auto &ch = c->ws_chunks[k];
  *n = ch.n;
  *m = ch.m;
  return ch.base + i * ch.bytes;
}
}  // namespace

int mgpu_ws_alloc(mgpu_ctx *c, int *slot) {
  if (!c || !slot) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_ws_alloc: no problem loaded");
  const int n = c->lp.n, m = c->lp.m;
  for (size_t k = 0; k < c->ws_chunks.size(); ++k) {
    auto &ch = c->ws_chunks[k];
    if (ch.n == n && ch.m == m && !ch.free.empty()) {
      *slot = (int)k * kWsChunkSlots + ch.free.back();
      ch.free.pop_back();
      return MGPU_OK;
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  mgpu_ctx::WsChunk ch;
  ch.n = n;
  ch.m = m;
  ch.cap = kWsChunkSlots;
  ch.bytes = ws_layout(n, m).bytes;
  HIPCHK(c, hipMalloc((void **)&ch.base, ch.bytes * ch.cap));
  note_dev_alloc(ch.bytes * ch.cap);
  ch.free.reserve(ch.cap);
  for (int i = ch.cap - 1; i >= 1; --i) ch.free.push_back(i);
  size_t k = c->ws_chunks.size();
  for (size_t t = 0; t < c->ws_chunks.size(); ++t)  // reuse a released chunk index
    if (!c->ws_chunks[t].base) { k = t; break; }
  if (k == c->ws_chunks.size()) c->ws_chunks.emplace_back();
  c->ws_chunks[k] = std::move(ch);
  *slot = (int)k * kWsChunkSlots;
  return MGPU_OK;
}

int mgpu_ws_free(mgpu_ctx *c, int slot) {
  if (!c || slot < 0) return MGPU_ERR_ARG;
  const size_t k = (size_t)slot / kWsChunkSlots;
  if (k >= c->ws_chunks.size() || !c->ws_chunks[k].base)
    return fail(c, MGPU_ERR_ARG, "mgpu_ws_free: bad slot %d", slot);
  c->ws_chunks[k].free.push_back(slot % kWsChunkSlots);
  return MGPU_OK;
}

int mgpu_ws_read(mgpu_ctx *c, int slot, int32_t *head, int8_t *st, double *d, double *binv) {
  if (!c) return MGPU_ERR_ARG;
  int n = 0, m = 0;
  char *p = ws_slot(c, slot, &n, &m);
  if (!p) return fail(c, MGPU_ERR_ARG, "mgpu_ws_read: bad slot %d", slot);
  const WsLayout L = ws_layout(n, m);
  const size_t N = (size_t)n + m;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (head) HIPCHK(c, hipMemcpy(head, p, (size_t)m * 4, hipMemcpyDeviceToHost));
  if (st) HIPCHK(c, hipMemcpy(st, p + L.st, N, hipMemcpyDeviceToHost));
  if (d) HIPCHK(c, hipMemcpy(d, p + L.d, N * 8, hipMemcpyDeviceToHost));
  if (binv) HIPCHK(c, hipMemcpy(binv, p + L.binv, (size_t)m * m * 8, hipMemcpyDeviceToHost));
  return MGPU_OK;
}

int mgpu_ws_write(mgpu_ctx *c, int slot, const int32_t *head, const int8_t *st,
                  const double *d, const double *binv) {
  if (!c || !head || !st || !binv) return MGPU_ERR_ARG;
  int n = 0, m = 0;
  char *p = ws_slot(c, slot, &n, &m);
  if (!p) return fail(c, MGPU_ERR_ARG, "mgpu_ws_write: bad slot %d", slot);
  const WsLayout L = ws_layout(n, m);
  const size_t N = (size_t)n + m;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(p, head, (size_t)m * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(p + L.st, st, N, hipMemcpyHostToDevice));
  if (d) HIPCHK(c, hipMemcpy(p + L.d, d, N * 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(p + L.binv, binv, (size_t)m * m * 8, hipMemcpyHostToDevice));
  return MGPU_OK;
}

int mgpu_lp_solve1(mgpu_ctx *c, const double *lb, const double *ub, int ws_in, int ws_d,
                   int ws_out, int iter_limit, int32_t *status, double *obj, int32_t *iters,
                   double *x, double *rc) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve1: no problem loaded");
  if (!lb || !ub || !status || !obj || !iters)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve1: bad argument");
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  int sn = 0, sm = 0;
  char *pin_ws = ws_in >= 0 ? ws_slot(c, ws_in, &sn, &sm) : nullptr;
  if (ws_in >= 0 && (!pin_ws || sn != n || sm != m))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve1: warm-start slot %d is not for this problem",
                ws_in);
  char *pout_ws = ws_out >= 0 ? ws_slot(c, ws_out, &sn, &sm) : nullptr;
  if (ws_out >= 0 && (!pout_ws || sn != n || sm != m))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve1: output slot %d is not for this problem",
                ws_out);
  if (ws_in >= 0 && ws_in == ws_out)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve1: input and output slot are the same");
  HIPCHK(c, hipSetDevice(c->device));
  // pinned block: [lb n][ub n][x n][rc N][obj][status, iters]
  const size_t o_ub = (size_t)n * 8, o_x = 2 * o_ub, o_rc = 3 * o_ub, o_obj = o_rc + (size_t)N * 8,
               o_st = o_obj + 8, bytes = o_st + 8;
  if (c->lp1_pin_bytes < bytes) {
    if (c->lp1_pin) (void)hipHostFree(c->lp1_pin);
    c->lp1_pin = nullptr;
    c->lp1_pin_bytes = 0;
    HIPCHK(c, hipHostMalloc((void **)&c->lp1_pin, bytes, hipHostMallocDefault));
    c->lp1_pin_bytes = bytes;
    note_dev_alloc(bytes);   // pinned host memory counts too
  }
  // (a staged variant, one H2D of the box and one D2H of the results, measured
  // 46 vs 44 us per LP through Python: the copy commands cost more than the
  // kernel's reads over the link)
  char *hp = c->lp1_pin, *dp = nullptr;
  HIPCHK(c, hipHostGetDevicePointer((void **)&dp, hp, 0));
  std::memcpy(hp, lb, (size_t)n * 8);
  std::memcpy(hp + o_ub, ub, (size_t)n * 8);
  LpIO io{};
  io.batch = 1;
  io.lb = (const double *)dp;
  io.ub = (const double *)(dp + o_ub);
  io.box_stride = n;
  if (pin_ws) {
    const WsLayout L = ws_layout(n, m);
    io.ws.head = (const int32_t *)pin_ws;
    io.ws.st = (const int8_t *)(pin_ws + L.st);
    io.ws.d = ws_d ? (const double *)(pin_ws + L.d) : nullptr;
    io.ws.binv = (const double *)(pin_ws + L.binv);
  }
  if (pout_ws) {
    const WsLayout L = ws_layout(n, m);
    io.wo_head = (int32_t *)pout_ws;
    io.wo_st = (int8_t *)(pout_ws + L.st);
    io.wo_d = (double *)(pout_ws + L.d);
    io.wo_binv = (double *)(pout_ws + L.binv);
  }
  io.iter_limit = lp_iter_limit(iter_limit);
  io.status = (int32_t *)(dp + o_st);
  io.iters = (int32_t *)(dp + o_st + 4);
  io.obj = (double *)(dp + o_obj);
  io.x = (double *)(dp + o_x);
  io.rc = (double *)(dp + o_rc);
  if (!use_large_lp(c)) {  // one workgroup, static schedule: nothing to reset
    if (c->lp.m > kLpMaxM || lp_lds_bytes(c->lp.n, c->lp.m, c->lp.nnz) > 160 * 1024)
      return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve1: problem too large for K3 (m=%d)", m);
    HIPCHK(c, launch_lp_dual(c->lp, io, c->num_cus, c->stream));
  } else {
    const int rc2 = launch_lp(c, io, "mgpu_lp_solve1");
    if (rc2 != MGPU_OK) return rc2;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *status = *(const int32_t *)(hp + o_st);
  *iters = *(const int32_t *)(hp + o_st + 4);
  *obj = *(const double *)(hp + o_obj);
  if (x) std::memcpy(x, hp + o_x, (size_t)n * 8);
  if (rc) std::memcpy(rc, hp + o_rc, (size_t)N * 8);
  return MGPU_OK;
}

int mgpu_lp_bound_dev(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                      const int32_t *obj_col, const double *obj_sign, const int32_t *ws_head,
                      const int8_t *ws_st, const double *ws_binv, int iter_limit,
                      int32_t *status, double *obj, int32_t *iters, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_bound: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !obj_col || !obj_sign || !status || !obj ||
                                  !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_bound: bad argument");
  if (ws_head && (!ws_st || !ws_binv))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_bound: warm start needs head, st and binv");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  LpIO io{};
  io.batch = batch;
  io.lb = lb;
  io.ub = ub;
  io.box_stride = 0;  // one box (the relaxation's) for every bound LP
  io.obj_col = obj_col;
  io.obj_sign = obj_sign;
  io.ws.head = ws_head;
  io.ws.st = ws_st;
  io.ws.d = nullptr;  // reduced costs are rebuilt for each objective
  io.ws.binv = ws_binv;
  io.iter_limit = lp_iter_limit(iter_limit);
  io.status = status;
  io.obj = obj;
  io.iters = iters;
  io.x = x;
  HIPCHK(c, hipEventRecord(c->ev2, c->stream));
  const int rc = launch_lp(c, io, "mgpu_lp_bound");
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipEventRecord(c->ev3, c->stream));
  return MGPU_OK;
}

int mgpu_lp_bound(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                  const int32_t *obj_col, const double *obj_sign, const int32_t *ws_head,
                  const int8_t *ws_st, const double *ws_binv, int iter_limit, int32_t *status,
                  double *obj, int32_t *iters, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_bound: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !obj_col || !obj_sign || !status || !obj ||
                                  !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_bound: bad argument");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  const size_t nb = (size_t)n * sizeof(double);
  HIPCHK(c, c->lp_lb.ensure(nb));
  HIPCHK(c, c->lp_ub.ensure(nb));
  const size_t sign_off = ((size_t)batch * 4 + 7) & ~(size_t)7;
  HIPCHK(c, c->lp_skip.ensure(sign_off + (size_t)batch * 8));  // cols, then signs
  HIPCHK(c, c->lp_st.ensure((size_t)batch * 4));
  HIPCHK(c, c->lp_obj.ensure((size_t)batch * 8));
  HIPCHK(c, c->lp_it.ensure((size_t)batch * 4));
  if (x) HIPCHK(c, c->lp_x.ensure((size_t)batch * nb));
  int32_t *d_col = c->lp_skip.as<int32_t>();
  double *d_sign = reinterpret_cast<double *>(c->lp_skip.as<char>() + sign_off);
  HIPCHK(c, hipMemcpyAsync(c->lp_lb.p, lb, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->lp_ub.p, ub, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_col, obj_col, (size_t)batch * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_sign, obj_sign, (size_t)batch * 8, hipMemcpyHostToDevice, c->stream));
  if (ws_head) {
    HIPCHK(c, c->lp_wh.ensure((size_t)m * 4 + 4));
    HIPCHK(c, c->lp_wst.ensure((size_t)N));
    HIPCHK(c, c->lp_wb.ensure((size_t)m * m * 8 + 8));
    HIPCHK(c, hipMemcpyAsync(c->lp_wh.p, ws_head, (size_t)m * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->lp_wst.p, ws_st, (size_t)N, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->lp_wb.p, ws_binv, (size_t)m * m * 8, hipMemcpyHostToDevice,
                             c->stream));
  }
  int rc = mgpu_lp_bound_dev(c, batch, c->lp_lb.as<double>(), c->lp_ub.as<double>(), d_col,
                             d_sign, ws_head ? c->lp_wh.as<int32_t>() : nullptr,
                             ws_head ? c->lp_wst.as<int8_t>() : nullptr,
                             ws_head ? c->lp_wb.as<double>() : nullptr, iter_limit,
                             c->lp_st.as<int32_t>(), c->lp_obj.as<double>(),
                             c->lp_it.as<int32_t>(), x ? c->lp_x.as<double>() : nullptr);
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(status, c->lp_st.p, (size_t)batch * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(obj, c->lp_obj.p, (size_t)batch * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(iters, c->lp_it.p, (size_t)batch * 4, hipMemcpyDeviceToHost, c->stream));
  if (x)
    HIPCHK(c, hipMemcpyAsync(x, c->lp_x.p, (size_t)batch * nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

int mgpu_lp_solve(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                  const int32_t *skip, const int32_t *ws_head, const int8_t *ws_st,
                  const double *ws_d, const double *ws_binv, int ws_shared, int iter_limit,
                  int32_t *status, double *obj, int32_t *iters, double *x, int32_t *wo_head,
                  int8_t *wo_st, double *wo_d, double *wo_binv) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve: bad argument");
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
  if (skip) HIPCHK(c, h2d(c->lp_skip, skip, B * 4));
  if (ws_head) {
    HIPCHK(c, h2d(c->lp_wh, ws_head, wsB * m * 4));
    HIPCHK(c, h2d(c->lp_wst, ws_st, wsB * N));
    if (ws_d) HIPCHK(c, h2d(c->lp_wd, ws_d, wsB * N * 8));
    HIPCHK(c, h2d(c->lp_wb, ws_binv, wsB * m * m * 8));
  }
  HIPCHK(c, c->lp_st.ensure(B * 4));
  HIPCHK(c, c->lp_obj.ensure(B * 8));
  HIPCHK(c, c->lp_it.ensure(B * 4));
  if (x) HIPCHK(c, c->lp_x.ensure(B * n * 8));
  if (wo_head) {
    HIPCHK(c, c->lp_oh.ensure(B * m * 4 + 16));
    HIPCHK(c, c->lp_ost.ensure(B * N + 16));
    HIPCHK(c, c->lp_od.ensure(B * N * 8 + 16));
    HIPCHK(c, c->lp_ob.ensure(B * m * m * 8 + 16));
  }
  int rc = mgpu_lp_solve_dev(
      c, batch, c->lp_lb.as<double>(), c->lp_ub.as<double>(),
      skip ? c->lp_skip.as<int32_t>() : nullptr, ws_head ? c->lp_wh.as<int32_t>() : nullptr,
      ws_head ? c->lp_wst.as<int8_t>() : nullptr, ws_d ? c->lp_wd.as<double>() : nullptr,
      ws_head ? c->lp_wb.as<double>() : nullptr, ws_shared, iter_limit, c->lp_st.as<int32_t>(),
      c->lp_obj.as<double>(), c->lp_it.as<int32_t>(), x ? c->lp_x.as<double>() : nullptr,
      wo_head ? c->lp_oh.as<int32_t>() : nullptr, wo_head ? c->lp_ost.as<int8_t>() : nullptr,
      wo_head ? c->lp_od.as<double>() : nullptr, wo_head ? c->lp_ob.as<double>() : nullptr);
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(status, c->lp_st.p, B * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(obj, c->lp_obj.p, B * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(iters, c->lp_it.p, B * 4, hipMemcpyDeviceToHost, s));
  if (x) HIPCHK(c, hipMemcpyAsync(x, c->lp_x.p, B * n * 8, hipMemcpyDeviceToHost, s));
  if (wo_head) {
    HIPCHK(c, hipMemcpyAsync(wo_head, c->lp_oh.p, B * m * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(wo_st, c->lp_ost.p, B * N, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(wo_d, c->lp_od.p, B * N * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(wo_binv, c->lp_ob.p, B * m * m * 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(c, hipStreamSynchronize(s));
  return MGPU_OK;
}

int mgpu_lp_solve_path_dev(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                           const int32_t *skip, const int32_t *ws_head, const int8_t *ws_st,
                           const double *ws_d, const double *ws_binv, const int32_t *k_in,
                           const uint32_t *path_in, const int8_t *st_in, int inherit,
                           int iter_limit, int32_t *status, double *obj, int32_t *iters,
                           double *x, int32_t *k_out, uint32_t *path_out, int8_t *st_out) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_path: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters || !ws_head ||
                                  !ws_st || !ws_d || !ws_binv || !k_in || !path_in ||
                                  !st_in)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_path: bad argument");
  if (k_out && (!path_out || !st_out))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_path: path output needs k, path and st");
  if (inherit < 0 || inherit > MGPU_PATH_MAX)
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_path: inherit must be in 0..%d", MGPU_PATH_MAX);
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  LpIO io{};
  io.batch = batch;
  io.lb = lb;
  io.ub = ub;
  io.box_stride = c->lp.n;
  io.skip = skip;
  io.ws.head = ws_head;
  io.ws.st = ws_st;
  io.ws.d = ws_d;
  io.ws.binv = ws_binv;
  io.iter_limit = lp_iter_limit(iter_limit);
  io.status = status;
  io.obj = obj;
  io.iters = iters;
  io.x = x;
  io.path.k = k_in;
  io.path.path = path_in;
  io.path.st = st_in;
  io.path.k_out = k_out;
  io.path.path_out = path_out;
  io.path.st_out = st_out;
  io.path.inherit = inherit;
  if (!use_pfi(c, io))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_path: path warm starts need K3P (m <= 64, "
                "n + m <= %d, eta cap > 0)", 64 * kPfiSlots);
  HIPCHK(c, hipEventRecord(c->ev2, c->stream));
  const int rc = launch_lp(c, io, "mgpu_lp_solve_path");
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipEventRecord(c->ev3, c->stream));
  return MGPU_OK;
}

int mgpu_lp_solve_path(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                       const int32_t *ws_head, const int8_t *ws_st, const double *ws_d,
                       const double *ws_binv, const int32_t *k_in, const uint32_t *path_in,
                       const int8_t *st_in, int inherit, int iter_limit, int32_t *status,
                       double *obj, int32_t *iters, double *x, int32_t *k_out,
                       uint32_t *path_out, int8_t *st_out) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_lp_solve_path: no problem loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters || !ws_head ||
                                  !ws_st || !ws_d || !ws_binv || !k_in || !path_in || !st_in)))
    return fail(c, MGPU_ERR_ARG, "mgpu_lp_solve_path: bad argument");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = c->lp.n, m = c->lp.m, N = n + m;
  const size_t B = (size_t)batch, P = MGPU_PATH_MAX;
  hipStream_t s = c->stream;
  DevBuf buf;  // per-call workspace
  const size_t o_lb = 0, o_ub = o_lb + B * n * 8, o_wh = o_ub + B * n * 8,
               o_wst = o_wh + al16h((size_t)m * 4), o_wd = o_wst + al16h((size_t)N),
               o_wb = o_wd + (size_t)N * 8, o_k = o_wb + (size_t)m * m * 8,
               o_p = o_k + al16h(B * 4), o_st = o_p + B * P * 4, o_ost = o_st + al16h(B * N),
               o_ok = o_ost + al16h(B * N), o_op = o_ok + al16h(B * 4),
               o_stt = o_op + B * P * 4, o_obj = o_stt + al16h(B * 4),
               o_it = o_obj + B * 8, o_x = o_it + al16h(B * 4), total = o_x + B * n * 8;
  HIPCHK(c, buf.ensure(total));
  char *d = buf.as<char>();
  auto h2d = [&](size_t off, const void *src, size_t bytes) {
    return hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, s);
  };
  HIPCHK(c, h2d(o_lb, lb, B * n * 8));
  HIPCHK(c, h2d(o_ub, ub, B * n * 8));
  HIPCHK(c, h2d(o_wh, ws_head, (size_t)m * 4));
  HIPCHK(c, h2d(o_wst, ws_st, (size_t)N));
  HIPCHK(c, h2d(o_wd, ws_d, (size_t)N * 8));
  HIPCHK(c, h2d(o_wb, ws_binv, (size_t)m * m * 8));
  HIPCHK(c, h2d(o_k, k_in, B * 4));
  HIPCHK(c, h2d(o_p, path_in, B * P * 4));
  HIPCHK(c, h2d(o_st, st_in, B * N));
  int rc = mgpu_lp_solve_path_dev(
      c, batch, (double *)(d + o_lb), (double *)(d + o_ub), nullptr, (int32_t *)(d + o_wh),
      (int8_t *)(d + o_wst), (double *)(d + o_wd), (double *)(d + o_wb), (int32_t *)(d + o_k),
      (uint32_t *)(d + o_p), (int8_t *)(d + o_st), inherit, iter_limit, (int32_t *)(d + o_stt),
      (double *)(d + o_obj), (int32_t *)(d + o_it), x ? (double *)(d + o_x) : nullptr,
      k_out ? (int32_t *)(d + o_ok) : nullptr, k_out ? (uint32_t *)(d + o_op) : nullptr,
      k_out ? (int8_t *)(d + o_ost) : nullptr);
  if (rc != MGPU_OK) return rc;
  auto d2h = [&](void *dst, size_t off, size_t bytes) {
    return hipMemcpyAsync(dst, d + off, bytes, hipMemcpyDeviceToHost, s);
  };
  HIPCHK(c, d2h(status, o_stt, B * 4));
  HIPCHK(c, d2h(obj, o_obj, B * 8));
  HIPCHK(c, d2h(iters, o_it, B * 4));
  if (x) HIPCHK(c, d2h(x, o_x, B * n * 8));
  if (k_out) {
    HIPCHK(c, d2h(k_out, o_ok, B * 4));
    if (path_out) HIPCHK(c, d2h(path_out, o_op, B * P * 4));
    if (st_out) HIPCHK(c, d2h(st_out, o_ost, B * N));
  }
  HIPCHK(c, hipStreamSynchronize(s));
  return MGPU_OK;
}

int mgpu_node_decide_dev(mgpu_ctx *c, int batch, const int32_t *fbbt_infeas,
                         const int32_t *status, const double *obj, const double *x,
                         double incumbent, double abs_tol, double rel_tol, double cutoff,
                         double int_tol, int32_t *decision, double *inf_meas,
                         double *cand_obj) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->loaded) return fail(c, MGPU_ERR_STATE, "mgpu_node_decide: no problem loaded");
  if (batch < 0 || (batch > 0 && (!status || !obj || !x || !decision)))
    return fail(c, MGPU_ERR_ARG, "mgpu_node_decide: bad argument");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  DecideIO io{};
  io.batch = batch;
  io.fbbt_infeas = fbbt_infeas;
  io.status = status;
  io.obj = obj;
  io.x = x;
  io.incumbent = incumbent;
  io.abs_tol = abs_tol;
  io.rel_tol = rel_tol;
  io.cutoff = cutoff;
  io.int_tol = int_tol;
  io.decision = decision;
  io.inf_meas = inf_meas;
  io.cand_obj = cand_obj;
  HIPCHK(c, launch_node_decide(c->lp, io, c->stream));
  return MGPU_OK;
}

}  // extern "C"
