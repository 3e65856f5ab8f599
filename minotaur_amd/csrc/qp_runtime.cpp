// Host runtime of the batched QP relaxation solve (K5, qp_kkt.hip): problem
// load (padding to 16-multiples), per-batch workspaces, and the interior
// point iteration loop (include/mgpu.h: mgpu_load_qp, mgpu_qp_solve[_dev]).
//
// Replaces BqpdEngine::solve's per-node QP (src/interfaces/BqpdEngine.cpp:
// 449-534, driven by QPDRelaxer / QPDProcessor) for a batch of node boxes.
#include <cmath>
#include <cstring>

#include "ctx.h"
#include "qp_internal.h"

struct QpState {
  DevQP dq{};
  int n = 0, m = 0;
  DevBuf Q, c, A, AT, b;
  DevBuf l, u, x, zl, zu, y, rd, rp, K, W, WT, M, done, iters, status, obj;
  int maxB = 0;
  DevBuf h_l, h_u, h_st, h_obj, h_it, h_x;  // host-path device copies
  DevBuf f_mask, f_st, f_obj, f_it;          // the tree's feasibility LPs
  std::vector<hipEvent_t> kev;               // mgpu_set_qp_ktime: 4 per iteration
  void release() {
    for (hipEvent_t e : kev) (void)hipEventDestroy(e);
    kev.clear();
    for (DevBuf *p : {&Q, &c, &A, &AT, &b, &l, &u, &x, &zl, &zu, &y, &rd, &rp, &K, &W, &WT, &M,
                      &done, &iters, &status, &obj, &h_l, &h_u, &h_st, &h_obj, &h_it, &h_x,
                      &f_mask, &f_st, &f_obj, &f_it})
      p->release();
  }
};

void qp_state_free(mgpu_ctx *c) {
  if (c && c->qp) {
    c->qp->release();
    delete c->qp;
    c->qp = nullptr;
  }
}

namespace {

__global__ void pad_boxes(const double *l, const double *u, int n, int np, int B, double *pl,
                          double *pu) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)B * np) return;
  const size_t b = e / np;
  const int j = (int)(e % np);
  pl[e] = j < n ? l[b * n + j] : 0.0;
  pu[e] = j < n ? u[b * n + j] : 0.0;
}

__global__ void unpad_x(const double *px, int n, int np, int B, double *x) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)B * n) return;
  x[e] = px[(e / n) * np + e % n];
}

// the tree's nodes whose QP neither converged nor was proven infeasible
__global__ void qp_unsettled(const int32_t *st, int B, int32_t *skip) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) skip[b] = st[b] != 6;
}

// their feasibility LP decides: infeasible rows -> ProvenInfeasible; a
// feasible QP the interior point did not solve -> EngineUnknownStatus
__global__ void qp_settle(int32_t *st, double *obj, const int32_t *lst, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || st[b] != 6) return;
  st[b] = lst[b] == 2 ? 2 : 12;
  obj[b] = INFINITY;
}

int ensure_qp_batch(mgpu_ctx *c, QpState &s, int B) {
  if (B <= s.maxB) return MGPU_OK;
  const size_t np = s.dq.np, mp = s.dq.mp;
  for (DevBuf *p : {&s.l, &s.u, &s.x, &s.zl, &s.zu, &s.rd}) HIPCHK(c, p->ensure((size_t)B * np * 8));
  HIPCHK(c, s.y.ensure((size_t)B * mp * 8));
  HIPCHK(c, s.rp.ensure((size_t)B * mp * 8));
  HIPCHK(c, s.K.ensure((size_t)B * np * np * 8));
  HIPCHK(c, s.W.ensure((size_t)B * np * mp * 8));
  HIPCHK(c, s.WT.ensure((size_t)B * np * mp * 8));
  HIPCHK(c, s.M.ensure((size_t)B * mp * mp * 8));
  for (DevBuf *p : {&s.done, &s.iters, &s.status}) HIPCHK(c, p->ensure((size_t)B * 4));
  HIPCHK(c, s.obj.ensure((size_t)B * 8));
  s.maxB = B;
  return MGPU_OK;
}

}  // namespace

// The batch solve with an optional skip list (the batched tree: nodes its
// presolve found infeasible are not solved).
int qp_solve_nodes(mgpu_ctx *c, int batch, const double *lb, const double *ub,
                   const int32_t *skip, int maxit, int32_t *status, double *obj, int32_t *iters,
                   double *x) {
  QpState &s = *c->qp;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = ensure_qp_batch(c, s, batch);
  if (rc != MGPU_OK) return rc;
  const int np = s.dq.np;
  QpWork w{};
  w.B = batch;
  w.skip = skip;
  w.l = s.l.as<double>();
  w.u = s.u.as<double>();
  w.x = s.x.as<double>();
  w.zl = s.zl.as<double>();
  w.zu = s.zu.as<double>();
  w.y = s.y.as<double>();
  w.rd = s.rd.as<double>();
  w.rp = s.rp.as<double>();
  w.K = s.K.as<double>();
  w.W = s.W.as<double>();
  w.WT = s.WT.as<double>();
  w.M = s.M.as<double>();
  w.done = s.done.as<int32_t>();
  w.iters = s.iters.as<int32_t>();
  w.status = s.status.as<int32_t>();
  w.obj = s.obj.as<double>();
  const size_t tot = (size_t)batch * np;
  hipLaunchKernelGGL(pad_boxes, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, lb,
                     ub, s.n, np, batch, w.l, w.u);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev6, c->stream));
  HIPCHK(c, launch_qp_init(s.dq, w, c->stream));
  const int lim = maxit > 0 ? maxit : 80;
  std::vector<int32_t> hd(batch);
  if (c->qp_ktime && s.kev.size() < (size_t)4 * lim) {
    const size_t have = s.kev.size();
    s.kev.resize((size_t)4 * lim, nullptr);
    for (size_t e = have; e < s.kev.size(); ++e) HIPCHK(c, hipEventCreate(&s.kev[e]));
  }
  int nit = 0;
  for (int it = 0; it < lim; ++it) {
    HIPCHK(c, launch_qp_iteration(s.dq, w, c->stream, c->qp_ktime ? &s.kev[(size_t)4 * it] : nullptr));
    nit = it + 1;
    if (it % 4 == 3) {  // stop once every node has converged
      HIPCHK(c, hipMemcpyAsync(hd.data(), w.done, (size_t)batch * 4, hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      bool all = true;
      for (int b = 0; b < batch && all; ++b) all = hd[b] != 0;
      if (all) break;
    }
  }
  // a final residual pass marks nodes that converged on the last step
  HIPCHK(c, launch_qp_iteration_check(s.dq, w, c->stream));
  HIPCHK(c, launch_qp_final(s.dq, w, c->stream));
  HIPCHK(c, hipEventRecord(c->ev7, c->stream));
  if (c->qp_ktime) {   // per-kernel sums over the iterations (measurement mode)
    HIPCHK(c, hipEventSynchronize(s.kev[(size_t)4 * nit - 1]));
    for (int k = 0; k < 3; ++k) c->last_qp_kms[k] = 0.0;
    for (int it = 0; it < nit; ++it)
      for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, s.kev[(size_t)4 * it + k], s.kev[(size_t)4 * it + k + 1]));
        c->last_qp_kms[k] += ms;
      }
  }
  HIPCHK(c, hipMemcpyAsync(status, w.status, (size_t)batch * 4, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(obj, w.obj, (size_t)batch * 8, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(iters, w.iters, (size_t)batch * 4, hipMemcpyDeviceToDevice, c->stream));
  if (x) {
    const size_t tn = (size_t)batch * s.n;
    hipLaunchKernelGGL(unpad_x, dim3((unsigned)((tn + 255) / 256)), dim3(256), 0, c->stream, w.x,
                       s.n, np, batch, x);
    HIPCHK(c, hipGetLastError());
  }
  if (skip != nullptr) {
    // the batched tree: a node QP still unsettled after the iteration limit
    // (no convergence, no Farkas ray) gets a phase-1 answer from the loaded
    // rows: the LP min 0 over the node box (K3 / K3L from the slack basis),
    // as BQPD's own phase 1 would report an infeasible node QP
    const unsigned g = (unsigned)((batch + 255) / 256);
    for (DevBuf *p : {&s.f_mask, &s.f_st, &s.f_it}) HIPCHK(c, p->ensure((size_t)batch * 4));
    HIPCHK(c, s.f_obj.ensure((size_t)batch * 8));
    hipLaunchKernelGGL(qp_unsettled, dim3(g), dim3(256), 0, c->stream, status, batch,
                       s.f_mask.as<int32_t>());
    HIPCHK(c, hipGetLastError());
    int rc2 = mgpu_lp_solve_dev(c, batch, lb, ub, s.f_mask.as<int32_t>(), nullptr, nullptr,
                                nullptr, nullptr, 1, 0, s.f_st.as<int32_t>(),
                                s.f_obj.as<double>(), s.f_it.as<int32_t>(), nullptr, nullptr,
                                nullptr, nullptr, nullptr);
    if (rc2 != MGPU_OK) return rc2;
    hipLaunchKernelGGL(qp_settle, dim3(g), dim3(256), 0, c->stream, status, obj,
                       s.f_st.as<int32_t>(), batch);
    HIPCHK(c, hipGetLastError());
  }
  return MGPU_OK;
}

extern "C" {

int mgpu_load_qp(mgpu_ctx *c, int n, int m, const double *Q, const double *cvec, double k,
                 const double *A, const double *b) {
  if (!c) return MGPU_ERR_ARG;
  if (n <= 0 || n > 2048 || m < 0 || m > 64 || !Q || !cvec || (m > 0 && (!A || !b)))
    return fail(c, MGPU_ERR_ARG, "mgpu_load_qp: bad argument (n <= 2048 columns, m <= 64 rows "
                "supported)");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  qp_state_free(c);
  QpState *s = new QpState();
  c->qp = s;
  const int np = (n + 15) / 16 * 16, mp = m > 0 ? (m + 15) / 16 * 16 : 16;
  std::vector<double> hQ((size_t)np * np, 0.0), hc(np, 0.0), hA((size_t)mp * np, 0.0),
      hAT((size_t)np * mp, 0.0), hb(mp, 0.0);
  double cmax = 0.0, bmax = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) hQ[(size_t)i * np + j] = 0.5 * (Q[(size_t)i * n + j] + Q[(size_t)j * n + i]);
  for (int j = 0; j < n; ++j) {
    hc[j] = cvec[j];
    cmax = std::fmax(cmax, std::fabs(cvec[j]));
  }
  for (int i = 0; i < m; ++i) {
    hb[i] = b[i];
    bmax = std::fmax(bmax, std::fabs(b[i]));
    for (int j = 0; j < n; ++j) {
      hA[(size_t)i * np + j] = A[(size_t)i * n + j];
      hAT[(size_t)j * mp + i] = A[(size_t)i * n + j];
    }
  }
  HIPCHK(c, upload(s->Q, hQ.data(), hQ.size()));
  HIPCHK(c, upload(s->c, hc.data(), hc.size()));
  HIPCHK(c, upload(s->A, hA.data(), hA.size()));
  HIPCHK(c, upload(s->AT, hAT.data(), hAT.size()));
  HIPCHK(c, upload(s->b, hb.data(), hb.size()));
  s->n = n;
  s->m = m;
  DevQP &d = s->dq;
  d.n = n;
  d.m = m;
  d.np = np;
  d.mp = mp;
  d.Q = s->Q.as<double>();
  d.c = s->c.as<double>();
  d.A = s->A.as<double>();
  d.AT = s->AT.as<double>();
  d.b = s->b.as<double>();
  d.k = k;
  d.tp = 1e-9 * (1.0 + bmax);  // oracle/qp_ipm.py TOL_P, TOL_D
  d.td = 1e-9 * (1.0 + cmax);
  return MGPU_OK;
}

int mgpu_qp_solve_dev(mgpu_ctx *c, int batch, const double *lb, const double *ub, int maxit,
                      int32_t *status, double *obj, int32_t *iters, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->qp) return fail(c, MGPU_ERR_STATE, "mgpu_qp_solve: no QP loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_qp_solve: bad argument");
  if (batch == 0) return MGPU_OK;
  return qp_solve_nodes(c, batch, lb, ub, nullptr, maxit, status, obj, iters, x);
}

int mgpu_qp_solve(mgpu_ctx *c, int batch, const double *lb, const double *ub, int maxit,
                  int32_t *status, double *obj, int32_t *iters, double *x) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->qp) return fail(c, MGPU_ERR_STATE, "mgpu_qp_solve: no QP loaded");
  if (batch < 0 || (batch > 0 && (!lb || !ub || !status || !obj || !iters)))
    return fail(c, MGPU_ERR_ARG, "mgpu_qp_solve: bad argument");
  if (batch == 0) return MGPU_OK;
  QpState &s = *c->qp;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t nb = (size_t)batch * s.n * 8;
  HIPCHK(c, s.h_l.ensure(nb));
  HIPCHK(c, s.h_u.ensure(nb));
  HIPCHK(c, s.h_x.ensure(nb));
  HIPCHK(c, s.h_st.ensure((size_t)batch * 4));
  HIPCHK(c, s.h_it.ensure((size_t)batch * 4));
  HIPCHK(c, s.h_obj.ensure((size_t)batch * 8));
  HIPCHK(c, hipMemcpyAsync(s.h_l.p, lb, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(s.h_u.p, ub, nb, hipMemcpyHostToDevice, c->stream));
  int rc = mgpu_qp_solve_dev(c, batch, s.h_l.as<double>(), s.h_u.as<double>(), maxit,
                             s.h_st.as<int32_t>(), s.h_obj.as<double>(), s.h_it.as<int32_t>(),
                             x ? s.h_x.as<double>() : nullptr);
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(status, s.h_st.p, (size_t)batch * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(obj, s.h_obj.p, (size_t)batch * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(iters, s.h_it.p, (size_t)batch * 4, hipMemcpyDeviceToHost, c->stream));
  if (x) HIPCHK(c, hipMemcpyAsync(x, s.h_x.p, nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

}  // extern "C"
