// Host runtime of the quadratic node FBBT (K2): problem load, the host-side
// compilation of tightenQuad_'s per-function term programs, and the C-ABI
// wrappers (include/mgpu.h, mgpu_load_quad / mgpu_quad_rows /
// mgpu_quad_fbbt[_dev]).
//
// tightenQuad_ (src/base/QuadHandler.cpp:2683-2924) walks the original
// problem's objective (only with an incumbent, :2700) and constraints.  For
// each function of type Quadratic with a linear part it classifies the
// quadratic terms (univariate a x^2 + b x when x is also linear, else a
// product / square), skips it while no univariate term has been seen in
// this call (getQfLfBnds_ :2406-2410; the qvars vector accumulates over
// functions and is never cleared), and leaves out linear terms whose
// variable is in the accumulated qvars (:2412-2425).  All of that depends on
// structure only, so it is resolved once here into two programs (with and
// without the objective) of pre-classified term records.
#include <cmath>
#include <cstring>

#include "ctx.h"
#include "quad_state.h"

void quad_state_free(mgpu_ctx *c) {
  if (c && c->quad) {
    c->quad->release();
    delete c->quad;
    c->quad = nullptr;
  }
}

namespace {

struct QProg {
  std::vector<QFunRec> fun;
  std::vector<QTermRec> term;
};

QProg compile_program(int nv, int ncon, const int32_t *lptr, const int32_t *lvar,
                      const double *lval, const int32_t *qptr, const int32_t *qv1,
                      const int32_t *qv2, const double *qval, const double *clb,
                      const double *cub, bool with_obj) {
  QProg p;
  std::vector<char> isq(nv, 0);
  bool any = false;
  auto lin_weight = [&](int c, int v, double &w) {
    for (int k = lptr[c]; k < lptr[c + 1]; ++k)
      if (lvar[k] == v) {
        w = lval[k];
        return true;
      }
    w = 0.0;
    return false;
  };
  auto process = [&](int c, bool is_obj) {
    bool sq = false;
    for (int k = qptr[c]; k < qptr[c + 1]; ++k) sq |= qv1[k] == qv2[k];
    if (!sq || lptr[c + 1] == lptr[c]) return;  // not Quadratic, or no linear part
    const int t0 = (int)p.term.size();
    for (int k = qptr[c]; k < qptr[c + 1]; ++k) {
      QTermRec t{};
      double w;
      t.v1 = qv1[k];
      t.v2 = qv2[k];
      t.a = qval[k];
      if (qv1[k] == qv2[k] && lin_weight(c, qv1[k], w)) {
        isq[qv1[k]] = 1;
        any = true;
        t.kind = 0;
        t.b = w;
      } else {
        t.kind = 1;
      }
      p.term.push_back(t);
    }
    if (!any) {  // getQfLfBnds_ returns false: function skipped
      p.term.resize(t0);
      return;
    }
    for (int k = lptr[c]; k < lptr[c + 1]; ++k) {
      if (isq[lvar[k]]) continue;
      QTermRec t{};
      t.kind = 2;
      t.v1 = t.v2 = lvar[k];
      t.a = lval[k];
      p.term.push_back(t);
    }
    QFunRec f{};
    f.clb = is_obj ? -INFINITY : clb[c];
    f.cub = is_obj ? INFINITY : cub[c];
    f.t0 = t0;
    f.nt = (int)p.term.size() - t0;
    f.is_obj = is_obj ? 1 : 0;
    p.fun.push_back(f);
  };
  if (with_obj) process(ncon, true);
  for (int c = 0; c < ncon; ++c) process(c, false);
  return p;
}

double lf_keep(double a) { return std::fabs(a) > 1e-9 ? a : 0.0; }

}  // namespace

extern "C" {

int mgpu_load_quad(mgpu_ctx *c, int nv0, int nv, const int32_t *vtype, int nsq,
                   const int32_t *sq_x, const int32_t *sq_y, int nbil, const int32_t *bil_x0,
                   const int32_t *bil_x1, const int32_t *bil_y, int ncon, const int32_t *lptr,
                   const int32_t *lvar, const double *lval, const int32_t *qptr,
                   const int32_t *qv1, const int32_t *qv2, const double *qval,
                   const double *clb, const double *cub, int has_obj, double obj_const) {
  if (!c) return MGPU_ERR_ARG;
  if (nv <= 0 || nv0 < 0 || nv0 > nv || !vtype || nsq < 0 || nbil < 0 || ncon < 0 ||
      (nsq > 0 && (!sq_x || !sq_y)) || (nbil > 0 && (!bil_x0 || !bil_x1 || !bil_y)) ||
      !lptr || !qptr || (ncon > 0 && (!clb || !cub)))
    return fail(c, MGPU_ERR_ARG, "mgpu_load_quad: bad argument");
  for (int j = 0; j < nv; ++j)
    if (vtype[j] < 0 || vtype[j] > 4) return fail(c, MGPU_ERR_ARG, "bad vtype at %d", j);
  for (int k = 0; k < nsq; ++k) {
    if (sq_x[k] < 0 || sq_x[k] >= nv || sq_y[k] < 0 || sq_y[k] >= nv)
      return fail(c, MGPU_ERR_ARG, "square %d: index out of range", k);
    if (k > 0 && sq_x[k] <= sq_x[k - 1])
      return fail(c, MGPU_ERR_ARG, "squares not strictly ascending in x at %d", k);
  }
  for (int k = 0; k < nbil; ++k) {
    if (bil_x0[k] < 0 || bil_x1[k] >= nv || bil_x0[k] >= bil_x1[k] || bil_y[k] < 0 ||
        bil_y[k] >= nv)
      return fail(c, MGPU_ERR_ARG, "bilinear %d: bad indices", k);
    if (k > 0 && (bil_x0[k] < bil_x0[k - 1] ||
                  (bil_x0[k] == bil_x0[k - 1] && bil_x1[k] <= bil_x1[k - 1])))
      return fail(c, MGPU_ERR_ARG, "bilinears not strictly ascending at %d", k);
  }
  const int nfun = ncon + (has_obj ? 1 : 0);
  if (lptr[0] != 0 || qptr[0] != 0) return fail(c, MGPU_ERR_ARG, "lptr/qptr must start at 0");
  for (int f = 0; f < nfun; ++f) {
    if (lptr[f + 1] < lptr[f] || qptr[f + 1] < qptr[f])
      return fail(c, MGPU_ERR_ARG, "function %d: pointers not monotone", f);
    for (int k = lptr[f]; k < lptr[f + 1]; ++k) {
      if (!lvar || !lval || lvar[k] < 0 || lvar[k] >= nv0)
        return fail(c, MGPU_ERR_ARG, "function %d: linear var out of range", f);
      if (k > lptr[f] && lvar[k] <= lvar[k - 1])
        return fail(c, MGPU_ERR_ARG, "function %d: linear terms not strictly ascending", f);
      if (!(std::fabs(lval[k]) > 1e-9))
        return fail(c, MGPU_ERR_ARG, "function %d: linear weight below 1e-9", f);
    }
    for (int k = qptr[f]; k < qptr[f + 1]; ++k) {
      if (!qv1 || !qv2 || !qval || qv1[k] < 0 || qv2[k] >= nv0 || qv1[k] > qv2[k])
        return fail(c, MGPU_ERR_ARG, "function %d: bad quadratic term", f);
      if (k > qptr[f] && (qv1[k] < qv1[k - 1] || (qv1[k] == qv1[k - 1] && qv2[k] <= qv2[k - 1])))
        return fail(c, MGPU_ERR_ARG, "function %d: quadratic terms not strictly ascending", f);
      if (!(std::fabs(qval[k]) >= 1e-8))
        return fail(c, MGPU_ERR_ARG, "function %d: quadratic weight below 1e-8", f);
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  glob_state_free(c);  // a glob tree belongs to the problem it was started on
  quad_state_free(c);
  QuadState *q = new QuadState();
  c->quad = q;
  q->nv0 = nv0;
  q->nv = nv;
  q->R = 2 * nsq + 12 * nbil;
  q->sq_x.assign(sq_x, sq_x + nsq);
  q->sq_y.assign(sq_y, sq_y + nsq);
  q->bil_x0.assign(bil_x0, bil_x0 + nbil);
  q->bil_x1.assign(bil_x1, bil_x1 + nbil);
  q->bil_y.assign(bil_y, bil_y + nbil);
  q->obj_const = obj_const;
  // the original functions as given (the glob tree's QuadHandler::isFeasible)
  q->ncon = ncon;
  q->has_obj = has_obj != 0;
  q->h_lptr.assign(lptr, lptr + nfun + 1);
  q->h_qptr.assign(qptr, qptr + nfun + 1);
  q->h_lvar.assign(lvar, lvar + lptr[nfun]);
  q->h_lval.assign(lval, lval + lptr[nfun]);
  q->h_qv1.assign(qv1, qv1 + qptr[nfun]);
  q->h_qv2.assign(qv2, qv2 + qptr[nfun]);
  q->h_qval.assign(qval, qval + qptr[nfun]);
  q->h_clb.assign(clb, clb + ncon);
  q->h_cub.assign(cub, cub + ncon);
  q->h_vtype.assign(vtype, vtype + nv);

  std::vector<uint8_t> vt(nv);
  for (int j = 0; j < nv; ++j) vt[j] = (uint8_t)vtype[j];
  std::vector<int32_t> sqv(2 * (nsq > 0 ? nsq : 1)), bv(3 * (nbil > 0 ? nbil : 1));
  for (int k = 0; k < nsq; ++k) {
    sqv[2 * k] = sq_x[k];
    sqv[2 * k + 1] = sq_y[k];
  }
  for (int k = 0; k < nbil; ++k) {
    bv[3 * k] = bil_x0[k];
    bv[3 * k + 1] = bil_x1[k];
    bv[3 * k + 2] = bil_y[k];
  }
  QProg prog[2] = {
      compile_program(nv, ncon, lptr, lvar, lval, qptr, qv1, qv2, qval, clb, cub, false),
      compile_program(nv, ncon, lptr, lvar, lval, qptr, qv1, qv2, qval, clb, cub,
                      has_obj != 0)};
  q->obj_in_prog1 = !prog[1].fun.empty() && prog[1].fun[0].is_obj;
  int maxt = 1;
  for (int i = 0; i < 2; ++i)
    for (const QFunRec &f : prog[i].fun) maxt = f.nt > maxt ? f.nt : maxt;

  HIPCHK(c, upload(q->vtype, vt.data(), vt.size()));
  HIPCHK(c, upload(q->sq, sqv.data(), sqv.size()));
  HIPCHK(c, upload(q->bil, bv.data(), bv.size()));
  for (int i = 0; i < 2; ++i) {
    if (prog[i].fun.empty()) prog[i].fun.push_back(QFunRec{});  // keep a valid pointer
    if (prog[i].term.empty()) prog[i].term.push_back(QTermRec{});
    HIPCHK(c, upload(q->fun[i], prog[i].fun.data(), prog[i].fun.size()));
    HIPCHK(c, upload(q->term[i], prog[i].term.data(), prog[i].term.size()));
  }
  DevQuad &d = q->dq;
  d.nv = nv;
  d.nsq = nsq;
  d.nbil = nbil;
  d.maxt = maxt;
  d.vtype = q->vtype.as<uint8_t>();
  d.sq = q->sq.as<int32_t>();
  d.bil = q->bil.as<int32_t>();
  for (int i = 0; i < 2; ++i) {
    d.fun[i] = q->fun[i].as<QFunRec>();
    d.term[i] = q->term[i].as<QTermRec>();
    // the placeholder record of an empty program is not counted
    d.nfun[i] = (prog[i].fun.size() == 1 && prog[i].fun[0].nt == 0) ? 0 : (int)prog[i].fun.size();
  }
  d.obj_const = obj_const;
  return MGPU_OK;
}

int mgpu_quad_rows(mgpu_ctx *c, const double *lb, const double *ub, double *rows, int *nrows) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->quad) return fail(c, MGPU_ERR_STATE, "mgpu_quad_rows: no quadratic problem loaded");
  const QuadState &q = *c->quad;
  if (nrows) *nrows = q.R;
  if (!rows) return MGPU_OK;
  if (!lb || !ub) return fail(c, MGPU_ERR_ARG, "mgpu_quad_rows: bad argument");
  // QuadHandler::relax_ -> getNewSqLf_ / getNewBilLf_ (QuadHandler.cpp:702-803)
  int o = 0;
  for (size_t k = 0; k < q.sq_x.size(); ++k, o += 2) {
    const double l = lb[q.sq_x[k]], u = ub[q.sq_x[k]];
    if (l < -1e12 || u > 1e12)
      return fail(c, MGPU_ERR_ARG, "square %zu: |bound| > 1e12 needs a default bound", k);
    rows[o + 1] = -u * l;
    rows[o] = std::fabs(u + l) > 1e-5 ? lf_keep(-1. * (u + l)) : 0.0;
  }
  for (size_t k = 0; k < q.bil_x0.size(); ++k, o += 12) {
    const double l0 = lb[q.bil_x0[k]], u0 = ub[q.bil_x0[k]];
    const double l1 = lb[q.bil_x1[k]], u1 = ub[q.bil_x1[k]];
    if (l0 < -1e12 || l1 < -1e12 || u0 > 1e12 || u1 > 1e12)
      return fail(c, MGPU_ERR_ARG, "bilinear %zu: |bound| > 1e12 needs a default bound", k);
    double *r = rows + o;
    r[0] = lf_keep(l1);
    r[1] = lf_keep(l0);
    r[2] = l0 * l1;
    r[3] = lf_keep(u1);
    r[4] = lf_keep(u0);
    r[5] = u0 * u1;
    r[6] = lf_keep(-1.0 * u1);
    r[7] = lf_keep(-1.0 * l0);
    r[8] = -l0 * u1;
    r[9] = lf_keep(-1.0 * l1);
    r[10] = lf_keep(-1.0 * u0);
    r[11] = -u0 * l1;
  }
  return MGPU_OK;
}

int mgpu_quad_fbbt_dev(mgpu_ctx *c, int batch, const double *lb_in, const double *ub_in,
                       double incumbent, int qt, const double *rows_in, int rows_shared,
                       double *lb_out, double *ub_out, double *rows_out, int32_t *infeas,
                       int32_t *nmods, int mod_cap, int32_t *mod_kind, int32_t *mod_idx,
                       double *mod_v1, double *mod_v2) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->quad) return fail(c, MGPU_ERR_STATE, "mgpu_quad_fbbt: no quadratic problem loaded");
  QuadState &q = *c->quad;
  if (batch < 0 || (batch > 0 && (!lb_in || !ub_in || !lb_out || !ub_out || !infeas ||
                                  !nmods || (q.R > 0 && (!rows_in || !rows_out)))))
    return fail(c, MGPU_ERR_ARG, "mgpu_quad_fbbt: bad argument");
  if (mod_cap > 0 && (!mod_kind || !mod_idx || !mod_v1 || !mod_v2))
    return fail(c, MGPU_ERR_ARG, "mgpu_quad_fbbt: mod_cap > 0 needs mod buffers");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  QuadIO io{};
  io.batch = batch;
  io.lb_in = lb_in;
  io.ub_in = ub_in;
  io.lb_out = lb_out;
  io.ub_out = ub_out;
  io.rows_in = rows_in;
  io.rows_stride = rows_shared ? 0 : q.R;
  io.rows_out = rows_out;
  io.infeas = infeas;
  io.nmods = nmods;
  io.mod_cap = mod_cap > 0 ? mod_cap : 0;
  io.mod_kind = mod_cap > 0 ? mod_kind : nullptr;
  io.mod_idx = mod_cap > 0 ? mod_idx : nullptr;
  io.mod_v1 = mod_cap > 0 ? mod_v1 : nullptr;
  io.mod_v2 = mod_cap > 0 ? mod_v2 : nullptr;
  io.qt = qt ? 1 : 0;
  // tightenQuad_ :2698-2700: the objective only when bestSol - constant < inf
  io.prog = (q.obj_in_prog1 && incumbent - q.obj_const < INFINITY) ? 1 : 0;
  io.best = incumbent;
  // Variant (mgpu_set_fbbt_variant): 1 node state in LDS, 2 global scratch,
  // 0 auto = LDS while it leaves room for several waves per CU.
  const size_t lds = quad_lds_bytes(q.dq);
  int variant = c->fbbt_variant;
  if (variant != 1 && variant != 2) variant = lds <= 40 * 1024 ? 1 : 2;  // 0 auto (3, 4: K1 only)
  if (variant == 1 && lds > 160 * 1024)
    return fail(c, MGPU_ERR_ARG, "quad LDS variant needs %zu B > 160 KiB", lds);
  if (variant == 2) {
    const size_t waves = ((size_t)batch + kLanes - 1) / kLanes;
    HIPCHK(c, q.scratch.ensure(waves * (2 * q.dq.nv + 2 * q.dq.maxt) * kLanes * sizeof(double)));
    io.scratch = q.scratch.as<double>();
  }
  HIPCHK(c, hipEventRecord(c->ev4, c->stream));
  HIPCHK(c, launch_quad_fbbt(q.dq, io, variant == 1, c->stream));
  HIPCHK(c, hipEventRecord(c->ev5, c->stream));
  return MGPU_OK;
}

int mgpu_quad_fbbt(mgpu_ctx *c, int batch, const double *lb_in, const double *ub_in,
                   double incumbent, int qt, const double *rows_in, int rows_shared,
                   double *lb_out, double *ub_out, double *rows_out, int32_t *infeas,
                   int32_t *nmods, int mod_cap, int32_t *mod_kind, int32_t *mod_idx,
                   double *mod_v1, double *mod_v2) {
  if (!c) return MGPU_ERR_ARG;
  if (!c->quad) return fail(c, MGPU_ERR_STATE, "mgpu_quad_fbbt: no quadratic problem loaded");
  QuadState &q = *c->quad;
  if (batch < 0 || (batch > 0 && (!lb_in || !ub_in || !lb_out || !ub_out || !infeas ||
                                  !nmods || (q.R > 0 && (!rows_in || !rows_out)))))
    return fail(c, MGPU_ERR_ARG, "mgpu_quad_fbbt: bad argument");
  if (batch == 0) return MGPU_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t nb = (size_t)batch * q.nv * sizeof(double);
  const size_t rin = (size_t)(rows_shared ? 1 : batch) * (q.R > 0 ? q.R : 1) * sizeof(double);
  const size_t rout = (size_t)batch * (q.R > 0 ? q.R : 1) * sizeof(double);
  const int cap = mod_cap > 0 ? mod_cap : 0;
  HIPCHK(c, q.io_lb_in.ensure(nb));
  HIPCHK(c, q.io_ub_in.ensure(nb));
  HIPCHK(c, q.io_lb_out.ensure(nb));
  HIPCHK(c, q.io_ub_out.ensure(nb));
  HIPCHK(c, q.io_rin.ensure(rin));
  HIPCHK(c, q.io_rout.ensure(rout));
  HIPCHK(c, q.io_inf.ensure((size_t)batch * 4));
  HIPCHK(c, q.io_nm.ensure((size_t)batch * 4));
  if (cap) {
    HIPCHK(c, q.io_kind.ensure((size_t)batch * cap * 4));
    HIPCHK(c, q.io_idx.ensure((size_t)batch * cap * 4));
    HIPCHK(c, q.io_v1.ensure((size_t)batch * cap * 8));
    HIPCHK(c, q.io_v2.ensure((size_t)batch * cap * 8));
  }
  HIPCHK(c, hipMemcpyAsync(q.io_lb_in.p, lb_in, nb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(q.io_ub_in.p, ub_in, nb, hipMemcpyHostToDevice, c->stream));
  if (q.R > 0)
    HIPCHK(c, hipMemcpyAsync(q.io_rin.p, rows_in, rin, hipMemcpyHostToDevice, c->stream));
  int rc = mgpu_quad_fbbt_dev(c, batch, q.io_lb_in.as<double>(), q.io_ub_in.as<double>(),
                              incumbent, qt, q.io_rin.as<double>(), rows_shared,
                              q.io_lb_out.as<double>(), q.io_ub_out.as<double>(),
                              q.io_rout.as<double>(), q.io_inf.as<int32_t>(),
                              q.io_nm.as<int32_t>(), cap, q.io_kind.as<int32_t>(),
                              q.io_idx.as<int32_t>(), q.io_v1.as<double>(), q.io_v2.as<double>());
  if (rc != MGPU_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(lb_out, q.io_lb_out.p, nb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(ub_out, q.io_ub_out.p, nb, hipMemcpyDeviceToHost, c->stream));
  if (q.R > 0)
    HIPCHK(c, hipMemcpyAsync(rows_out, q.io_rout.p, rout, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(infeas, q.io_inf.p, (size_t)batch * 4, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipMemcpyAsync(nmods, q.io_nm.p, (size_t)batch * 4, hipMemcpyDeviceToHost,
                           c->stream));
  if (cap && mod_kind && mod_idx && mod_v1 && mod_v2) {
    HIPCHK(c, hipMemcpyAsync(mod_kind, q.io_kind.p, (size_t)batch * cap * 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mod_idx, q.io_idx.p, (size_t)batch * cap * 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mod_v1, q.io_v1.p, (size_t)batch * cap * 8,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(mod_v2, q.io_v2.p, (size_t)batch * cap * 8,
                             hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MGPU_OK;
}

}  // extern "C"
