// K2 — batched quadratic node FBBT, gfx950.
//
// Restates, per node, QuadHandler::presolveNode (src/base/QuadHandler.cpp:
// 1204-1269): propSqrBnds_ (:1361-1395) and propBilBnds_ (:1271-1301) over
// the y = x^2 / y = x0*x1 registries until nothing changes, then (first call
// or doQT_) tightenQuad_ (:2683-2924) over the original quadratic
// constraints and objective, then upSqCon_ / upBilCon_ (:3322-3419) secant
// and McCormick row rewrites.  Bound updates follow updatePBounds_
// (:3248-3320); interval primitives are Operations.cpp:100-246.  The C
// restatement is oracle/quad_fbbt.c; both are bit-exact with the reference.
//
// Mapping (MI355X-first): ONE NODE PER LANE, one wave64 per workgroup, like
// K1.  The registries and the tightenQuad_ program (pre-classified terms,
// see DevQuad) are the same for every node, so every loop over them is
// wave-uniform and their records are scalar loads.  The node's bounds and
// the forward term bounds (fwdLb/fwdUb) live in a [var][lane] layout —
// LDS when they fit, else a global scratch — so each access is one
// conflict-free / coalesced 512-B wave access.  Lanes whose node has
// converged or proved infeasible are masked; the propagation loop runs
// while any lane still changes.  -ffp-contract=off; sqrt and division are
// the correctly rounded IEEE operations, as on the reference's x86-64.
#include "mgpu_internal.h"

namespace mgpu {
namespace {

constexpr double kATol = 1e-6;   // QuadHandler.cpp:60-67
constexpr double kBTol = 1e-8;
constexpr double kRTol = 1e-7;
constexpr double kLfTol = 1e-9;  // LinearFunction.cpp:22, :89-95
constexpr int kPropCap = 100000; // the reference loop is uncapped (:1215)

__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }

// Operations.cpp:122-177
__device__ __forceinline__ void bounds_on_product(bool zxiz, double l0, double u0, double l1,
                                                  double u1, double &lb, double &ub) {
  if (fabs(l1) <= 1e-10 && fabs(u1) <= 1e-10) {
    double p = l1; l1 = l0; l0 = p;
    p = u1; u1 = u0; u0 = p;
  }
  if (fabs(l0) <= 1e-10 && fabs(u0) <= 1e-10) {
    if (zxiz) {
      lb = 0.0;
      ub = 0.0;
    } else {
      lb = l1 == -INFINITY ? -INFINITY : 0.0;
      ub = u1 == INFINITY ? INFINITY : 0.0;
    }
  } else if ((l1 == -INFINITY && u1 == INFINITY) || (l0 == -INFINITY && u0 == INFINITY)) {
    lb = -INFINITY;
    ub = INFINITY;
  } else {
    double p = l0 * l1;
    if (isnan(p)) p = -INFINITY;
    double lo = p, hi = p;
    p = u0 * l1;
    if (isnan(p)) p = INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    p = u0 * u1;
    if (isnan(p)) p = -INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    p = l0 * u1;
    if (isnan(p)) p = INFINITY;
    lo = smin(lo, p);
    hi = smax(hi, p);
    lb = lo;
    ub = hi;
  }
}

// Operations.cpp:180-210
__device__ __forceinline__ void bounds_on_recip(double l0, double u0, double &lb, double &ub) {
  if (fabs(u0) < 1e-10 && fabs(l0) < 1e-10) {
    lb = -INFINITY;
    ub = INFINITY;
  } else if (l0 < -1e-10 && u0 > 1e-10) {
    lb = -INFINITY;
    ub = INFINITY;
  } else if (fabs(u0) < 1e-10 && l0 < 0) {
    lb = -INFINITY;
    ub = 1.0 / l0;
  } else if (fabs(l0) < 1e-10 && u0 < 0) {
    lb = 1.0 / u0;
    ub = INFINITY;
  } else {
    lb = 1.0 / u0;
    ub = 1.0 / l0;
  }
}

// Operations.cpp:100-106
__device__ __forceinline__ void bounds_on_div(double l0, double u0, double l1, double u1,
                                              double &lb, double &ub) {
  double tl, tu;
  bounds_on_recip(l1, u1, tl, tu);
  bounds_on_product(false, l0, u0, tl, tu, lb, ub);
}

// Operations.cpp:213-227
__device__ __forceinline__ void bounds_on_square(double l1, double u1, double &lb, double &ub) {
  if (u1 < 0.) {
    lb = u1 * u1;
    ub = l1 * l1;
  } else if (l1 > 0.) {
    lb = l1 * l1;
    ub = u1 * u1;
  } else {
    lb = 0.;
    ub = smax(l1 * l1, u1 * u1);
  }
}

// Per-lane view of one node: bounds and forward-term slots at [i][lane].
template <bool kLds>
struct QNode {
  double *lb, *ub, *fl, *fu;
  int stride, lane;
  const uint8_t *vtype;
  int nmods, cap;
  int32_t *kind, *idx;
  double *v1, *v2;
  __device__ __forceinline__ double &L(int j) const { return lb[j * stride + lane]; }
  __device__ __forceinline__ double &U(int j) const { return ub[j * stride + lane]; }
  __device__ __forceinline__ double &FL(int t) const { return fl[t * stride + lane]; }
  __device__ __forceinline__ double &FU(int t) const { return fu[t * stride + lane]; }
  __device__ __forceinline__ void push(int k, int i, double a, double b) {
    if (kind != nullptr && nmods < cap) {
      kind[nmods] = k;
      idx[nmods] = i;
      v1[nmods] = a;
      v2[nmods] = b;
    }
    ++nmods;
  }
};

// updatePBounds_ (relaxation form), QuadHandler.cpp:3248-3320
template <class N>
__device__ __forceinline__ bool update_pbounds(N &s, int v, double lb, double ub, bool &ch) {
  const int t = s.vtype[v];
  const double L = s.L(v), U = s.U(v);
  if (t <= 3) {  // Binary, Integer, ImplBin, ImplInt
    ub = floor(ub);
    lb = ceil(lb);
  }
  if (lb > U + kBTol || ub < L - kBTol) return true;
  if (lb > L + kBTol && ub < U - kBTol && (L == -INFINITY || lb > L + kRTol * fabs(L)) &&
      (U == INFINITY || ub < U - kRTol * fabs(U))) {
    ch = true;
    s.L(v) = lb;
    s.U(v) = ub;
    s.push(2, v, lb, ub);
  } else if (lb > L + kBTol && (L == -INFINITY || lb > L + kRTol * fabs(L))) {
    ch = true;
    s.L(v) = lb;
    s.push(0, v, lb, 0.0);
  } else if (ub < U - kBTol && (U == INFINITY || ub < U - kRTol * fabs(U))) {
    ch = true;
    s.U(v) = ub;
    s.push(1, v, ub, 0.0);
  }
  return false;
}

// propSqrBnds_, QuadHandler.cpp:1361-1395 (true = infeasible)
template <class N>
__device__ __forceinline__ bool prop_sqr(N &s, int x, int y, bool &ch) {
  double lb, ub;
  bounds_on_square(s.L(x), s.U(x), lb, ub);
  if (update_pbounds(s, y, lb, ub, ch)) return true;
  const double uy = s.U(y);
  if (uy > kBTol) {
    ub = sqrt(uy);
    lb = -ub;
    const double ly = s.L(y);
    if (s.L(x) > -sqrt(ly) + kBTol) lb = sqrt(ly);
    return update_pbounds(s, x, lb, ub, ch);
  }
  if (uy < -kBTol) return true;
  return update_pbounds(s, x, 0.0, 0.0, ch);
}

// propBilBnds_, QuadHandler.cpp:1271-1301
template <class N>
__device__ __forceinline__ bool prop_bil(N &s, int x0, int x1, int y, bool &ch) {
  double lb, ub;
  bounds_on_product(true, s.L(x0), s.U(x0), s.L(x1), s.U(x1), lb, ub);
  if (update_pbounds(s, y, lb, ub, ch)) return true;
  bounds_on_div(s.L(y), s.U(y), s.L(x0), s.U(x0), lb, ub);
  if (update_pbounds(s, x1, lb, ub, ch)) return true;
  bounds_on_div(s.L(y), s.U(y), s.L(x1), s.U(x1), lb, ub);
  return update_pbounds(s, x0, lb, ub, ch);
}

// calcUpperUnivar_, QuadHandler.cpp:1707-1720
__device__ __forceinline__ double calc_upper_univar(double a, double b, double lx, double ux) {
  double u = smax(lx * (a * lx + b), ux * (a * ux + b));
  const double sh = b / 2.0, t = sh / (-a);
  if (t > lx) {
    const double r = (-2.0 * a) * ux;
    if (r > b) u = smax(u, sh * t);
  }
  return u;
}

// getTermBnds_ overloads, QuadHandler.cpp:1723-1771, one per term kind
template <class N>
__device__ __forceinline__ void term_bnds(const N &s, const QTermRec &t, double &lb, double &ub) {
  if (t.kind == 0) {  // a x^2 + b x
    const double lx = s.L(t.v1), ux = s.U(t.v1), a = t.a, b = t.b;
    if (lx > -kATol) {
      ub = calc_upper_univar(a, b, lx, ux);
      lb = -calc_upper_univar(-a, -b, lx, ux);
    } else if (ux < kATol) {
      ub = calc_upper_univar(a, -b, -ux, -lx);
      lb = -calc_upper_univar(-a, b, -ux, -lx);
    } else {
      ub = calc_upper_univar(a, b, 0.0, ux);
      ub = smax(ub, calc_upper_univar(a, -b, 0.0, -lx));
      lb = -calc_upper_univar(-a, -b, 0.0, ux);
      lb = smin(lb, -calc_upper_univar(-a, b, 0.0, -lx));
    }
    return;
  }
  double ql, qu;
  if (t.kind == 1) {
    if (t.v1 == t.v2) bounds_on_square(s.L(t.v1), s.U(t.v1), ql, qu);
    else bounds_on_product(true, s.L(t.v1), s.U(t.v1), s.L(t.v2), s.U(t.v2), ql, qu);
  } else {
    ql = s.L(t.v1);
    qu = s.U(t.v1);
  }
  const double c = t.a;
  if (c > 0) {
    lb = ql > -INFINITY ? c * ql : -INFINITY;
    ub = qu < INFINITY ? c * qu : INFINITY;
  } else {
    lb = qu < INFINITY ? c * qu : -INFINITY;
    ub = ql > -INFINITY ? c * ql : INFINITY;
  }
}

// calcVarBnd_(rel, v, a, b, ly, uy), QuadHandler.cpp:1968-2078
template <class N>
__device__ __forceinline__ bool calc_univar(N &s, int v, double a, double b, double ly,
                                            double uy, bool &ch) {
  const double lx = s.L(v), ux = s.U(v);
  double lb = -INFINITY, ub = INFINITY, delta, lb2, ub2;
  if (fabs(a) <= kATol) {
    lb = ly / b;
    ub = uy / b;
  } else if (a > kATol) {
    if (uy < INFINITY) {
      delta = b * b + 4.0 * a * uy;
      if (delta < -kATol) return true;
      if (fabs(delta) <= kATol) {
        lb = -b / (2.0 * a);
        ub = lb;
      } else {
        lb = (-b - sqrt(delta)) / (2.0 * a);
        ub = (-b + sqrt(delta)) / (2.0 * a);
        delta = b * b + 4.0 * a * ly;
        if (delta > kATol) {
          lb2 = (-b - sqrt(delta)) / (2.0 * a);
          ub2 = (-b + sqrt(delta)) / (2.0 * a);
          if (lx > lb2 + kBTol) lb = ub2;
          if (ux < ub2 - kBTol) ub = lb2;
        }
      }
    } else {
      delta = b * b + 4.0 * a * ly;
      if (delta > kATol) {
        lb2 = (-b - sqrt(delta)) / (2.0 * a);
        ub2 = (-b + sqrt(delta)) / (2.0 * a);
        if (lx > lb2 + kBTol && lx < ub2 - kBTol) lb = ub2;
        if (ux > lb2 + kBTol && ux < ub2 - kBTol) ub = lb2;
      }
    }
  } else {
    if (ly > -INFINITY) {
      delta = b * b + 4.0 * a * ly;
      if (delta < -kATol) return true;
      if (fabs(delta) <= kATol) {
        lb = -b / (2.0 * a);
        ub = lb;
      } else {
        lb = (-b + sqrt(delta)) / (2.0 * a);
        ub = (-b - sqrt(delta)) / (2.0 * a);
        delta = b * b + 4.0 * a * uy;
        if (delta > kATol) {
          lb2 = (-b + sqrt(delta)) / (2.0 * a);
          ub2 = (-b - sqrt(delta)) / (2.0 * a);
          if (lx > lb2 + kBTol) lb = ub2;
          if (ux < ub2 - kBTol) ub = lb2;
        }
      }
    } else {
      delta = b * b + 4.0 * a * uy;
      if (delta > kATol) {
        lb2 = (-b - sqrt(delta)) / (2.0 * a);
        ub2 = (-b + sqrt(delta)) / (2.0 * a);
        if (lx > lb2 + kBTol && lx < ub2 - kBTol) lb = ub2;
        if (ux > lb2 + kBTol && ux < ub2 - kBTol) ub = lb2;
      }
    }
  }
  return update_pbounds(s, v, lb, ub, ch);
}

// calcVarBnd_(rel, v1, v2, coef, ...), QuadHandler.cpp:1841-1881 (the square
// branch starts vlb from -ub, the function argument, as :1852 does) and
// calcVarBnd_(rel, v, coef, ...), :1786-1797
template <class N>
__device__ __forceinline__ bool calc_var_bnd(N &s, const QTermRec &t, double lb, double ub,
                                             bool &ch) {
  if (t.kind == 0) return calc_univar(s, t.v1, t.a, t.b, lb, ub, ch);
  const double c = t.a;
  if (t.kind == 2) {
    const double vlb = c > 0 ? lb / c : ub / c;
    const double vub = c > 0 ? ub / c : lb / c;
    return update_pbounds(s, t.v1, vlb, vub, ch);
  }
  double qlb = c > 0 ? lb / c : ub / c;
  const double qub = c > 0 ? ub / c : lb / c;
  double vlb, vub;
  if (t.v1 == t.v2) {
    if (qub > kBTol) {
      vub = sqrt(qub);
      vlb = -ub;
      qlb = qlb >= 0 ? qlb : 0;
      if (s.L(t.v1) > -sqrt(qlb) + kBTol) vlb = sqrt(qlb);
      return update_pbounds(s, t.v1, vlb, vub, ch);
    }
    if (qub < -kBTol) return true;
    return update_pbounds(s, t.v1, 0.0, 0.0, ch);
  }
  bounds_on_div(qlb, qub, s.L(t.v1), s.U(t.v1), vlb, vub);
  if (update_pbounds(s, t.v2, vlb, vub, ch)) return true;
  bounds_on_div(qlb, qub, s.L(t.v2), s.U(t.v2), vlb, vub);
  return update_pbounds(s, t.v1, vlb, vub, ch);
}

// getSumExcept1_, QuadHandler.cpp:2111-2146, over the lane's forward slots
template <class N>
__device__ __forceinline__ double sum_except1(const N &s, bool upper, int nf, int cur,
                                              double bound, unsigned ninf) {
  if (ninf == 0) return bound - (upper ? s.FU(cur) : s.FL(cur));
  if (ninf == 1) {
    const double fc = upper ? s.FU(cur) : s.FL(cur);
    if (upper ? fc >= INFINITY : fc <= -INFINITY) {
      double sum = 0.0;
      for (int i = 0; i < nf; ++i)
        if (i != cur) sum += upper ? s.FU(i) : s.FL(i);
      return sum;
    }
  }
  return upper ? INFINITY : -INFINITY;
}

__device__ __forceinline__ double lf_keep(double a) { return fabs(a) > kLfTol ? a : 0.0; }

// upSqCon_ / upBilCon_ (QuadHandler.cpp:3322-3419) with getNewSqLf_ /
// getNewBilLf_ (:702-803) on the lane's row state
// Returns true when a rebuild would need addDefaultBounds_ (|bound| > 1e12,
// :709-722 / :780-787), which mutates handler state: reported, not emulated.
template <class N>
__device__ __forceinline__ bool up_rows(N &s, const DevQuad &q, const double *rin, double *rout) {
  const double eps = kATol / 10.0;
  bool dflt = false;
  for (int k = 0; k < q.nsq; ++k) {
    const int x = q.sq[2 * k];
    const double lb = s.L(x), ub = s.U(x);
    double ax = rin[2 * k], rhs = rin[2 * k + 1];
    if ((lb * lb + ax * lb < rhs - eps) || (ub * ub + ax * ub < rhs - eps)) {
      dflt |= lb < -1e12 || ub > 1e12;
      rhs = -ub * lb;
      ax = fabs(ub + lb) > 1e-5 ? lf_keep(-1. * (ub + lb)) : 0.0;
      s.push(3, k, rhs, 0.0);
    }
    rout[2 * k] = ax;
    rout[2 * k + 1] = rhs;
  }
  const int o = 2 * q.nsq;
  for (int k = 0; k < q.nbil; ++k) {
    const int x0 = q.bil[3 * k], x1 = q.bil[3 * k + 1];
    const double l0 = s.L(x0), u0 = s.U(x0), l1 = s.L(x1), u1 = s.U(x1);
    const bool wide = l0 < -1e12 || l1 < -1e12 || u0 > 1e12 || u1 > 1e12;
    const double *ri = rin + o + 12 * k;
    double *ro = rout + o + 12 * k;
    const int rb = q.nsq + 4 * k;
    double a0, a1, r;
    a0 = ri[0]; a1 = ri[1]; r = ri[2];
    if (a0 * l0 + a1 * l1 - l0 * l1 < r - eps || a0 * l0 + a1 * u1 - l0 * u1 < r - eps ||
        a0 * u0 + a1 * l1 - u0 * l1 < r - eps) {
      a0 = lf_keep(l1); a1 = lf_keep(l0); r = l0 * l1;
      s.push(3, rb, r, 0.0);
      dflt |= wide;
    }
    ro[0] = a0; ro[1] = a1; ro[2] = r;
    a0 = ri[3]; a1 = ri[4]; r = ri[5];
    if (a0 * l0 + a1 * u1 - l0 * u1 < r - eps || a0 * u0 + a1 * l1 - u0 * l1 < r - eps ||
        a0 * u0 + a1 * u1 - u0 * u1 < r - eps) {
      a0 = lf_keep(u1); a1 = lf_keep(u0); r = u0 * u1;
      s.push(3, rb + 1, r, 0.0);
      dflt |= wide;
    }
    ro[3] = a0; ro[4] = a1; ro[5] = r;
    a0 = ri[6]; a1 = ri[7]; r = ri[8];
    if (a0 * l0 + a1 * l1 + l0 * l1 < r - eps || a0 * l0 + a1 * u1 + l0 * u1 < r - eps ||
        a0 * u0 + a1 * u1 + u0 * u1 < r - eps) {
      a0 = lf_keep(-1.0 * u1); a1 = lf_keep(-1.0 * l0); r = -l0 * u1;
      s.push(3, rb + 2, r, 0.0);
      dflt |= wide;
    }
    ro[6] = a0; ro[7] = a1; ro[8] = r;
    a0 = ri[9]; a1 = ri[10]; r = ri[11];
    if (a0 * l0 + a1 * l1 + l0 * l1 < r - eps || a0 * u0 + a1 * l1 + u0 * l1 < r - eps ||
        a0 * u0 + a1 * u1 + u0 * u1 < r - eps) {
      a0 = lf_keep(-1.0 * l1); a1 = lf_keep(-1.0 * u0); r = -u0 * l1;
      s.push(3, rb + 3, r, 0.0);
      dflt |= wide;
    }
    ro[9] = a0; ro[10] = a1; ro[11] = r;
  }
  return dflt;
}

template <bool kLds>
__global__ __launch_bounds__(kLanes) void quad_fbbt_kernel(DevQuad q, QuadIO io) {
  extern __shared__ double qlds[];
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * kLanes;
  const int nb = min(kLanes, io.batch - b0);
  const int nv = q.nv;
  const bool live = lane < nb;
  const int b = b0 + lane;

  QNode<kLds> s;
  s.lane = lane;
  s.vtype = q.vtype;
  double *base;
  if constexpr (kLds) {
    s.stride = kLdsStride;
    base = qlds;
  } else {
    s.stride = kLanes;
    base = io.scratch + (size_t)blockIdx.x * (2 * nv + 2 * q.maxt) * kLanes;
  }
  s.lb = base;
  s.ub = base + (size_t)nv * s.stride;
  s.fl = base + (size_t)2 * nv * s.stride;
  s.fu = base + (size_t)(2 * nv + q.maxt) * s.stride;
  s.nmods = 0;
  s.cap = io.mod_cap;
  s.kind = nullptr;
  s.idx = nullptr;
  s.v1 = nullptr;
  s.v2 = nullptr;
  if (io.mod_kind != nullptr && io.mod_cap > 0 && live) {
    const size_t o = (size_t)b * io.mod_cap;
    s.kind = io.mod_kind + o;
    s.idx = io.mod_idx + o;
    s.v1 = io.mod_v1 + o;
    s.v2 = io.mod_v2 + o;
  }
  // stage the wave's boxes ([node][var] in HBM) into [var][lane]
  for (int nd = 0; nd < nb; ++nd) {
    const double *src_l = io.lb_in + (size_t)(b0 + nd) * nv;
    const double *src_u = io.ub_in + (size_t)(b0 + nd) * nv;
    for (int j = lane; j < nv; j += kLanes) {
      s.lb[j * s.stride + nd] = src_l[j];
      s.ub[j * s.stride + nd] = src_u[j];
    }
  }
  __syncthreads();

  // propSqrBnds_ / propBilBnds_ until no change (QuadHandler.cpp:1215-1239)
  int status = 0;  // 0 running, 1 infeasible, 2 propagation cap
  bool changed = live;
  int iters = 0;
  while (__any(changed && status == 0)) {
    bool go = changed && status == 0;
    if (go && ++iters > kPropCap) {
      status = 2;
      go = false;
    }
    bool lch = false;
    for (int k = 0; k < q.nsq; ++k) {
      const int x = q.sq[2 * k], y = q.sq[2 * k + 1];
      if (go && prop_sqr(s, x, y, lch)) {
        status = 1;
        go = false;
      }
    }
    for (int k = 0; k < q.nbil; ++k) {
      const int x0 = q.bil[3 * k], x1 = q.bil[3 * k + 1], y = q.bil[3 * k + 2];
      if (go && prop_bil(s, x0, x1, y, lch)) {
        status = 1;
        go = false;
      }
    }
    changed = go && lch;
  }

  // tightenQuad_ (QuadHandler.cpp:1241-1250, :2683-2924)
  if (io.qt) {
    const QFunRec *fun = q.fun[io.prog];
    const QTermRec *term = q.term[io.prog];
    const int nfun = q.nfun[io.prog];
    for (int f = 0; f < nfun; ++f) {
      const QFunRec fr = fun[f];
      bool go = live && status == 0;
      if (!__any(go)) break;
      double il = 0.0, iu = 0.0;
      unsigned cil = 0, ciu = 0;
      if (go) {
        for (int t = 0; t < fr.nt; ++t) {  // forward (getQfLfBnds_)
          const QTermRec tr = term[fr.t0 + t];
          double lb, ub;
          term_bnds(s, tr, lb, ub);
          if (lb <= -INFINITY) ++cil;
          if (ub >= INFINITY) ++ciu;
          il += lb;
          iu += ub;
          s.FL(t) = lb;
          s.FU(t) = ub;
        }
      }
      double clb, cub;
      if (fr.is_obj) {
        clb = -INFINITY;
        cub = io.best - q.obj_const;
      } else {
        clb = fr.clb;
        cub = fr.cub;
        if (go && (il > cub + kATol || iu < clb - kATol)) {
          status = 1;
          go = false;
        }
      }
      clb = clb > il ? clb : il;
      cub = cub < iu ? cub : iu;
      bool ch = false;
      for (int t = 0; t < fr.nt; ++t) {  // backward
        const QTermRec tr = term[fr.t0 + t];
        if (!go) continue;
        const double lb = clb - sum_except1(s, true, fr.nt, t, iu, ciu);
        const double ub = cub - sum_except1(s, false, fr.nt, t, il, cil);
        if (calc_var_bnd(s, tr, lb, ub, ch)) {
          status = 1;
          go = false;
        }
      }
    }
  }

  // secant / McCormick rows, bounds out
  if (live) {
    const int R = 2 * q.nsq + 12 * q.nbil;
    const double *rin = io.rows_in + (size_t)b * io.rows_stride;
    double *rout = io.rows_out + (size_t)b * R;
    if (status == 0) {
      if (up_rows(s, q, rin, rout)) status = 3;
    } else {
      for (int i = 0; i < R; ++i) rout[i] = rin[i];
    }
    io.infeas[b] = status;
    io.nmods[b] = s.nmods;
  }
  __syncthreads();
  for (int nd = 0; nd < nb; ++nd) {
    double *dst_l = io.lb_out + (size_t)(b0 + nd) * nv;
    double *dst_u = io.ub_out + (size_t)(b0 + nd) * nv;
    for (int j = lane; j < nv; j += kLanes) {
      dst_l[j] = s.lb[j * s.stride + nd];
      dst_u[j] = s.ub[j * s.stride + nd];
    }
  }
}

}  // namespace

size_t quad_lds_bytes(const DevQuad &q) {
  return (size_t)(2 * q.nv + 2 * q.maxt) * kLdsStride * sizeof(double);
}

hipError_t launch_quad_fbbt(const DevQuad &q, const QuadIO &io, bool use_lds,
                            hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  const int waves = (io.batch + kLanes - 1) / kLanes;
  const size_t lds = quad_lds_bytes(q);
  if (use_lds) {
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr_set = false;  // dynamic LDS above 64 KiB must be opted in
    if (!attr_set) {
      hipError_t e = hipFuncSetAttribute((const void *)quad_fbbt_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
      attr_set = true;
    }
    hipLaunchKernelGGL((quad_fbbt_kernel<true>), dim3(waves), dim3(kLanes), lds, stream, q, io);
  } else {
    if (io.scratch == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL((quad_fbbt_kernel<false>), dim3(waves), dim3(kLanes), 0, stream, q, io);
  }
  return hipGetLastError();
}

}  // namespace mgpu
