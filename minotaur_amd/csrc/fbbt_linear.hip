// K1 — batched node FBBT over linear rows, gfx950.
//
// Restates, per node, LinearHandler::presolveNode -> simplePresolve in node
// mode (src/base/LinearHandler.cpp:1592-1653) and the helpers it calls:
// varBndsFromCons_ (:493-541), linBndTighten_ (:952-1045),
// updateLfBoundsFromLb_/Ub_ (:1048-1226), changeBFlag_ (:1229-1234),
// getLfBnds_ (:1237-1258), getSingLfBnds_ (:1261-1319), varBndsFromObj_
// (:544-597), tightenInts_ (:415-490), checkBounds_ (:328-359).
//
// Mapping (MI355X-first): ONE NODE PER LANE, one wave64 per workgroup.
//  * FBBT inside a node is Gauss-Seidel: rows in index order, bounds updated
//    in place, order-dependent f64 sums.  Bit-exactness forbids splitting a
//    row sum, so parallelism is across nodes only.
//  * Every node shares the same rows, so the row/term loops are wave-uniform:
//    CSR terms are read with scalar (SMEM) loads and broadcast to all lanes;
//    only the comparisons/updates diverge (EXEC-masked).
//  * The node's bounds live in LDS as [var][lane] f64 with a 65-element
//    stride: term j of a row is one conflict-free ds_read_b64 per bound for
//    the whole wave.  Row flags (Constraint::BFlag) are bytes [row][lane].
//  * Problems whose bounds do not fit the 160 KiB LDS use the same code on a
//    global [var][lane] scratch (coalesced 512-B wave accesses, L2-resident).
//  * Compiled with -ffp-contract=off: no fused multiply-add, as the
//    reference's x86-64 build (no FMA without -march).
#include "mgpu_internal.h"

namespace mgpu {
namespace {

struct NodeView {
  double *lb;
  double *ub;
  uint8_t *flag;
  int stride;  // elements between consecutive variables (same lane)
  int lane;
  __device__ __forceinline__ double &L(int j) const { return lb[j * stride + lane]; }
  __device__ __forceinline__ double &U(int j) const { return ub[j * stride + lane]; }
  __device__ __forceinline__ uint8_t &F(int r) const { return flag[r * kLanes + lane]; }
};

struct NodeState {
  int nmods;
  unsigned nintmods;
};

__device__ __forceinline__ bool is_int_type(uint8_t t) {
  return t == kBinary || t == kInteger;
}

struct ModLog {
  int32_t *var, *lu;
  double *val;
  int cap;
  __device__ __forceinline__ void push(NodeState &s, int j, int lu_, double v) const {
    if (var != nullptr && s.nmods < cap) {
      var[s.nmods] = j;
      lu[s.nmods] = lu_;
      val[s.nmods] = v;
    }
    s.nmods++;
  }
};

// changeBFlag_: every row holding column j is flagged (LinearHandler.cpp:1229).
__device__ __forceinline__ void change_bflag(const DevLP &lp, const NodeView &v, int j) {
  const int k0 = lp.colptr[j], k1 = lp.colptr[j + 1];
  for (int k = k0; k < k1; ++k) v.F(lp.rowidx[k]) = 1;
}

// getLfBnds_ (LinearHandler.cpp:1237-1258): ascending-column f64 sums.
__device__ __forceinline__ void lf_bnds(const Term *t, int nt, const NodeView &v,
                                        double &lo, double &up) {
  double l = 0.0, u = 0.0;
  for (int k = 0; k < nt; ++k) {
    const double c = t[k].a;
    const int j = t[k].j;
    const double vl = v.L(j), vu = v.U(j);
    if (c > 0) {
      l += c * vl;
      u += c * vu;
    } else {
      l += c * vu;
      u += c * vl;
    }
  }
  lo = l;
  up = u;
}

// getSingLfBnds_ (LinearHandler.cpp:1261-1319): sums that skip a single
// infinite term; a second infinite term makes the side infinite.
__device__ void sing_lf_bnds(const Term *t, int nt, const NodeView &v, double &lo,
                             double &up) {
  double l = 0.0, u = 0.0;
  bool lo_sing = false, up_sing = false, lo_fin = true, up_fin = true;
  for (int k = 0; k < nt; ++k) {
    const double c = t[k].a;
    const int j = t[k].j;
    const double vl = v.L(j), vu = v.U(j);
    if (c > kETol) {
      if (vu < kInfty && up_fin) {
        u += c * vu;
      } else if (up_sing) {
        up_sing = false; u = INFINITY; up_fin = false;
      } else {
        up_sing = true;
      }
      if (vl > -kInfty && lo_fin) {
        l += c * vl;
      } else if (lo_sing) {
        lo_sing = false; l = -INFINITY; lo_fin = false;
      } else {
        lo_sing = true;
      }
    } else if (c < -kETol) {
      if (vu < kInfty && lo_fin) {
        l += c * vu;
      } else if (lo_sing) {
        lo_sing = false; l = -INFINITY; lo_fin = false;
      } else {
        lo_sing = true;
      }
      if (vl > -kInfty && up_fin) {
        u += c * vl;
      } else if (up_sing) {
        up_sing = false; u = INFINITY; up_fin = false;
      } else {
        up_sing = true;
      }
    }
  }
  lo = l;
  up = u;
}

// updateLfBoundsFromLb_ (LinearHandler.cpp:1048-1134).
__device__ void upd_from_lb(const DevLP &lp, const Term *t, int nt, const NodeView &v,
                            NodeState &s, const ModLog &log, double lb, double uu,
                            bool is_sing, bool &changed, bool count_int) {
  for (int k = 0; k < nt; ++k) {
    const double c = t[k].a;
    const int j = t[k].j;
    double vlb = v.L(j), vub = v.U(j);
    if (c > kETol && (!is_sing || vub >= kInfty)) {
      if (vub >= kInfty) vub = 0.;
      double nlb = (lb - uu) / c + vub;
      if (nlb > vlb + kETol) {
        const double cur_ub = v.U(j);
        if (nlb > cur_ub - kETol) nlb = cur_ub;
        change_bflag(lp, v, j);
        v.L(j) = nlb;
        log.push(s, j, 0, nlb);
        if (count_int && is_int_type(lp.vtype[j])) s.nintmods++;
        changed = true;
      }
    } else if (c < -kETol && (!is_sing || vlb <= -kInfty)) {
      if (vlb <= -kInfty) vlb = 0.;
      double nub = (lb - uu) / c + vlb;
      if (nub < vub - kETol) {
        const double cur_lb = v.L(j);
        if (nub < cur_lb + kETol) nub = cur_lb;
        change_bflag(lp, v, j);
        v.U(j) = nub;
        log.push(s, j, 1, nub);
        if (count_int && is_int_type(lp.vtype[j])) s.nintmods++;
        changed = true;
      }
    }
  }
}

// updateLfBoundsFromUb_ (LinearHandler.cpp:1137-1226).
__device__ void upd_from_ub(const DevLP &lp, const Term *t, int nt, const NodeView &v,
                            NodeState &s, const ModLog &log, double ub, double ll,
                            bool is_sing, bool &changed, bool count_int) {
  for (int k = 0; k < nt; ++k) {
    const double c = t[k].a;
    const int j = t[k].j;
    double vlb = v.L(j), vub = v.U(j);
    if (c > kETol && (!is_sing || vlb <= -kInfty)) {
      if (vlb <= -kInfty) vlb = 0.;
      double nub = (ub - ll) / c + vlb;
      if (nub < vub - kETol) {
        const double cur_lb = v.L(j);
        if (nub < cur_lb + kETol) nub = cur_lb;
        change_bflag(lp, v, j);
        v.U(j) = nub;
        log.push(s, j, 1, nub);
        if (count_int && is_int_type(lp.vtype[j])) s.nintmods++;
        changed = true;
      }
    } else if (c < -kETol && (!is_sing || vub >= kInfty)) {
      if (vub >= kInfty) vub = 0.;
      double nlb = (ub - ll) / c + vub;
      if (nlb > vlb + kETol) {
        const double cur_ub = v.U(j);
        if (nlb > cur_ub - kETol) nlb = cur_ub;
        change_bflag(lp, v, j);
        v.L(j) = nlb;
        log.push(s, j, 0, nlb);
        if (count_int && is_int_type(lp.vtype[j])) s.nintmods++;
        changed = true;
      }
    }
  }
}

// linBndTighten_ in node mode (LinearHandler.cpp:952-1045).  Returns true if
// the row proves the node infeasible.
__device__ bool lin_bnd_tighten(const DevLP &lp, int r, const NodeView &v, NodeState &s,
                                const ModLog &log, bool &changed) {
  const int k0 = lp.rowptr[r];
  const int nt = lp.rowptr[r + 1] - k0;
  const Term *t = lp.terms + k0;
  const double lb = lp.rlo[r], ub = lp.rhi[r];
  double ll, uu, sing_ll = -INFINITY, sing_uu = INFINITY;
  changed = false;
  lf_bnds(t, nt, v, ll, uu);
  if (ll < -kInfty || uu > kInfty) sing_lf_bnds(t, nt, v, sing_ll, sing_uu);
  if (ll > ub + kETol) return true;
  if (uu < lb - kETol) return true;
  if (lb > -kInfty) {
    if (uu < kInfty) {
      upd_from_lb(lp, t, nt, v, s, log, lb, uu, false, changed, true);
    } else if (sing_uu < kInfty) {
      upd_from_lb(lp, t, nt, v, s, log, lb, sing_uu, true, changed, true);
    }
  }
  if (changed) {
    lf_bnds(t, nt, v, ll, uu);
    if (ll < -kInfty || uu > kInfty) sing_lf_bnds(t, nt, v, sing_ll, sing_uu);
  }
  if (ub < kInfty) {
    if (ll > -kInfty) {
      upd_from_ub(lp, t, nt, v, s, log, ub, ll, false, changed, true);
    } else if (sing_ll > -kInfty) {
      upd_from_ub(lp, t, nt, v, s, log, ub, sing_ll, true, changed, true);
    }
  }
  return false;
}

// varBndsFromObj_ (LinearHandler.cpp:544-597).  The reference loops until no
// change; the 100000 cap is a safety net never reached on real data (the
// oracle uses the same cap).
__device__ void bnds_from_obj(const DevLP &lp, const NodeView &v, NodeState &s,
                              const ModLog &log, double ub, bool &changed) {
  bool tch = true;
  long guard = 0;
  while (tch) {
    double ll, uu, sing_ll = INFINITY, sing_uu = INFINITY;
    tch = false;
    lf_bnds(lp.obj, lp.nobj, v, ll, uu);
    if (ll < -kInfty || uu > kInfty) sing_lf_bnds(lp.obj, lp.nobj, v, sing_ll, sing_uu);
    if (ll > ub + kETol) return;  // SolvedInfeasible, ignored by the caller
    if (ll > -kInfty) {
      upd_from_ub(lp, lp.obj, lp.nobj, v, s, log, ub, ll, false, tch, false);
    } else if (sing_ll > -kInfty) {
      upd_from_ub(lp, lp.obj, lp.nobj, v, s, log, ub, sing_ll, true, tch, false);
    }
    if (tch) changed = true;
    if (++guard > 100000L) break;
  }
}

// tightenInts_ in node mode (LinearHandler.cpp:415-490).
__device__ void tighten_ints(const DevLP &lp, const NodeView &v, NodeState &s,
                             const ModLog &log, bool &changed) {
  for (int j = 0; j < lp.n; ++j) {
    if (!is_int_type(lp.vtype[j])) continue;
    const double l = v.L(j), u = v.U(j);
    if (l > -kInfty && fabs(l - floor(l + 0.5)) > kIntTol) {
      const double nv = ceil(l);
      change_bflag(lp, v, j);
      v.L(j) = nv;
      log.push(s, j, 0, nv);
      changed = true;
    }
    if (u < kInfty && fabs(u - floor(u + 0.5)) > kIntTol) {
      const double nv = floor(u);
      v.U(j) = nv;
      change_bflag(lp, v, j);
      log.push(s, j, 1, nv);
      changed = true;
    }
  }
}

// checkBounds_ (LinearHandler.cpp:328-359).
__device__ bool check_bounds(const DevLP &lp, const NodeView &v) {
  for (int j = 0; j < lp.n; ++j) {
    if (v.L(j) > v.U(j) + kETol) return true;
  }
  return lp.cons_bad != 0;
}

template <bool kLds>
__global__ __launch_bounds__(kLanes) void fbbt_linear_kernel(DevLP lp, FbbtIO io) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * kLanes;
  const int nb = min(kLanes, io.batch - b0);
  const int n = lp.n, m = lp.m;

  NodeView v;
  v.lane = lane;
  if constexpr (kLds) {
    v.stride = kLdsStride;
    v.lb = lds;
    v.ub = lds + (size_t)n * kLdsStride;
    v.flag = reinterpret_cast<uint8_t *>(lds + (size_t)2 * n * kLdsStride);
  } else {
    v.stride = kLanes;
    v.lb = io.scratch + (size_t)blockIdx.x * 2 * n * kLanes;
    v.ub = v.lb + (size_t)n * kLanes;
    v.flag = io.flag_scratch + (size_t)blockIdx.x * m * kLanes;
  }

  // Stage the wave's node boxes (row-major [node][var] in HBM, coalesced
  // reads) into the [var][lane] layout.
  for (int nd = 0; nd < nb; ++nd) {
    const double *src_l = io.lb_in + (size_t)(b0 + nd) * n;
    const double *src_u = io.ub_in + (size_t)(b0 + nd) * n;
    for (int j = lane; j < n; j += kLanes) {
      v.lb[j * v.stride + nd] = src_l[j];
      v.ub[j * v.stride + nd] = src_u[j];
    }
  }
  // simplePresolve: every constraint's BFlag set (LinearHandler.cpp:1618-1622)
  for (int r = 0; r < m; ++r) v.F(r) = 1;
  __syncthreads();

  const bool live = lane < nb;
  NodeState s{0, 0u};
  ModLog log{nullptr, nullptr, nullptr, io.mod_cap};
  if (io.mod_var != nullptr && io.mod_cap > 0 && live) {
    const size_t o = (size_t)(b0 + lane) * io.mod_cap;
    log.var = io.mod_var + o;
    log.lu = io.mod_lu + o;
    log.val = io.mod_val + o;
  }

  // simplePresolve sweep loop (LinearHandler.cpp:1624-1644).  The status
  // returns of varBndsFromCons_/varBndsFromObj_ are ignored (:1630, :1637);
  // only checkBounds_ ends the loop as infeasible.
  bool changed = live;
  bool infeas = false;
  unsigned iters = 1;
  while (true) {
    const bool go = changed && iters <= 10u && (iters <= 2u || s.nintmods > 0u) && !infeas;
    if (!__any(go)) break;
    if (go) {
      s.nintmods = 0u;
      changed = false;
      ++iters;
    }
    // varBndsFromCons_: one pass over the rows in index order; a row that
    // proves infeasibility ends this lane's pass (early return, :527-529).
    bool cons_on = go;
    for (int r = 0; r < m; ++r) {
      const bool mine = cons_on && v.F(r) != 0;
      if (!__any(mine)) continue;
      if (mine) {
        bool tch;
        v.F(r) = 0;
        if (lin_bnd_tighten(lp, r, v, s, log, tch)) {
          cons_on = false;
        } else if (tch) {
          changed = true;
        }
      }
    }
    if (go && io.has_inc && lp.nobj > 0) bnds_from_obj(lp, v, s, log, io.inc_ub, changed);
    if (go) {
      tighten_ints(lp, v, s, log, changed);
      infeas = check_bounds(lp, v);
    }
  }
  if (live) {
    io.infeas[b0 + lane] = infeas ? 1 : 0;
    io.nmods[b0 + lane] = s.nmods;
  }
  __syncthreads();
  for (int nd = 0; nd < nb; ++nd) {
    double *dst_l = io.lb_out + (size_t)(b0 + nd) * n;
    double *dst_u = io.ub_out + (size_t)(b0 + nd) * n;
    for (int j = lane; j < n; j += kLanes) {
      dst_l[j] = v.lb[j * v.stride + nd];
      dst_u[j] = v.ub[j * v.stride + nd];
    }
  }
}

}  // namespace

size_t fbbt_lds_bytes(int n, int m) {
  return (size_t)2 * n * kLdsStride * sizeof(double) + (size_t)m * kLanes;
}

hipError_t launch_fbbt_linear(const DevLP &lp, const FbbtIO &io, int variant,
                              hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  const int waves = (io.batch + kLanes - 1) / kLanes;
  const size_t lds = fbbt_lds_bytes(lp.n, lp.m);
  const bool use_lds = variant == 1 || (variant == 0 && lds <= 160 * 1024);
  if (use_lds) {
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr_set = false;  // dynamic LDS above 64 KiB must be opted in
    if (!attr_set) {
      hipError_t e = hipFuncSetAttribute((const void *)fbbt_linear_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return e;
      attr_set = true;
    }
    hipLaunchKernelGGL(fbbt_linear_kernel<true>, dim3(waves), dim3(kLanes), lds, stream,
                       lp, io);
  } else {
    if (io.scratch == nullptr || io.flag_scratch == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fbbt_linear_kernel<false>, dim3(waves), dim3(kLanes), 0, stream,
                       lp, io);
  }
  return hipGetLastError();
}

}  // namespace mgpu
