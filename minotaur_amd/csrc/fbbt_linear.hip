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
//  * Every node shares the same rows, so row/term loops are wave-uniform.
//    Row and term records are fetched 64 at a time with one coalesced vector
//    load (lane t holds record t) and broadcast with v_readlane into SGPRs;
//    the inner loops issue only LDS reads and VALU (scalar-memory loads
//    would share lgkmcnt with the LDS reads and serialise every term).
//  * The node's bounds live in LDS as [var][lane] f64 with a 65-element
//    stride: term j of a row is one conflict-free ds_read_b64 per bound for
//    the whole wave.  Row flags (Constraint::BFlag) are a per-lane 64-bit
//    mask in VGPRs when m <= 64 (changeBFlag_ = OR of the column's row
//    mask), else bytes [row][lane].
//  * Problems whose bounds do not fit the 160 KiB LDS run the same code on a
//    global [var][lane] scratch (coalesced 512-B wave accesses).
//  * Compiled with -ffp-contract=off: no fused multiply-add, as the
//    reference's x86-64 build (no FMA without -march).
#include "mgpu_internal.h"

#include <type_traits>

namespace mgpu {
namespace {

// write-out order of the global variant: var-outer (each store one
// coalesced 512-B row; the node-outer order measured the same)
constexpr bool kFbbtOutVarOuter = true;

// ---- wave-uniform broadcast ------------------------------------------------
__device__ __forceinline__ int rl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ double rld(double v, int k) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), k);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ uint64_t rlu64(uint64_t v, int k) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(v & 0xffffffffu), k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(v >> 32), k);
  return ((uint64_t)hi << 32) | lo;
}

// v_readfirstlane: the value of the first ACTIVE lane, so it is correct
// under any EXEC mask (v_readlane of a fixed lane is not: inside a
// divergent region the compiler may copy or reload a VGPR for the active
// lanes only, and a fixed lane may be inactive -- round 5 met exactly that)
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double rfld(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ uint64_t rflu64(uint64_t v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(v & 0xffffffffu));
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Per-lane slice of a chunk of up to 64 term records (tightenInts_'s column
// list, read with v_readlane in uniform control flow only).
struct TermChunk {
  uint64_t cmask;
  int j, cs, ce, isint;
};

__device__ __forceinline__ TermChunk load_terms(const TermRec *base, int cnt, int lane) {
  TermChunk c{0ull, 0, 0, 0, 0};
  if (lane < cnt) {
    const TermRec r = base[lane];
    c.cmask = r.cmask;
    c.j = r.j;
    c.cs = r.cs;
    c.ce = r.ce;
    c.isint = r.isint;
  }
  return c;
}

struct Term1 {  // one term, every field wave-uniform
  double a;
  uint64_t cmask;
  int j, cs, ce, isint;
};

// Term k of a record list (LDS in the persistent and staged kernels, HBM
// otherwise): a wave-uniform address read by every active lane, made
// uniform with readfirstlane.  Row visits run in divergent code (only the
// lanes whose node flagged the row), so every record read there goes this
// way.
__device__ __forceinline__ Term1 term_at(const TermRec *base, int k) {
  const TermRec r = base[k];
  return Term1{rfld(r.a), rflu64(r.cmask), rfl(r.j), rfl(r.cs), rfl(r.ce), rfl(r.isint)};
}

// Calls f(Term1) for every term of a term list, in order.
template <class F>
__device__ __forceinline__ void for_terms(const TermRec *base, int nt, F &&f) {
  for (int k = 0; k < nt; ++k) f(term_at(base, k));
}

// ---- per-lane node view ----------------------------------------------------
// kIL (global variant): lb and ub interleaved, [var][lane][2], so a term's
// two bounds are one 16-B load per lane (one 1-KB wave access)
template <bool kBitFlags, bool kIL>
struct NodeView {
  double *lb;
  double *ub;
  uint8_t *flag;     // byte flags [row][lane] (m > 64)
  uint64_t bits;     // bit flags (m <= 64)
  int stride;        // elements between consecutive variables (same lane)
  int lane;
  const int32_t *rowidx;
  static constexpr bool kBits = kBitFlags;
  __device__ __forceinline__ double &L(int j) const {
    if constexpr (kIL) return lb[((size_t)j * kLanes + lane) * 2];
    else return lb[j * stride + lane];
  }
  __device__ __forceinline__ double &U(int j) const {
    if constexpr (kIL) return lb[((size_t)j * kLanes + lane) * 2 + 1];
    else return ub[j * stride + lane];
  }
  __device__ __forceinline__ bool flagged(int r) const {
    if constexpr (kBitFlags) return (bits >> r) & 1ull;
    else return flag[r * kLanes + lane] != 0;
  }
  __device__ __forceinline__ void clear(int r) {
    if constexpr (kBitFlags) bits &= ~(1ull << r);
    else flag[r * kLanes + lane] = 0;
  }
  // changeBFlag_ (LinearHandler.cpp:1229-1234): flag every row holding the
  // column of term k of chunk ch.
  __device__ __forceinline__ void change_bflag(const Term1 &t) {
    if constexpr (kBitFlags) {
      bits |= t.cmask;
    } else {
      for (int q = t.cs; q < t.ce; ++q) flag[rowidx[q] * kLanes + lane] = 1;
    }
  }
};

// bounds loaded per batch in the column loops (tightenInts_, checkBounds_,
// staging, write-out): loads issued together, one memory round trip
constexpr int kBnd = 8;

// box in (row-major [node][var] in HBM) -> this lane's node view, and back;
// kBnd loads in flight before the stores (src and dst may alias as far as
// the compiler knows, which would make every column its own round trip)
template <class V>
__device__ __forceinline__ void box_in(V &v, const double *src_l, const double *src_u, int n) {
  for (int j0 = 0; j0 < n; j0 += kBnd) {
    double a[kBnd], b[kBnd];
#pragma unroll
    for (int e = 0; e < kBnd; ++e) {
      const int j = j0 + e < n ? j0 + e : j0;
      a[e] = src_l[j];
      b[e] = src_u[j];
    }
#pragma unroll
    for (int e = 0; e < kBnd; ++e)
      if (j0 + e < n) {
        v.L(j0 + e) = a[e];
        v.U(j0 + e) = b[e];
      }
  }
}
template <class V>
__device__ __forceinline__ void box_out(const V &v, double *dst_l, double *dst_u, int n) {
  for (int j0 = 0; j0 < n; j0 += kBnd) {
    double a[kBnd], b[kBnd];
#pragma unroll
    for (int e = 0; e < kBnd; ++e) {
      const int j = j0 + e < n ? j0 + e : j0;
      a[e] = v.L(j);
      b[e] = v.U(j);
    }
#pragma unroll
    for (int e = 0; e < kBnd; ++e)
      if (j0 + e < n) {
        dst_l[j0 + e] = a[e];
        dst_u[j0 + e] = b[e];
      }
  }
}

struct NodeState {
  int nmods;
  unsigned nintmods;
};

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

// getLfBnds_ (LinearHandler.cpp:1237-1258): ascending-column f64 sums.
template <class V>
__device__ __forceinline__ void lf_bnds(const TermRec *base, int nt, const V &v, double &lo,
                                        double &up) {
  double l = 0.0, u = 0.0;
  for_terms(base, nt, [&](const Term1 &t) {
    const double vl = v.L(t.j), vu = v.U(t.j);
    if (t.a > 0) {
      l += t.a * vl;
      u += t.a * vu;
    } else {
      l += t.a * vu;
      u += t.a * vl;
    }
  });
  lo = l;
  up = u;
}

// getSingLfBnds_ (LinearHandler.cpp:1261-1319): sums that skip a single
// infinite term; a second infinite term makes the side infinite.
template <class V>
__device__ __forceinline__ void sing_lf_bnds(const TermRec *base, int nt, const V &v, double &lo,
                                             double &up) {
  double l = 0.0, u = 0.0;
  bool lo_sing = false, up_sing = false, lo_fin = true, up_fin = true;
  for_terms(base, nt, [&](const Term1 &t) {
    const double c = t.a;
    const double vl = v.L(t.j), vu = v.U(t.j);
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
  });
  lo = l;
  up = u;
}

// updateLfBoundsFromLb_ (LinearHandler.cpp:1048-1134) when from_lb, with
// diff = lb - uu; updateLfBoundsFromUb_ (:1137-1226) otherwise, with
// diff = ub - ll.  A term with coef > 0 (from_lb) / coef < 0 (from_ub)
// raises its column's lower bound, the other sign lowers the upper bound.
//
// Terms are taken four at a time: phase A computes the four candidate
// bounds (four independent f64 divisions in flight), phase B applies them
// in term order.  This is exactly the reference's sequential loop because
// each term of a row is a different column and a term only reads and writes
// its own column's bounds; the order-dependent effects (mod log, nintmods)
// are produced in phase B in term order.
template <class V>
__device__ __forceinline__ void upd_side(const TermRec *base, int nt, V &v,
                         NodeState &s, const ModLog &log, double diff, bool from_lb,
                         bool is_sing, bool &changed, bool count_int) {
  for (int k0 = 0; k0 < nt; k0 += 4) {
    Term1 t[4];
    double cand[4], cur[4];
    bool hit[4], low[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      hit[u] = false;
      low[u] = false;
      cand[u] = 0.0;
      cur[u] = 0.0;
      if (k0 + u < nt) {
        t[u] = term_at(base, k0 + u);
        const double c = t[u].a;
        if (c > kETol || c < -kETol) {
          const double vl = v.L(t[u].j), vu = v.U(t[u].j);
          low[u] = from_lb ? c > 0 : c < 0;
          if (low[u]) {
            // new lower bound: diff/c + (vub, or 0 for a singleton infinity)
            const bool ok = !is_sing || vu >= kInfty;
            const double nb = diff / c + (vu >= kInfty ? 0. : vu);
            hit[u] = ok && nb > vl + kETol;
            cand[u] = nb;
            cur[u] = vu;          // var->getUb() for the clamp
          } else {
            const bool ok = !is_sing || vl <= -kInfty;
            const double nb = diff / c + (vl <= -kInfty ? 0. : vl);
            hit[u] = ok && nb < vu - kETol;
            cand[u] = nb;
            cur[u] = vl;          // var->getLb() for the clamp
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (hit[u]) {
        const int j = t[u].j;
        double nb = cand[u];
        if (low[u]) {
          if (nb > cur[u] - kETol) nb = cur[u];
          v.change_bflag(t[u]);
          v.L(j) = nb;
          log.push(s, j, 0, nb);
        } else {
          if (nb < cur[u] + kETol) nb = cur[u];
          v.change_bflag(t[u]);
          v.U(j) = nb;
          log.push(s, j, 1, nb);
        }
        if (count_int && t[u].isint) s.nintmods++;
        changed = true;
      }
    }
  }
}

// ---- register-cached rows ---------------------------------------------------
// A row of nt <= RC terms is tightened with all of its bounds gathered into
// registers ONCE (2*RC independent loads in flight), reused by the 4-5 passes
// of linBndTighten_ and written through on every update.  The passes are
// straight-line over RC slots; slots >= nt are masked.  Same arithmetic, same
// order as the generic path (and the reference): sums run over k = 0..nt-1,
// masked slots contribute nothing and never update.
template <int RC>
struct RowCache {
  double l[RC], u[RC];
  double a[RC];
};

template <int RC, class V>
__device__ __forceinline__ void rc_load(RowCache<RC> &c, const TermRec *base, int nt,
                                        const V &v) {
#pragma unroll
  for (int k = 0; k < RC; ++k) {
    const int kk = k < nt ? k : 0;   // clamped: loads are unconditional
    const TermRec *r = base + kk;    // the record's first 16 B: a, j
    const int j = rfl(r->j);
    c.a[k] = k < nt ? rfld(r->a) : 0.0;
    c.l[k] = v.L(j);
    c.u[k] = v.U(j);
  }
}

template <int RC>
__device__ __forceinline__ void rc_lf_bnds(const RowCache<RC> &c, int nt, double &lo,
                                           double &up) {
  double l = 0.0, u = 0.0;
#pragma unroll
  for (int k = 0; k < RC; ++k) {
    if (k < nt) {
      const double a = c.a[k];
      if (a > 0) {
        l += a * c.l[k];
        u += a * c.u[k];
      } else {
        l += a * c.u[k];
        u += a * c.l[k];
      }
    }
  }
  lo = l;
  up = u;
}

template <int RC>
__device__ __forceinline__ void rc_sing_lf_bnds(const RowCache<RC> &c, int nt, double &lo, double &up) {
  double l = 0.0, u = 0.0;
  bool lo_sing = false, up_sing = false, lo_fin = true, up_fin = true;
#pragma unroll
  for (int k = 0; k < RC; ++k) {
    if (k >= nt) continue;
    const double cc = c.a[k], vl = c.l[k], vu = c.u[k];
    if (cc > kETol) {
      if (vu < kInfty && up_fin) {
        u += cc * vu;
      } else if (up_sing) {
        up_sing = false; u = INFINITY; up_fin = false;
      } else {
        up_sing = true;
      }
      if (vl > -kInfty && lo_fin) {
        l += cc * vl;
      } else if (lo_sing) {
        lo_sing = false; l = -INFINITY; lo_fin = false;
      } else {
        lo_sing = true;
      }
    } else if (cc < -kETol) {
      if (vu < kInfty && lo_fin) {
        l += cc * vu;
      } else if (lo_sing) {
        lo_sing = false; l = -INFINITY; lo_fin = false;
      } else {
        lo_sing = true;
      }
      if (vl > -kInfty && up_fin) {
        u += cc * vl;
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

// upd_side on the cache: phase A computes every slot's candidate (RC
// independent divisions), phase B applies hits in term order.
template <int RC, class V>
__device__ __forceinline__ void rc_upd_side(RowCache<RC> &c, const TermRec *base, int nt, V &v,
                            NodeState &s, const ModLog &log, double diff, bool from_lb,
                            bool is_sing, bool &changed, bool count_int) {
  double cand[RC];
  bool hit[RC];
#pragma unroll
  for (int k = 0; k < RC; ++k) {
    const double cc = c.a[k];
    const double vl = c.l[k], vu = c.u[k];
    const bool act = k < nt && (cc > kETol || cc < -kETol);
    const bool low = from_lb ? cc > 0 : cc < 0;
    const double den = act ? cc : 1.0;
    if (low) {
      const bool ok = !is_sing || vu >= kInfty;
      const double nb = diff / den + (vu >= kInfty ? 0. : vu);
      hit[k] = act && ok && nb > vl + kETol;
      cand[k] = nb;
    } else {
      const bool ok = !is_sing || vl <= -kInfty;
      const double nb = diff / den + (vl <= -kInfty ? 0. : vl);
      hit[k] = act && ok && nb < vu - kETol;
      cand[k] = nb;
    }
  }
#pragma unroll
  for (int k = 0; k < RC; ++k) {
    if (k < nt && hit[k]) {
      const Term1 t = term_at(base, k);   // t.a == c.a[k]
      const bool low = from_lb ? t.a > 0 : t.a < 0;
      double nb = cand[k];
      if (low) {
        if (nb > c.u[k] - kETol) nb = c.u[k];
        v.change_bflag(t);
        v.L(t.j) = nb;
        c.l[k] = nb;
        log.push(s, t.j, 0, nb);
      } else {
        if (nb < c.l[k] + kETol) nb = c.l[k];
        v.change_bflag(t);
        v.U(t.j) = nb;
        c.u[k] = nb;
        log.push(s, t.j, 1, nb);
      }
      if (count_int && t.isint) s.nintmods++;
      changed = true;
    }
  }
}

// linBndTighten_ (LinearHandler.cpp:952-1045) on a register-cached row.
template <int RC, class V>
__device__ __forceinline__ bool rc_lin_bnd_tighten(int nt, const TermRec *base, double lb, double ub, V &v,
                                   NodeState &s, const ModLog &log, bool &changed) {
  RowCache<RC> c;
  rc_load<RC>(c, base, nt, v);
  double ll = 0.0, uu = 0.0, sing_ll = -INFINITY, sing_uu = INFINITY;
  changed = false;
  // pass 0: the lb side (updateLfBoundsFromLb_ with lb - uu, or lb - the
  // singleton sum), pass 1: the ub side; the activity sums are recomputed
  // before pass 1 only if pass 0 changed a bound.  The side and the
  // singleton case are run-time values, so each pass holds one copy of the
  // update (two before: the code is half the size, same operations)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (p == 0 || changed) {
      rc_lf_bnds<RC>(c, nt, ll, uu);
      if (ll < -kInfty || uu > kInfty) rc_sing_lf_bnds<RC>(c, nt, sing_ll, sing_uu);
    }
    if (p == 0 && (ll > ub + kETol || uu < lb - kETol)) return true;
    const bool lo_side = p == 0;
    const bool side_fin = lo_side ? lb > -kInfty : ub < kInfty;
    const double act = lo_side ? uu : ll, sact = lo_side ? sing_uu : sing_ll;
    const bool act_fin = lo_side ? act < kInfty : act > -kInfty;
    const bool sact_fin = lo_side ? sact < kInfty : sact > -kInfty;
    if (side_fin && (act_fin || sact_fin))
      rc_upd_side<RC>(c, base, nt, v, s, log, (lo_side ? lb : ub) - (act_fin ? act : sact), lo_side,
                      !act_fin, changed, true);
  }
  return false;
}

// varBndsFromObj_ (LinearHandler.cpp:544-597) on a register-cached
// objective (nobj <= RC).
template <int RC, class V>
__device__ __forceinline__ void rc_bnds_from_obj(int nobj, const TermRec *base, V &v, NodeState &s,
                                 const ModLog &log, double ub, bool &changed) {
  RowCache<RC> c;
  rc_load<RC>(c, base, nobj, v);
  bool tch = true;
  long guard = 0;
  while (tch) {
    double ll, uu, sing_ll = INFINITY, sing_uu = INFINITY;
    tch = false;
    rc_lf_bnds<RC>(c, nobj, ll, uu);
    if (ll < -kInfty || uu > kInfty) rc_sing_lf_bnds<RC>(c, nobj, sing_ll, sing_uu);
    if (ll > ub + kETol) return;
    const bool fin = ll > -kInfty;
    if (fin || sing_ll > -kInfty)
      rc_upd_side<RC>(c, base, nobj, v, s, log, ub - (fin ? ll : sing_ll), false, !fin, tch, false);
    if (tch) changed = true;
    if (++guard > 100000L) break;
  }
}

// linBndTighten_ in node mode (LinearHandler.cpp:952-1045).  Returns true if
// the row proves the node infeasible.
template <class V>
__device__ __forceinline__ bool lin_bnd_tighten(const TermRec *base, int nt, double lb,
                                double ub, V &v, NodeState &s, const ModLog &log,
                                bool &changed) {
  double ll = 0.0, uu = 0.0, sing_ll = -INFINITY, sing_uu = INFINITY;
  changed = false;
  // the two sides as in rc_lin_bnd_tighten
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (p == 0 || changed) {
      lf_bnds(base, nt, v, ll, uu);
      if (ll < -kInfty || uu > kInfty) sing_lf_bnds(base, nt, v, sing_ll, sing_uu);
    }
    if (p == 0 && (ll > ub + kETol || uu < lb - kETol)) return true;
    const bool lo_side = p == 0;
    const bool side_fin = lo_side ? lb > -kInfty : ub < kInfty;
    const double act = lo_side ? uu : ll, sact = lo_side ? sing_uu : sing_ll;
    const bool act_fin = lo_side ? act < kInfty : act > -kInfty;
    const bool sact_fin = lo_side ? sact < kInfty : sact > -kInfty;
    if (side_fin && (act_fin || sact_fin))
      upd_side(base, nt, v, s, log, (lo_side ? lb : ub) - (act_fin ? act : sact), lo_side,
               !act_fin, changed, true);
  }
  return false;
}

// varBndsFromObj_ (LinearHandler.cpp:544-597).  The reference loops until no
// change; the 100000 cap is a safety net never reached on real data (the
// oracle uses the same cap).
template <class V>
__device__ __forceinline__ void bnds_from_obj(const TermRec *orec, int nobj, V &v, NodeState &s,
                              const ModLog &log, double ub, bool &changed) {
  bool tch = true;
  long guard = 0;
  while (tch) {
    double ll, uu, sing_ll = INFINITY, sing_uu = INFINITY;
    tch = false;
    lf_bnds(orec, nobj, v, ll, uu);
    if (ll < -kInfty || uu > kInfty) sing_lf_bnds(orec, nobj, v, sing_ll, sing_uu);
    if (ll > ub + kETol) return;  // SolvedInfeasible, ignored by the caller
    const bool fin = ll > -kInfty;
    if (fin || sing_ll > -kInfty)
      upd_side(orec, nobj, v, s, log, ub - (fin ? ll : sing_ll), false, !fin, tch, false);
    if (tch) changed = true;
    if (++guard > 100000L) break;
  }
}

// tightenInts_ in node mode (LinearHandler.cpp:415-490), over the list of
// Binary/Integer columns in ascending order.
template <class V>
__device__ __forceinline__ bool tighten_ints(const DevLP &lp, const TermRec *irec, V &v, NodeState &s, const ModLog &log,
                             bool act, bool &changed) {
  bool bad = false;  // checkBounds_ over the integer columns, after tightening
  // called with the full wave active: `act` predicates this lane's updates
  for (int c0 = 0; c0 < lp.nint; c0 += kLanes) {
    const int cnt = lp.nint - c0 < kLanes ? lp.nint - c0 : kLanes;
    // full wave active here: the column records broadcast with v_readlane
    const TermChunk ch = load_terms(irec + c0, cnt, v.lane);
    // the columns are distinct, so the bounds of 8 of them are loaded before
    // any is written: one memory round trip per 8 columns instead of one per
    // column (the compiler cannot prove the stores do not alias later loads)
    for (int k0 = 0; k0 < cnt; k0 += kBnd) {
      double lv[kBnd], uv[kBnd];
#pragma unroll
      for (int e = 0; e < kBnd; ++e) {
        const int jj = rl(ch.j, k0 + e < cnt ? k0 + e : k0);
        lv[e] = v.L(jj);
        uv[e] = v.U(jj);
      }
#pragma unroll
      for (int e = 0; e < kBnd; ++e) {
      const int k = k0 + e;
      if (k >= cnt) break;
      const Term1 t{0.0, rlu64(ch.cmask, k), rl(ch.j, k), rl(ch.cs, k), rl(ch.ce, k), 1};
      const int j = t.j;
      const double l = lv[e], u = uv[e];
      if (act && l > -kInfty && fabs(l - floor(l + 0.5)) > kIntTol) {
        const double nv = ceil(l);
        v.change_bflag(t);
        v.L(j) = nv;
        log.push(s, j, 0, nv);
        changed = true;
      }
      double l2 = l, u2 = u;
      if (act && l > -kInfty && fabs(l - floor(l + 0.5)) > kIntTol) l2 = ceil(l);
      if (act && u < kInfty && fabs(u - floor(u + 0.5)) > kIntTol) {
        const double nv = floor(u);
        v.U(j) = nv;
        v.change_bflag(t);
        log.push(s, j, 1, nv);
        changed = true;
        u2 = nv;
      }
      bad |= l2 > u2 + kETol;
      }
    }
  }
  return bad;
}

// checkBounds_ (LinearHandler.cpp:328-359) after tightenInts_, fused: the
// integer columns are checked inside tighten_ints on the bounds it just
// wrote (no second load), the other columns here.  An OR over columns, so
// the order does not matter.  Call with the full wave active: the column
// list is broadcast with v_readlane.
template <class V>
__device__ __forceinline__ bool check_bounds_rest(const DevLP &lp, const V &v, bool bad) {
  for (int c0 = 0; c0 < lp.ncont; c0 += kLanes) {
    const int cnt = lp.ncont - c0 < kLanes ? lp.ncont - c0 : kLanes;
    const int jl = v.lane < cnt ? lp.ccont[c0 + v.lane] : 0;
    for (int k0 = 0; k0 < cnt; k0 += kBnd) {
      double lv[kBnd], uv[kBnd];
#pragma unroll
      for (int e = 0; e < kBnd; ++e) {
        const int j = rl(jl, k0 + e < cnt ? k0 + e : k0);
        lv[e] = v.L(j);
        uv[e] = v.U(j);
      }
#pragma unroll
      for (int e = 0; e < kBnd; ++e)
        if (k0 + e < cnt) bad |= lv[e] > uv[e] + kETol;
    }
  }
  return bad || lp.cons_bad != 0;
}

template <bool kLds, bool kBitFlags, bool kTL>
__global__ __launch_bounds__(kLanes) void fbbt_linear_kernel(DevLP lp, FbbtIO io) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * io.npw;
  const int nb = min(io.npw, io.batch - b0);
  const int n = lp.n, m = lp.m;

  NodeView<kBitFlags, !kLds> v;
  v.lane = lane;
  v.rowidx = lp.rowidx;
  v.bits = 0ull;
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

  // kTL: the row and term records are staged once into LDS (after the
  // bounds, if any): a row visit then reads its records with ds_read
  // (lgkmcnt) instead of global loads that would also wait (vmcnt, in
  // order) for the previous row's bound stores in the global variant.
  const TermRec *trec = lp.trec;
  const RowRec *rows = lp.rows;
  if constexpr (kTL) {
    char *tp = reinterpret_cast<char *>(lds) +
               (kLds ? (size_t)2 * n * kLdsStride * sizeof(double) : 0);
    RowRec *s_rows = reinterpret_cast<RowRec *>(tp);
    TermRec *s_trec = reinterpret_cast<TermRec *>(tp + (size_t)m * sizeof(RowRec));
    const uint4 *src = reinterpret_cast<const uint4 *>(lp.rows);
    uint4 *dst = reinterpret_cast<uint4 *>(s_rows);
    for (int i = lane; i < 2 * m; i += kLanes) dst[i] = src[i];
    src = reinterpret_cast<const uint4 *>(lp.trec);
    dst = reinterpret_cast<uint4 *>(s_trec);
    for (int i = lane; i < 2 * lp.nnz; i += kLanes) dst[i] = src[i];
    trec = s_trec;
    rows = s_rows;
  }
  // Stage the wave's node boxes (row-major [node][var] in HBM) into the
  // [var][lane] layout.  Global variant: var-outer, each lane walks its own
  // node's row (consecutive vars share cache lines) and every store is one
  // coalesced 512-B scratch row.  LDS variant: node-outer, coalesced reads.
  if constexpr (!kLds) {
    if (lane < nb)
      box_in(v, io.lb_in + (size_t)(b0 + lane) * n, io.ub_in + (size_t)(b0 + lane) * n, n);
  }
  for (int nd = 0; nd < (kLds ? nb : 0); ++nd) {
    const double *src_l = io.lb_in + (size_t)(b0 + nd) * n;
    const double *src_u = io.ub_in + (size_t)(b0 + nd) * n;
    for (int j = lane; j < n; j += kLanes) {
      v.lb[j * v.stride + nd] = src_l[j];
      v.ub[j * v.stride + nd] = src_u[j];
    }
  }
  // simplePresolve: every constraint's BFlag set (LinearHandler.cpp:1618-1622)
  if constexpr (kBitFlags) {
    v.bits = m >= 64 ? ~0ull : ((1ull << m) - 1ull);
  } else {
    for (int r = 0; r < m; ++r) v.flag[r * kLanes + lane] = 1;
  }
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
  // objective terms for varBndsFromObj_, loaded once with the full wave
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
    for (int r0 = 0; r0 < m; r0 += kLanes) {
      const int rcnt = m - r0 < kLanes ? m - r0 : kLanes;
      RowRec rr{0.0, 0.0, 0, 0, 0, 0};
      if (lane < rcnt) rr = rows[r0 + lane];
      for (int q = 0; q < rcnt; ++q) {
        const int r = r0 + q;
        const bool mine = cons_on && v.flagged(r);
        if (!__any(mine)) continue;
        // full wave active here: load the row's first 64 terms for broadcast
        const int k0 = rl(rr.k0, q), nt = rl(rr.nt, q);
        // the row bounds broadcast here, in uniform control flow
        const double rlo = rld(rr.lo, q), rhi = rld(rr.hi, q);
        if (mine) {
          bool tch;
          v.clear(r);
          bool inf;
          // row-length classes: fewer masked slots (each costs a division)
          if (nt <= 3) inf = rc_lin_bnd_tighten<3>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 4) inf = rc_lin_bnd_tighten<4>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 5) inf = rc_lin_bnd_tighten<5>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 6) inf = rc_lin_bnd_tighten<6>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 8) inf = rc_lin_bnd_tighten<8>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 11) inf = rc_lin_bnd_tighten<11>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 16) inf = rc_lin_bnd_tighten<16>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else inf = lin_bnd_tighten(trec + k0, nt, rlo, rhi, v, s, log, tch);
          if (inf) {
            cons_on = false;
          } else if (tch) {
            changed = true;
          }
        }
      }
    }
    if (go && io.has_inc && lp.nobj > 0) {
      if (lp.nobj <= 16) rc_bnds_from_obj<16>(lp.nobj, lp.orec, v, s, log, io.inc_ub, changed);
      else bnds_from_obj(lp.orec, lp.nobj, v, s, log, io.inc_ub, changed);
    }
    // both called with the full wave active (v_readlane broadcasts inside)
    const bool bad = check_bounds_rest(lp, v, tighten_ints(lp, lp.irec, v, s, log, go, changed));
    if (go) infeas = bad;
  }
  if (live) {
    io.infeas[b0 + lane] = infeas ? 1 : 0;
    io.nmods[b0 + lane] = s.nmods;
  }
  __syncthreads();
  if constexpr (!kLds) {  // var-outer: coalesced scratch reads (as the staging)
    if (kFbbtOutVarOuter && lane < nb)
      box_out(v, io.lb_out + (size_t)(b0 + lane) * n, io.ub_out + (size_t)(b0 + lane) * n, n);
  }
  for (int nd = 0; nd < (kLds || !kFbbtOutVarOuter ? nb : 0); ++nd) {
    double *dst_l = io.lb_out + (size_t)(b0 + nd) * n;
    double *dst_u = io.ub_out + (size_t)(b0 + nd) * n;
    for (int j = lane; j < n; j += kLanes) {
      dst_l[j] = v.lb[j * v.stride + nd];
      dst_u[j] = v.ub[j * v.stride + nd];
    }
  }
}

// Persistent variant (global scratch, bit flags): a fixed grid of waves
// takes nodes from a device queue.  A lane whose node ends its sweep loop
// (simplePresolve's termination rule) writes the node out at the next sweep
// boundary and takes the next node from the queue, which starts its first
// sweep in that same wave sweep.  The rows and arithmetic per node are
// unchanged (bit-exact); what changes is the packing: the one-node-per-lane
// kernel keeps a whole wave looping until its slowest node's last sweep
// (nodes need 1-6 sweeps, 2.3 on average on tls4-lin), this one refills the
// lanes of the nodes that finished early.
// kWG waves per workgroup share one LDS copy of the records (each wave has
// its own scratch slot and node queue position; no barrier after staging).
// Three waves per SIMD (168 VGPRs, a few spilled): 524 288 tls4-OA nodes
// 8.29 -> 7.75 ms with 12 waves per CU (profiles/r04s).
template <int kWG>
__global__ __launch_bounds__(kLanes * kWG, 3) void fbbt_linear_persist(DevLP lp,
                                                                                   FbbtIO io) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x & (kLanes - 1);
  const int wave = blockIdx.x * kWG + (int)(threadIdx.x / kLanes);
  const int n = lp.n, m = lp.m;
  NodeView<true, true> v;
  v.lane = lane;
  v.rowidx = lp.rowidx;
  v.bits = 0ull;
  v.stride = kLanes;
  v.lb = io.scratch + (size_t)wave * 2 * n * kLanes;
  v.ub = v.lb + (size_t)n * kLanes;
  v.flag = nullptr;
  // row and term records staged once into LDS
  // row, term, objective and integer-column records staged once into LDS
  RowRec *s_rows = reinterpret_cast<RowRec *>(lds);
  TermRec *s_trec = reinterpret_cast<TermRec *>(reinterpret_cast<char *>(lds) +
                                                (size_t)m * sizeof(RowRec));
  TermRec *s_orec = s_trec + lp.nnz;
  TermRec *s_irec = s_orec + lp.nobj;
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(lp.rows);
    uint4 *dst = reinterpret_cast<uint4 *>(s_rows);
    for (int i = threadIdx.x; i < 2 * m; i += kLanes * kWG) dst[i] = src[i];
    src = reinterpret_cast<const uint4 *>(lp.trec);
    dst = reinterpret_cast<uint4 *>(s_trec);
    for (int i = threadIdx.x; i < 2 * lp.nnz; i += kLanes * kWG) dst[i] = src[i];
    src = reinterpret_cast<const uint4 *>(lp.orec);
    dst = reinterpret_cast<uint4 *>(s_orec);
    for (int i = threadIdx.x; i < 2 * lp.nobj; i += kLanes * kWG) dst[i] = src[i];
    src = reinterpret_cast<const uint4 *>(lp.irec);
    dst = reinterpret_cast<uint4 *>(s_irec);
    for (int i = threadIdx.x; i < 2 * lp.nint; i += kLanes * kWG) dst[i] = src[i];
  }
  __syncthreads();
  if (wave >= io.npw) return;   // the grid is rounded up to whole workgroups
  const TermRec *trec = s_trec;
  const RowRec *rows = s_rows;
  const uint64_t all_rows = m >= 64 ? ~0ull : ((1ull << m) - 1ull);
  const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));

  int node = -1;
  bool has = false, changed = false, infeas = false, exhausted = false;
  unsigned iters = 1;
  NodeState s{0, 0u};
  ModLog log{nullptr, nullptr, nullptr, io.mod_cap};
  while (true) {
    bool go = has && changed && iters <= 10u && (iters <= 2u || s.nintmods > 0u) && !infeas;
    // retire: nodes whose sweep loop ended (checked at the sweep boundary,
    // exactly where simplePresolve's loop test runs, LinearHandler.cpp:1625)
    const bool fin = has && !go;
    if (__any(fin)) {
      if (fin) {
        io.infeas[node] = infeas ? 1 : 0;
        io.nmods[node] = s.nmods;
        box_out(v, io.lb_out + (size_t)node * n, io.ub_out + (size_t)node * n, n);
        has = false;
      }
    }
    // refill idle lanes from the queue (one atomic per wave)
    if (!exhausted) {
      const uint64_t idle = __ballot(!has);
      if (idle && (__popcll(idle) >= io.refill_min || idle == ~0ull)) {
        const int cnt = __popcll(idle);
        int base = 0;
        if (lane == (int)__builtin_ctzll(idle)) base = atomicAdd(io.next, cnt);
        base = __shfl(base, (int)__builtin_ctzll(idle), kLanes);
        if (base + cnt >= io.batch) exhausted = true;
        if (!has) {
          const int my = base + __popcll(idle & lt_mask);
          if (my < io.batch) {
            node = my;
            has = true;
            box_in(v, io.lb_in + (size_t)node * n, io.ub_in + (size_t)node * n, n);
            // simplePresolve: every constraint's BFlag set (:1618-1622)
            v.bits = all_rows;
            s.nmods = 0;
            s.nintmods = 0u;
            changed = true;
            infeas = false;
            iters = 1;
            log = ModLog{nullptr, nullptr, nullptr, io.mod_cap};
            if (io.mod_var != nullptr && io.mod_cap > 0) {
              const size_t o = (size_t)node * io.mod_cap;
              log.var = io.mod_var + o;
              log.lu = io.mod_lu + o;
              log.val = io.mod_val + o;
            }
            go = true;
          }
        }
      }
    }
    if (!__any(go)) {
      if (exhausted || !__any(has)) break;
      continue;
    }
    if (go) {
      s.nintmods = 0u;
      changed = false;
      ++iters;
    }
    bool cons_on = go;
    for (int r0 = 0; r0 < m; r0 += kLanes) {
      const int rcnt = m - r0 < kLanes ? m - r0 : kLanes;
      RowRec rr{0.0, 0.0, 0, 0, 0, 0};
      if (lane < rcnt) rr = rows[r0 + lane];
      for (int q = 0; q < rcnt; ++q) {
        const int r = r0 + q;
        const bool mine = cons_on && v.flagged(r);
        if (!__any(mine)) continue;
        const int k0 = rl(rr.k0, q), nt = rl(rr.nt, q);
        // the row bounds broadcast here, in uniform control flow
        const double rlo = rld(rr.lo, q), rhi = rld(rr.hi, q);
        if (mine) {
          bool tch;
          v.clear(r);
          bool inf;
          if (nt <= 3) inf = rc_lin_bnd_tighten<3>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 4) inf = rc_lin_bnd_tighten<4>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 5) inf = rc_lin_bnd_tighten<5>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 6) inf = rc_lin_bnd_tighten<6>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 8) inf = rc_lin_bnd_tighten<8>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 11) inf = rc_lin_bnd_tighten<11>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else if (nt <= 16) inf = rc_lin_bnd_tighten<16>(nt, trec + k0, rlo, rhi, v, s, log, tch);
          else inf = lin_bnd_tighten(trec + k0, nt, rlo, rhi, v, s, log, tch);
          if (inf) {
            cons_on = false;
          } else if (tch) {
            changed = true;
          }
        }
      }
    }
    if (go && io.has_inc && lp.nobj > 0) {
      if (lp.nobj <= 16) rc_bnds_from_obj<16>(lp.nobj, s_orec, v, s, log, io.inc_ub, changed);
      else bnds_from_obj(s_orec, lp.nobj, v, s, log, io.inc_ub, changed);
    }
    const bool bad = check_bounds_rest(lp, v, tighten_ints(lp, s_irec, v, s, log, go, changed));
    if (go) infeas = bad;
  }
}

template <bool kLds, bool kBits, bool kTL>
hipError_t launch_variant(const DevLP &lp, const FbbtIO &io, size_t lds, hipStream_t stream) {
  const int waves = (io.batch + io.npw - 1) / io.npw;
  {
    static bool attr_set = false;  // dynamic LDS above 64 KiB must be opted in
    if (!attr_set) {
      hipError_t e = hipFuncSetAttribute((const void *)fbbt_linear_kernel<kLds, kBits, kTL>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return e;
      attr_set = true;
    }
  }
  hipLaunchKernelGGL((fbbt_linear_kernel<kLds, kBits, kTL>), dim3(waves), dim3(kLanes),
                     lds, stream, lp, io);
  return hipGetLastError();
}

}  // namespace

size_t fbbt_persist_lds(const DevLP &lp) {
  return (size_t)lp.m * sizeof(RowRec) + (size_t)(lp.nnz + lp.nobj + lp.nint) * sizeof(TermRec);
}

size_t fbbt_lds_bytes(int n, int m) {
  return (size_t)2 * n * kLdsStride * sizeof(double) + (m > 64 ? (size_t)m * kLanes : 0);
}

hipError_t launch_fbbt_linear(const DevLP &lp, const FbbtIO &io, int variant,
                              hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  const size_t lds = fbbt_lds_bytes(lp.n, lp.m);
  const bool use_lds = variant == 1 || (variant == 0 && lds <= 160 * 1024);
  const bool bits = lp.m <= 64;
  // records table next to the bounds (LDS variant) or alone (global variant)
  const size_t tab = (size_t)lp.m * sizeof(RowRec) + (size_t)lp.nnz * sizeof(TermRec);
  static const bool no_tl = getenv("MGPU_FBBT_NOTL") != nullptr;  // A/B switch
  if (use_lds) {
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const bool tl = !no_tl && bits && lds + tab <= 160 * 1024;
    if (tl) return launch_variant<true, true, true>(lp, io, lds + tab, stream);
    return bits ? launch_variant<true, true, false>(lp, io, lds, stream)
                : launch_variant<true, false, false>(lp, io, lds, stream);
  }
  if (io.scratch == nullptr || (!bits && io.flag_scratch == nullptr)) return hipErrorInvalidValue;
  if (variant == 3) {  // persistent refill (caller sized the grid in io.npw units)
    const size_t ptab = fbbt_persist_lds(lp);
    if (!bits || io.next == nullptr || ptab > 64 * 1024) return hipErrorInvalidValue;
    static const int wg = getenv("MGPU_FBBT_WG") ? atoi(getenv("MGPU_FBBT_WG")) : 4;
    static bool attr_set = false;
    if (!attr_set) {
      for (const void *f : {(const void *)fbbt_linear_persist<1>,
                            (const void *)fbbt_linear_persist<4>}) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024);
        if (e != hipSuccess) return e;
      }
      attr_set = true;
    }
    if (wg == 1)
      hipLaunchKernelGGL(fbbt_linear_persist<1>, dim3(io.npw), dim3(kLanes), ptab, stream, lp, io);
    else
      hipLaunchKernelGGL(fbbt_linear_persist<4>, dim3((io.npw + 3) / 4), dim3(4 * kLanes), ptab,
                         stream, lp, io);
    return hipGetLastError();
  }
  const bool tl = !no_tl && bits && tab <= 64 * 1024;
  if (tl) return launch_variant<false, true, true>(lp, io, tab, stream);
  return bits ? launch_variant<false, true, false>(lp, io, 0, stream)
              : launch_variant<false, false, false>(lp, io, 0, stream);
}

}  // namespace mgpu
