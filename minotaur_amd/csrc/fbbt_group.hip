// K1G — batched node FBBT over linear rows with 16 lanes per node, gfx950.
//
// The same restatement as K1 (repo:minotaur_amd/csrc/fbbt_linear.hip,
// oracle/fbbt_linear.c): LinearHandler::presolveNode -> simplePresolve in
// node mode (src/base/LinearHandler.cpp:1592-1653), varBndsFromCons_
// (:493-541), linBndTighten_ (:952-1045), updateLfBoundsFromLb_/Ub_
// (:1048-1226), changeBFlag_ (:1229-1234), getLfBnds_ (:1237-1258),
// getSingLfBnds_ (:1261-1319), varBndsFromObj_ (:544-597), tightenInts_
// (:415-490), checkBounds_ (:328-359) — bit for bit, mapped differently:
//
//  * FOUR NODES PER WAVE, 16 lanes each; the lanes of a node hold the terms
//    of the row being tightened.  Inside one update pass a term's new bound
//    depends only on the row's activity bound (fixed for the pass) and its
//    own column's bounds (the columns of a row are distinct), so the 16
//    candidate bounds and their divisions run in parallel.  The activity
//    sums are order-dependent f64 sums: each is a left fold in term order,
//    carried lane to lane by DPP row_shr:1 (lane k adds its product to lane
//    k-1's running sum), exactly the reference's sequential loop.
//  * A node's bounds live in LDS ([lb | ub] per node, 16 B per column), so
//    no global scratch round-trips: HBM traffic is the boxes in and out.
//    Row / term / integer-column records are staged once per workgroup.
//  * Row flags (Constraint::BFlag) are one 64-bit mask per node (m <= 64),
//    group-uniform; changeBFlag_ is an OR-reduction of the changed terms'
//    column masks inside the 16-lane row (DPP).  The wave walks the union of
//    its four nodes' flagged rows in index order, so every node sees its own
//    Gauss-Seidel order; a node whose row proved it infeasible stops its
//    sweep (varBndsFromCons_ returns at once).
//  * Compiled with -ffp-contract=off: no fused multiply-add (the reference's
//    x86-64 build has none).
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

constexpr int kG = 16;          // lanes per node
constexpr int kNG = 64 / kG;    // nodes per wave
constexpr int kMaxW = 16;       // waves per workgroup (LDS permitting)
constexpr int kDppShr1 = 0x111; // row_shr:1 inside each 16-lane row

__device__ __forceinline__ double shr1(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), kDppShr1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kDppShr1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// OR over the 16 lanes of each row (symmetric exchanges: every lane ends
// with the row's OR)
__device__ __forceinline__ uint64_t group_or(uint64_t v) {
  unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  lo |= dpp_i32<kDppXor1>((int)lo);
  hi |= dpp_i32<kDppXor1>((int)hi);
  lo |= dpp_i32<kDppXor2>((int)lo);
  hi |= dpp_i32<kDppXor2>((int)hi);
  lo |= dpp_i32<kDppHalfMirror>((int)lo);
  hi |= dpp_i32<kDppHalfMirror>((int)hi);
  lo |= dpp_i32<kDppMirror>((int)lo);
  hi |= dpp_i32<kDppMirror>((int)hi);
  return ((uint64_t)hi << 32) | lo;
}

// lane `src` of this lane's 16-lane group, to every lane of the group
__device__ __forceinline__ double group_bcast(double v, int src, int lane) {
  return __shfl(v, (lane & ~(kG - 1)) + src, 64);
}

// Left folds of two per-lane values over lanes 0 .. len-1 of every group
// (len wave-uniform), each started from its carry: lane k ends with
// carry + p_0 + ... + p_k added left to right; a skipped lane passes the
// running sum on unchanged.  Returns the group totals in every lane.
__device__ __forceinline__ void fold2(double pa, bool sa, double pb, bool sb, double &ca,
                                      double &cb, int len, int gl, int lane) {
  double va = gl == 0 ? (sa ? ca : ca + pa) : pa;
  double vb = gl == 0 ? (sb ? cb : cb + pb) : pb;
  for (int i = 1; i < len; ++i) {
    const double xa = shr1(va), xb = shr1(vb);
    if (gl == i) {
      va = sa ? xa : xa + pa;
      vb = sb ? xb : xb + pb;
    }
  }
  ca = group_bcast(va, len - 1, lane);
  cb = group_bcast(vb, len - 1, lane);
}

struct GTab {
  const RowRec *rows;
  const TermRec *trec, *orec, *irec;
  const int32_t *ccont;
};

struct GNode {
  double *L, *U;        // this node's bounds in LDS
  uint64_t flags;       // rows to tighten (group-uniform)
  int nmods;            // bound changes (VarBoundMods), group-uniform
  unsigned nint;        // integer-column changes of this sweep
  bool changed;         // this sweep changed a bound
};

// getLfBnds_ (and getSingLfBnds_ when an activity bound is infinite) over
// a term list: ll, uu and the singleton sums, group-uniform
__device__ __forceinline__ void activity(const TermRec *t0, int nt, const GNode &s, int gl,
                                         int lane, double &ll, double &uu, double &sll,
                                         double &suu, double sll0 = -INFINITY) {
  ll = 0.0;
  uu = 0.0;
  for (int c0 = 0; c0 < nt; c0 += kG) {
    const int len = nt - c0 < kG ? nt - c0 : kG;
    double pl = 0.0, pu = 0.0;
    if (gl < len) {
      const TermRec t = t0[c0 + gl];
      const double c = t.a, vl = s.L[t.j], vu = s.U[t.j];
      pl = c > 0 ? c * vl : c * vu;
      pu = c > 0 ? c * vu : c * vl;
    }
    fold2(pl, false, pu, false, ll, uu, len, gl, lane);
  }
  sll = sll0;   // the caller's initial value when no singleton sum is taken
  suu = INFINITY;
  if (ll < -kInfty || uu > kInfty) {
    // the singleton sums: the ordered sum of the finite contributions when at
    // most one is infinite, else the infinite bound (the reference's state
    // machine, :1261-1319); |a| <= eTol terms take no part
    double sl = 0.0, su = 0.0;
    int nl = 0, nu = 0;
    const int g = lane >> 4;
    for (int c0 = 0; c0 < nt; c0 += kG) {
      const int len = nt - c0 < kG ? nt - c0 : kG;
      double pl = 0.0, pu = 0.0;
      bool inf_l = false, inf_u = false, skip = true;
      if (gl < len) {
        const TermRec t = t0[c0 + gl];
        const double c = t.a, vl = s.L[t.j], vu = s.U[t.j];
        if (c > kETol) {
          skip = false;
          pu = c * vu;
          pl = c * vl;
          inf_u = !(vu < kInfty);
          inf_l = !(vl > -kInfty);
        } else if (c < -kETol) {
          skip = false;
          pl = c * vu;
          pu = c * vl;
          inf_l = !(vu < kInfty);
          inf_u = !(vl > -kInfty);
        }
      }
      nl += __popcll((__ballot(!skip && inf_l) >> (16 * g)) & 0xFFFFull);
      nu += __popcll((__ballot(!skip && inf_u) >> (16 * g)) & 0xFFFFull);
      fold2(pl, skip || inf_l, pu, skip || inf_u, sl, su, len, gl, lane);
    }
    sll = nl >= 2 ? -INFINITY : sl;
    suu = nu >= 2 ? INFINITY : su;
  }
}

// updateLfBoundsFromLb_ (from_lb) / updateLfBoundsFromUb_ over a term list:
// every term's candidate bound in parallel, applied at once (distinct
// columns), the changed columns' rows flagged
__device__ __forceinline__ bool update_pass(const TermRec *t0, int nt, GNode &s, bool from_lb,
                                            double rb, double act, bool is_sing, bool count_int,
                                            int gl, int lane) {
  const int g = lane >> 4;
  bool any = false;
  for (int c0 = 0; c0 < nt; c0 += kG) {
    const int len = nt - c0 < kG ? nt - c0 : kG;
    bool hit = false, isint = false;
    uint64_t cm = 0;
    if (gl < len) {
      const TermRec t = t0[c0 + gl];
      const int j = t.j;
      const double c = t.a, vl = s.L[j], vu = s.U[j];
      cm = t.cmask;
      isint = t.isint != 0;
      // from_lb: c > 0 moves lb up, c < 0 moves ub down (:1048-1134);
      // from_ub: c > 0 moves ub down, c < 0 moves lb up (:1137-1226)
      const bool up_side = from_lb ? c > kETol : c < -kETol;    // new lower bound
      const bool dn_side = from_lb ? c < -kETol : c > kETol;    // new upper bound
      if (up_side && (!is_sing || vu >= kInfty)) {
        const double nb0 = (rb - act) / c + (vu >= kInfty ? 0. : vu);
        if (nb0 > vl + kETol) {
          s.L[j] = nb0 > vu - kETol ? vu : nb0;
          hit = true;
        }
      } else if (dn_side && (!is_sing || vl <= -kInfty)) {
        const double nb0 = (rb - act) / c + (vl <= -kInfty ? 0. : vl);
        if (nb0 < vu - kETol) {
          s.U[j] = nb0 < vl + kETol ? vl : nb0;
          hit = true;
        }
      }
    }
    const uint64_t hits = (__ballot(hit) >> (16 * g)) & 0xFFFFull;
    if (hits) {
      s.flags |= group_or(hit ? cm : 0ull);
      s.nmods += __popcll(hits);
      if (count_int) s.nint += __popcll((__ballot(hit && isint) >> (16 * g)) & 0xFFFFull);
      any = true;
    }
  }
  return any;
}

// linBndTighten_ in node mode: false = the row proved the node infeasible
__device__ __forceinline__ bool tighten_row(const RowRec &R, const TermRec *trec, GNode &s,
                                            int gl, int lane) {
  const TermRec *t0 = trec + R.k0;
  double ll, uu, sll, suu;
  activity(t0, R.nt, s, gl, lane, ll, uu, sll, suu);
  if (ll > R.hi + kETol) return false;
  if (uu < R.lo - kETol) return false;
  bool ch = false;
  if (R.lo > -kInfty) {
    if (uu < kInfty) ch = update_pass(t0, R.nt, s, true, R.lo, uu, false, true, gl, lane);
    else if (suu < kInfty) ch = update_pass(t0, R.nt, s, true, R.lo, suu, true, true, gl, lane);
  }
  if (ch) activity(t0, R.nt, s, gl, lane, ll, uu, sll, suu);
  bool ch2 = false;
  if (R.hi < kInfty) {
    if (ll > -kInfty) ch2 = update_pass(t0, R.nt, s, false, R.hi, ll, false, true, gl, lane);
    else if (sll > -kInfty) ch2 = update_pass(t0, R.nt, s, false, R.hi, sll, true, true, gl, lane);
  }
  if (ch || ch2) s.changed = true;
  return true;
}

// varBndsFromObj_ (:544-597): the objective row against the incumbent, to
// a fixed point (the oracle's 100000-pass safety cap)
__device__ __forceinline__ void bnds_from_obj(const TermRec *orec, int nobj, GNode &s,
                                              double inc_ub, int gl, int lane) {
  bool tch = true;
  long guard = 0;
  while (tch) {
    tch = false;
    double ll, uu, sll, suu;
    // varBndsFromObj_ starts its singleton lower sum at +inf (:551)
    activity(orec, nobj, s, gl, lane, ll, uu, sll, suu, INFINITY);
    if (ll > inc_ub + kETol) return;
    if (ll > -kInfty) tch = update_pass(orec, nobj, s, false, inc_ub, ll, false, false, gl, lane);
    else if (sll > -kInfty) tch = update_pass(orec, nobj, s, false, inc_ub, sll, true, false, gl, lane);
    if (tch) s.changed = true;
    if (++guard > 100000L) break;
  }
}

// tightenInts_ (:415-490) then checkBounds_ (:328-359): true = infeasible
__device__ __forceinline__ bool ints_and_check(const GTab &T, int nint, int ncont, int n,
                                               bool cons_bad, GNode &s, int gl, int lane) {
  const int g = lane >> 4;
  bool bad = false;
  for (int c0 = 0; c0 < nint; c0 += kG) {
    const int k = c0 + gl;
    bool hl = false, hu = false;
    uint64_t cm = 0;
    if (k < nint) {
      const TermRec t = T.irec[k];
      const int j = t.j;
      double l = s.L[j], u = s.U[j];
      cm = t.cmask;
      if (l > -kInfty && fabs(l - floor(l + 0.5)) > kIntTol) {
        l = ceil(l);
        s.L[j] = l;
        hl = true;
      }
      if (u < kInfty && fabs(u - floor(u + 0.5)) > kIntTol) {
        u = floor(u);
        s.U[j] = u;
        hu = true;
      }
      bad |= l > u + kETol;
    }
    const uint64_t ml = (__ballot(hl) >> (16 * g)) & 0xFFFFull;
    const uint64_t mu = (__ballot(hu) >> (16 * g)) & 0xFFFFull;
    if (ml | mu) {
      s.flags |= group_or((hl || hu) ? cm : 0ull);
      s.nmods += __popcll(ml) + __popcll(mu);
      s.changed = true;
    }
  }
  for (int c0 = 0; c0 < ncont; c0 += kG) {
    const int k = c0 + gl;
    if (k < ncont) {
      const int j = T.ccont[k];
      bad |= s.L[j] > s.U[j] + kETol;
    }
  }
  (void)n;
  return ((__ballot(bad) >> (16 * g)) & 0xFFFFull) != 0 || cons_bad;
}

__global__ __launch_bounds__(64 * kMaxW) void fbbt_group_kernel(DevLP lp, FbbtIO io) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, gl = lane & (kG - 1);
  // ---- stage the records once per workgroup ----
  unsigned char *p = smem;
  RowRec *s_rows = (RowRec *)p;   p += sizeof(RowRec) * (size_t)m;
  TermRec *s_trec = (TermRec *)p; p += sizeof(TermRec) * (size_t)lp.nnz;
  TermRec *s_orec = (TermRec *)p; p += sizeof(TermRec) * (size_t)lp.nobj;
  TermRec *s_irec = (TermRec *)p; p += sizeof(TermRec) * (size_t)lp.nint;
  int32_t *s_ccont = (int32_t *)p; p += ((sizeof(int32_t) * (size_t)lp.ncont + 15) & ~(size_t)15);
  for (int t = threadIdx.x; t < m; t += blockDim.x) s_rows[t] = lp.rows[t];
  for (int t = threadIdx.x; t < lp.nnz; t += blockDim.x) s_trec[t] = lp.trec[t];
  for (int t = threadIdx.x; t < lp.nobj; t += blockDim.x) s_orec[t] = lp.orec[t];
  for (int t = threadIdx.x; t < lp.nint; t += blockDim.x) s_irec[t] = lp.irec[t];
  for (int t = threadIdx.x; t < lp.ncont; t += blockDim.x) s_ccont[t] = lp.ccont[t];
  __syncthreads();
  const GTab T{s_rows, s_trec, s_orec, s_irec, s_ccont};

  // ---- this lane's node ----
  double *nb = (double *)p + (size_t)(wave * kNG + g) * 2 * n;
  const long b = ((long)blockIdx.x * W + wave) * kNG + g;
  const bool live = b < io.batch;
  GNode s{nb, nb + n, 0ull, 0, 0u, true};
  if (live) {
    for (int j = gl; j < n; j += kG) {
      s.L[j] = io.lb_in[(size_t)b * n + j];
      s.U[j] = io.ub_in[(size_t)b * n + j];
    }
    s.flags = m == 64 ? ~0ull : ((1ull << m) - 1ull);
  }
  wave_sync();
  // simplePresolve's sweep loop (:1620-1650), per node
  unsigned iters = 1;
  bool infeas = false;
  bool run = live;
  for (;;) {
    run = run && s.changed && iters <= 10u && (iters <= 2u || s.nint > 0u) && !infeas;
    if (__ballot(run) == 0ull) break;
    if (run) {
      s.nint = 0u;
      s.changed = false;
      ++iters;
    }
    // varBndsFromCons_: the wave walks the union of its running nodes'
    // flagged rows in index order; a node tightens the rows it has flagged
    // when the walk reaches them (flags set by earlier rows of this sweep
    // included), and stops at a row that proves it infeasible
    bool cut = !run;
    int r = -1;
    for (;;) {
      uint64_t want = cut ? 0ull : s.flags;
      uint64_t un = rlu64(want, 0) | rlu64(want, 16) | rlu64(want, 32) | rlu64(want, 48);
      un &= r >= 63 ? 0ull : (~0ull << (r + 1));
      if (un == 0ull) break;
      r = __builtin_ctzll(un);
      if (!cut && ((s.flags >> r) & 1ull)) {
        s.flags &= ~(1ull << r);
        if (!tighten_row(T.rows[r], T.trec, s, gl, lane)) cut = true;
      }
      wave_sync();
    }
    if (run) {
      if (io.has_inc && lp.nobj > 0) bnds_from_obj(T.orec, lp.nobj, s, io.inc_ub, gl, lane);
      infeas = ints_and_check(T, lp.nint, lp.ncont, n, lp.cons_bad != 0, s, gl, lane);
    }
    wave_sync();
  }
  if (live) {
    for (int j = gl; j < n; j += kG) {
      io.lb_out[(size_t)b * n + j] = s.L[j];
      io.ub_out[(size_t)b * n + j] = s.U[j];
    }
    if (gl == 0) {
      io.infeas[b] = infeas ? 1 : 0;
      io.nmods[b] = s.nmods;
    }
  }
}

size_t group_table_bytes(const DevLP &lp) {
  return sizeof(RowRec) * (size_t)lp.m + sizeof(TermRec) * (size_t)(lp.nnz + lp.nobj + lp.nint) +
         ((sizeof(int32_t) * (size_t)lp.ncont + 15) & ~(size_t)15);
}

}  // namespace

int fbbt_group_waves(const DevLP &lp) {
  if (lp.m > 64 || lp.n <= 0) return 0;
  const size_t tab = group_table_bytes(lp), per_wave = (size_t)kNG * 2 * lp.n * sizeof(double);
  if (tab + per_wave > 160 * 1024) return 0;
  const size_t w = (160 * 1024 - tab) / per_wave;
  return w > (size_t)kMaxW ? kMaxW : (int)w;
}

hipError_t launch_fbbt_group(const DevLP &lp, const FbbtIO &io, hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  const int W = fbbt_group_waves(lp);
  if (W <= 0 || io.mod_cap > 0) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)fbbt_group_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const long waves = ((long)io.batch + kNG - 1) / kNG;
  const long blocks = (waves + W - 1) / W;
  const size_t lds = group_table_bytes(lp) + (size_t)W * kNG * 2 * lp.n * sizeof(double);
  hipLaunchKernelGGL(fbbt_group_kernel, dim3((unsigned)blocks), dim3(64 * W), lds, stream, lp, io);
  return hipGetLastError();
}

}  // namespace mgpu
