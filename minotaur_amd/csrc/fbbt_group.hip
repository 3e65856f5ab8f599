// K1G — batched node FBBT over linear rows with G lanes per node (G = 16, 8
// or 4), gfx950.
//
// The same restatement as K1 (repo:minotaur_amd/csrc/fbbt_linear.hip,
// oracle/fbbt_linear.c): LinearHandler::presolveNode -> simplePresolve in
// node mode (src/base/LinearHandler.cpp:1592-1653), varBndsFromCons_
// (:493-541), linBndTighten_ (:952-1045), updateLfBoundsFromLb_/Ub_
// (:1048-1226), changeBFlag_ (:1229-1234), getLfBnds_ (:1237-1258),
// getSingLfBnds_ (:1261-1319), varBndsFromObj_ (:544-597), tightenInts_
// (:415-490), checkBounds_ (:328-359) — bit for bit, mapped differently:
//
//  * 64 / G NODES PER WAVE, G lanes each; the lanes of a node hold the terms
//    of the row being tightened (G at a time).  Inside one update pass a
//    term's new bound depends only on the row's activity bound (fixed for the
//    pass) and its own column's bounds (the columns of a row are distinct),
//    so the G candidate bounds and their divisions run in parallel.
//  * The activity sums are order-dependent f64 sums.  Each lane writes its
//    term's two products to the node's product slots in LDS and every lane
//    of the node then adds the chunk's products in term order (broadcast
//    reads): the reference's sequential loop, bit for bit, in ~1.5 VALU
//    instructions per term (the round-4 DPP left fold took ~12).  A skipped
//    term (singleton sums) contributes +0.0, which leaves the running sum
//    unchanged: that sum starts at +0.0 and can never be -0.0.
//  * A node's bounds live in LDS ((lb, ub) interleaved per column, one
//    ds_read_b128 per term), so no global scratch round-trips: HBM traffic is
//    the boxes in and out.  Row / term / integer-column records are staged
//    once per workgroup.
//  * Row flags (Constraint::BFlag) are one 64-bit mask per node (m <= 64),
//    group-uniform; changeBFlag_ is an OR-reduction of the changed terms'
//    column masks inside the G-lane group (DPP).  The wave walks the union of
//    its nodes' flagged rows in index order, so every node sees its own
//    Gauss-Seidel order; a node whose row proved it infeasible stops its
//    sweep (varBndsFromCons_ returns at once).
//  * Compiled with -ffp-contract=off: no fused multiply-add (the reference's
//    x86-64 build has none).
#include "mgpu_internal.h"
#include "wave.h"

namespace mgpu {
namespace {

constexpr int kMaxW = 16;       // waves per workgroup (LDS permitting)

// OR over the G lanes of each group (symmetric exchanges: every lane ends
// with the group's OR)
template <int G>
__device__ __forceinline__ uint64_t group_or(uint64_t v) {
  unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  lo |= dpp_i32<kDppXor1>((int)lo);
  hi |= dpp_i32<kDppXor1>((int)hi);
  lo |= dpp_i32<kDppXor2>((int)lo);
  hi |= dpp_i32<kDppXor2>((int)hi);
  if constexpr (G >= 8) {
    lo |= dpp_i32<kDppHalfMirror>((int)lo);
    hi |= dpp_i32<kDppHalfMirror>((int)hi);
  }
  if constexpr (G >= 16) {
    lo |= dpp_i32<kDppMirror>((int)lo);
    hi |= dpp_i32<kDppMirror>((int)hi);
  }
  return ((uint64_t)hi << 32) | lo;
}

// this lane's group's bits of a ballot
template <int G>
__device__ __forceinline__ uint64_t gbits(uint64_t ballot, int g) {
  constexpr uint64_t kMask = G == 64 ? ~0ull : ((1ull << G) - 1ull);
  return (ballot >> (G * g)) & kMask;
}

struct GTab {
  const RowRec *rows;
  const TermRec *trec, *orec, *irec;
  const int32_t *ccont;
};

struct GNode {
  double2 *B;           // this node's (lb, ub) per column, LDS
  double2 *P;           // this node's product slots (G of them), LDS
  uint64_t flags;       // rows to tighten (group-uniform)
  int nmods;            // bound changes (VarBoundMods), group-uniform
  unsigned nint;        // integer-column changes of this sweep
  bool changed;         // this sweep changed a bound
};

// Adds the chunk's products (pl, pu) of lanes 0 .. len-1 to (ll, uu) in term
// order, in every lane of the group.  The slots are read four at a time
// (loads in flight together), the adds stay in term order.
template <int G>
__device__ __forceinline__ void chunk_sum(GNode &s, double pl, double pu, bool wr, int gl,
                                          int len, double &ll, double &uu) {
  if (wr) s.P[gl] = make_double2(pl, pu);
  wave_sync();
  for (int k0 = 0; k0 < len; k0 += 4) {
    double2 q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = s.P[k0 + e];   // k0 + 3 < G: inside the slots
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (k0 + e < len) {
        ll += q[e].x;
        uu += q[e].y;
      }
  }
  wave_sync();   // the next chunk's writes after these reads
}

// One lane's term of a chunk: its record and its column's bounds
struct Slot {
  double a;
  uint64_t cm;
  int j;
  bool isint, on;
  double2 b;
};

__device__ __forceinline__ Slot slot_load(const TermRec *t0, int c0, int len, int gl,
                                          const GNode &s) {
  Slot sl{0.0, 0ull, 0, false, false, make_double2(0.0, 0.0)};
  if (gl < len) {
    const TermRec t = t0[c0 + gl];
    sl.a = t.a;
    sl.cm = t.cmask;
    sl.j = t.j;
    sl.isint = t.isint != 0;
    sl.on = true;
    sl.b = s.B[t.j];
  }
  return sl;
}

// getLfBnds_ products of one term
__device__ __forceinline__ void slot_prod(const Slot &sl, double &pl, double &pu) {
  pl = sl.a > 0 ? sl.a * sl.b.x : sl.a * sl.b.y;
  pu = sl.a > 0 ? sl.a * sl.b.y : sl.a * sl.b.x;
}

// getSingLfBnds_ contributions of one term: the finite product, or +0.0 and
// a flag for an infinite one; |a| <= eTol terms take no part
__device__ __forceinline__ void slot_sing(const Slot &sl, double &pl, double &pu, bool &inf_l,
                                          bool &inf_u) {
  const double c = sl.a, vl = sl.b.x, vu = sl.b.y;
  pl = 0.0;
  pu = 0.0;
  inf_l = false;
  inf_u = false;
  if (!sl.on) return;
  if (c > kETol) {
    inf_u = !(vu < kInfty);
    inf_l = !(vl > -kInfty);
    pu = inf_u ? 0.0 : c * vu;
    pl = inf_l ? 0.0 : c * vl;
  } else if (c < -kETol) {
    inf_l = !(vu < kInfty);
    inf_u = !(vl > -kInfty);
    pl = inf_l ? 0.0 : c * vu;
    pu = inf_u ? 0.0 : c * vl;
  }
}

// updateLfBoundsFromLb_ (from_lb) / updateLfBoundsFromUb_ for one term:
// from_lb: c > 0 moves lb up, c < 0 moves ub down (:1048-1134); from_ub:
// c > 0 moves ub down, c < 0 moves lb up (:1137-1226).  The new bound goes
// to the slot and to LDS.
__device__ __forceinline__ bool slot_update(Slot &sl, GNode &s, bool from_lb, double rb,
                                            double act, bool is_sing) {
  if (!sl.on) return false;
  const double c = sl.a, vl = sl.b.x, vu = sl.b.y;
  const bool up_side = from_lb ? c > kETol : c < -kETol;    // new lower bound
  const bool dn_side = from_lb ? c < -kETol : c > kETol;    // new upper bound
  if (up_side && (!is_sing || vu >= kInfty)) {
    const double nb0 = (rb - act) / c + (vu >= kInfty ? 0. : vu);
    if (nb0 > vl + kETol) {
      sl.b.x = nb0 > vu - kETol ? vu : nb0;
      s.B[sl.j].x = sl.b.x;
      return true;
    }
  } else if (dn_side && (!is_sing || vl <= -kInfty)) {
    const double nb0 = (rb - act) / c + (vl <= -kInfty ? 0. : vl);
    if (nb0 < vu - kETol) {
      sl.b.y = nb0 < vl + kETol ? vl : nb0;
      s.B[sl.j].y = sl.b.y;
      return true;
    }
  }
  return false;
}

// getLfBnds_ (and getSingLfBnds_ when an activity bound is infinite) over
// a term list: ll, uu and the singleton sums, group-uniform.  `one`: the
// list is a single chunk already loaded into `sl`.
template <int G, bool one>
__device__ __forceinline__ void activity(const TermRec *t0, int nt, GNode &s, int gl, int g,
                                         const Slot &sl, double &ll, double &uu,
                                         double &sll, double &suu, double sll0 = -INFINITY) {
  ll = 0.0;
  uu = 0.0;
  for (int c0 = 0; c0 < nt; c0 += G) {
    const int len = nt - c0 < G ? nt - c0 : G;
    Slot t;
    if constexpr (one) t = sl; else t = slot_load(t0, c0, len, gl, s);
    double pl = 0.0, pu = 0.0;
    if (t.on) slot_prod(t, pl, pu);
    chunk_sum<G>(s, pl, pu, t.on, gl, len, ll, uu);
  }
  sll = sll0;   // the caller's initial value when no singleton sum is taken
  suu = INFINITY;
  if (ll < -kInfty || uu > kInfty) {
    // the ordered sum of the finite contributions when at most one is
    // infinite, else the infinite bound (the reference's state machine,
    // :1261-1319)
    double sl_ = 0.0, su = 0.0;
    int nl = 0, nu = 0;
    for (int c0 = 0; c0 < nt; c0 += G) {
      const int len = nt - c0 < G ? nt - c0 : G;
      Slot t;
      if constexpr (one) t = sl; else t = slot_load(t0, c0, len, gl, s);
      double pl, pu;
      bool inf_l, inf_u;
      slot_sing(t, pl, pu, inf_l, inf_u);
      nl += __popcll(gbits<G>(__ballot(inf_l), g));
      nu += __popcll(gbits<G>(__ballot(inf_u), g));
      chunk_sum<G>(s, pl, pu, t.on, gl, len, sl_, su);
    }
    sll = nl >= 2 ? -INFINITY : sl_;
    suu = nu >= 2 ? INFINITY : su;
  }
}

// updateLfBoundsFrom{Lb,Ub}_ over a term list: every term's candidate bound
// in parallel, applied at once (distinct columns), the changed columns' rows
// flagged
template <int G, bool one>
__device__ __forceinline__ bool update_pass(const TermRec *t0, int nt, GNode &s, Slot &sl,
                                            bool from_lb, double rb, double act,
                                            bool is_sing, bool count_int, int gl, int g) {
  bool any = false;
  for (int c0 = 0; c0 < nt; c0 += G) {
    const int len = nt - c0 < G ? nt - c0 : G;
    Slot t;
    if constexpr (one) t = sl; else t = slot_load(t0, c0, len, gl, s);
    const bool hit = slot_update(t, s, from_lb, rb, act, is_sing);
    if constexpr (one) sl = t;
    const uint64_t hits = gbits<G>(__ballot(hit), g);
    if (hits) {
      s.flags |= group_or<G>(hit ? t.cm : 0ull);
      s.nmods += __popcll(hits);
      if (count_int) s.nint += __popcll(gbits<G>(__ballot(hit && t.isint), g));
      any = true;
    }
  }
  return any;
}

// linBndTighten_ in node mode: false = the row proved the node infeasible.
// one: the row has at most G terms, loaded once into the lanes' slots and
// kept there (updated in place) through its passes.
template <int G, bool one>
__device__ __forceinline__ bool tighten_row_(const RowRec &R, const TermRec *trec, GNode &s,
                                             int gl, int g) {
  const TermRec *t0 = trec + R.k0;
  Slot sl{0.0, 0ull, 0, false, false, {0.0, 0.0}};
  if constexpr (one) sl = slot_load(t0, 0, R.nt, gl, s);
  double ll, uu, sll, suu;
  activity<G, one>(t0, R.nt, s, gl, g, sl, ll, uu, sll, suu);
  if (ll > R.hi + kETol) return false;
  if (uu < R.lo - kETol) return false;
  bool ch = false;
  if (R.lo > -kInfty) {
    if (uu < kInfty) ch = update_pass<G, one>(t0, R.nt, s, sl, true, R.lo, uu, false, true, gl, g);
    else if (suu < kInfty) ch = update_pass<G, one>(t0, R.nt, s, sl, true, R.lo, suu, true, true, gl, g);
  }
  if (ch) activity<G, one>(t0, R.nt, s, gl, g, sl, ll, uu, sll, suu);
  bool ch2 = false;
  if (R.hi < kInfty) {
    if (ll > -kInfty) ch2 = update_pass<G, one>(t0, R.nt, s, sl, false, R.hi, ll, false, true, gl, g);
    else if (sll > -kInfty) ch2 = update_pass<G, one>(t0, R.nt, s, sl, false, R.hi, sll, true, true, gl, g);
  }
  if (ch || ch2) s.changed = true;
  return true;
}

// A row of at most H terms in two phases, for the paired-row walk below:
// phase 1 loads it into the slots and takes its activity bounds, and returns
// its verdict (false: the row proves the node infeasible) before any bound
// moves; phase 2 is the rest of linBndTighten_ (tighten_row_<H, true>'s
// operations in its order).
template <int H>
__device__ __forceinline__ bool row_phase1(const RowRec &R, const TermRec *trec, GNode &s, int gl,
                                           int g, Slot &sl, double &ll, double &uu, double &sll,
                                           double &suu) {
  const TermRec *t0 = trec + R.k0;
  sl = slot_load(t0, 0, R.nt, gl, s);
  activity<H, true>(t0, R.nt, s, gl, g, sl, ll, uu, sll, suu);
  return !(ll > R.hi + kETol) && !(uu < R.lo - kETol);
}

template <int H>
__device__ __forceinline__ void row_phase2(const RowRec &R, const TermRec *trec, GNode &s, int gl,
                                           int g, Slot &sl, double ll, double uu, double sll,
                                           double suu) {
  const TermRec *t0 = trec + R.k0;
  bool ch = false;
  if (R.lo > -kInfty) {
    if (uu < kInfty) ch = update_pass<H, true>(t0, R.nt, s, sl, true, R.lo, uu, false, true, gl, g);
    else if (suu < kInfty) ch = update_pass<H, true>(t0, R.nt, s, sl, true, R.lo, suu, true, true, gl, g);
  }
  if (ch) activity<H, true>(t0, R.nt, s, gl, g, sl, ll, uu, sll, suu);
  bool ch2 = false;
  if (R.hi < kInfty) {
    if (ll > -kInfty) ch2 = update_pass<H, true>(t0, R.nt, s, sl, false, R.hi, ll, false, true, gl, g);
    else if (sll > -kInfty) ch2 = update_pass<H, true>(t0, R.nt, s, sl, false, R.hi, sll, true, true, gl, g);
  }
  if (ch || ch2) s.changed = true;
}

template <int G>
__device__ __forceinline__ bool tighten_row(const RowRec &R, const TermRec *trec, GNode &s,
                                            int gl, int g) {
  return R.nt <= G ? tighten_row_<G, true>(R, trec, s, gl, g)
                   : tighten_row_<G, false>(R, trec, s, gl, g);
}

// varBndsFromObj_ (:544-597): the objective row against the incumbent, to
// a fixed point (the oracle's 100000-pass safety cap)
template <int G, bool one>
__device__ __forceinline__ void bnds_from_obj_(const TermRec *orec, int nobj, GNode &s,
                                               double inc_ub, int gl, int g) {
  Slot sl{0.0, 0ull, 0, false, false, {0.0, 0.0}};
  if constexpr (one) sl = slot_load(orec, 0, nobj, gl, s);
  bool tch = true;
  long guard = 0;
  while (tch) {
    tch = false;
    double ll, uu, sll, suu;
    // varBndsFromObj_ starts its singleton lower sum at +inf (:551)
    activity<G, one>(orec, nobj, s, gl, g, sl, ll, uu, sll, suu, INFINITY);
    if (ll > inc_ub + kETol) return;
    if (ll > -kInfty) tch = update_pass<G, one>(orec, nobj, s, sl, false, inc_ub, ll, false, false, gl, g);
    else if (sll > -kInfty) tch = update_pass<G, one>(orec, nobj, s, sl, false, inc_ub, sll, true, false, gl, g);
    if (tch) s.changed = true;
    if (++guard > 100000L) break;
  }
}

template <int G>
__device__ __forceinline__ void bnds_from_obj(const TermRec *orec, int nobj, GNode &s,
                                              double inc_ub, int gl, int g) {
  if (nobj <= G) bnds_from_obj_<G, true>(orec, nobj, s, inc_ub, gl, g);
  else bnds_from_obj_<G, false>(orec, nobj, s, inc_ub, gl, g);
}

// tightenInts_ (:415-490) then checkBounds_ (:328-359): true = infeasible
template <int G>
__device__ __forceinline__ bool ints_and_check(const GTab &T, int nint, int ncont, bool cons_bad,
                                               GNode &s, int gl, int g) {
  bool bad = false;
  for (int c0 = 0; c0 < nint; c0 += G) {
    const int k = c0 + gl;
    bool hl = false, hu = false;
    uint64_t cm = 0;
    if (k < nint) {
      const TermRec t = T.irec[k];
      const int j = t.j;
      const double2 b = s.B[j];
      double l = b.x, u = b.y;
      cm = t.cmask;
      if (l > -kInfty && fabs(l - floor(l + 0.5)) > kIntTol) {
        l = ceil(l);
        hl = true;
      }
      if (u < kInfty && fabs(u - floor(u + 0.5)) > kIntTol) {
        u = floor(u);
        hu = true;
      }
      if (hl || hu) s.B[j] = make_double2(l, u);
      bad |= l > u + kETol;
    }
    const uint64_t ml = gbits<G>(__ballot(hl), g);
    const uint64_t mu = gbits<G>(__ballot(hu), g);
    if (ml | mu) {
      s.flags |= group_or<G>((hl || hu) ? cm : 0ull);
      s.nmods += __popcll(ml) + __popcll(mu);
      s.changed = true;
    }
  }
  for (int c0 = 0; c0 < ncont; c0 += G) {
    const int k = c0 + gl;
    if (k < ncont) {
      const double2 b = s.B[T.ccont[k]];
      bad |= b.x > b.y + kETol;
    }
  }
  return gbits<G>(__ballot(bad), g) != 0 || cons_bad;
}

// per-node LDS: (lb, ub) per column and G product slots
__host__ __device__ constexpr size_t node_bytes(int n, int G) {
  return (size_t)(n + G) * sizeof(double2);
}

template <int G>
__global__ __launch_bounds__(64 * kMaxW) void fbbt_group_kernel(DevLP lp, FbbtIO io) {
  constexpr int kNG = 64 / G;    // nodes per wave
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = lp.n, m = lp.m;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane / G, gl = lane & (G - 1);
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

  // Rows r and r + 1 that can be tightened at once, one per half of a
  // node's lanes (G = 16): both of at most G / 2 terms, no column in common.
  // Row r then cannot flag row r + 1, and their bound updates touch
  // different columns, so the pair gives the sequential walk's result.
  uint64_t pairs = 0ull;
  if constexpr (G == 16) {
    bool ok = false;
    if (lane + 1 < m) {
      const RowRec ra = s_rows[lane], rb = s_rows[lane + 1];
      if (ra.nt <= G / 2 && rb.nt <= G / 2) {
        uint64_t cols = 0ull;
        for (int k = 0; k < ra.nt; ++k) cols |= s_trec[ra.k0 + k].cmask;
        ok = ((cols >> (lane + 1)) & 1ull) == 0ull;
      }
    }
    pairs = __ballot(ok);
  }

  // ---- this lane's node ----
  double2 *nb = (double2 *)(p + (size_t)(wave * kNG + g) * node_bytes(n, G));
  const long b = ((long)blockIdx.x * W + wave) * kNG + g;
  const bool live = b < io.batch;
  GNode s{nb, nb + n, 0ull, 0, 0u, true};
  if (live) {
    for (int j = gl; j < n; j += G)
      s.B[j] = make_double2(io.lb_in[(size_t)b * n + j], io.ub_in[(size_t)b * n + j]);
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
      const uint64_t want = cut ? 0ull : s.flags;
      uint64_t un = 0ull;
#pragma unroll
      for (int q = 0; q < kNG; ++q) un |= rlu64(want, q * G);
      un &= r >= 63 ? 0ull : (~0ull << (r + 1));
      if (un == 0ull) break;
      r = __builtin_ctzll(un);
      if (G == 16 && ((pairs >> r) & 1ull) && ((un >> (r + 1)) & 1ull)) {
        // rows r (lanes 0..7 of each node) and r + 1 (lanes 8..15) at once;
        // each half works on a copy of the node's state, merged after
        constexpr int H = G / 2;
        const int hg = lane / H, hl = lane & (H - 1);
        const bool inB = gl >= H;
        const bool fA = !cut && ((s.flags >> r) & 1ull);
        const bool fB = !cut && ((s.flags >> (r + 1)) & 1ull);
        if (fA) s.flags &= ~(1ull << r);
        if (fB) s.flags &= ~(1ull << (r + 1));
        GNode h = s;
        if (inB) h.P = s.P + H;   // the upper half's product slots
        const RowRec &R = T.rows[inB ? r + 1 : r];
        const bool act = inB ? fB : fA;
        Slot sl{0.0, 0ull, 0, false, false, {0.0, 0.0}};
        double ll = 0.0, uu = 0.0, sll = 0.0, suu = 0.0;
        bool feas = true;
        if (act) feas = row_phase1<H>(R, T.trec, h, hl, hg, sl, ll, uu, sll, suu);
        wave_sync();
        // row r's verdict (lane 0 of the node): an infeasible row r ends the
        // node's walk before row r + 1, as in the sequential walk
        const int a_inf = __shfl((act && !feas) ? 1 : 0, lane & ~(G - 1), 64);
        if (act && feas && !(inB && a_inf))
          row_phase2<H>(R, T.trec, h, hl, hg, sl, ll, uu, sll, suu);
        wave_sync();
        const int b_inf = __shfl((act && !feas) ? 1 : 0, (lane & ~(G - 1)) + H, 64);
        const int dm = h.nmods - s.nmods, dn = (int)(h.nint - s.nint);
        const int om = __shfl_xor(dm, H, 64), on = __shfl_xor(dn, H, 64);
        const int oc = __shfl_xor(h.changed ? 1 : 0, H, 64);
        s.flags = group_or<G>(h.flags);
        // row r proved the node infeasible: row r + 1 was not visited and
        // keeps its flag (simplePresolve ignores the verdict, :1620-1650, so
        // the next sweep visits it)
        if (a_inf && fB) s.flags |= 1ull << (r + 1);
        s.nmods += dm + om;
        s.nint += (unsigned)(dn + on);
        s.changed = h.changed || oc != 0;
        if (a_inf || (b_inf && fB)) cut = true;
        r = r + 1;
      } else if (!cut && ((s.flags >> r) & 1ull)) {
        s.flags &= ~(1ull << r);
        if (!tighten_row<G>(T.rows[r], T.trec, s, gl, g)) cut = true;
      }
      wave_sync();
    }
    if (run) {
      if (io.has_inc && lp.nobj > 0) bnds_from_obj<G>(T.orec, lp.nobj, s, io.inc_ub, gl, g);
      infeas = ints_and_check<G>(T, lp.nint, lp.ncont, lp.cons_bad != 0, s, gl, g);
    }
    wave_sync();
  }
  if (live) {
    for (int j = gl; j < n; j += G) {
      const double2 v = s.B[j];
      io.lb_out[(size_t)b * n + j] = v.x;
      io.ub_out[(size_t)b * n + j] = v.y;
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

template <int G>
hipError_t launch_g(const DevLP &lp, const FbbtIO &io, int W, hipStream_t stream) {
  constexpr int kNG = 64 / G;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)fbbt_group_kernel<G>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const long waves = ((long)io.batch + kNG - 1) / kNG;
  const long blocks = (waves + W - 1) / W;
  const size_t lds = group_table_bytes(lp) + (size_t)W * kNG * node_bytes(lp.n, G);
  hipLaunchKernelGGL(fbbt_group_kernel<G>, dim3((unsigned)blocks), dim3(64 * W), lds, stream, lp, io);
  return hipGetLastError();
}

}  // namespace

int fbbt_group_waves(const DevLP &lp, int g) {
  if (lp.m > 64 || lp.n <= 0 || (g != 4 && g != 8 && g != 16)) return 0;
  const size_t tab = group_table_bytes(lp), per_wave = (size_t)(64 / g) * node_bytes(lp.n, g);
  if (tab + per_wave > 160 * 1024) return 0;
  const size_t w = (160 * 1024 - tab) / per_wave;
  return w > (size_t)kMaxW ? kMaxW : (int)w;
}

hipError_t launch_fbbt_group(const DevLP &lp, const FbbtIO &io, int g, int num_cus,
                             hipStream_t stream) {
  if (io.batch <= 0) return hipSuccess;
  int W = fbbt_group_waves(lp, g);
  if (W <= 0 || io.mod_cap > 0) return hipErrorInvalidValue;
  // a batch of fewer than W waves per CU is spread over every CU (one
  // workgroup per CU, fewer waves each): 16-wave workgroups would pile a
  // small batch onto a few CUs, four waves to a SIMD
  const long waves = ((long)io.batch * g + 63) / 64;
  const long per_cu = (waves + num_cus - 1) / (num_cus > 0 ? num_cus : 1);
  if (per_cu < W) W = per_cu < 1 ? 1 : (int)per_cu;
  switch (g) {
    case 4: return launch_g<4>(lp, io, W, stream);
    case 8: return launch_g<8>(lp, io, W, stream);
    default: return launch_g<16>(lp, io, W, stream);
  }
}

}  // namespace mgpu
