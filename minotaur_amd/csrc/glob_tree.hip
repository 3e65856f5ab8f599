// Batched spatial branch-and-bound over the McCormick relaxation (the glob
// path), gfx950: the node decision, summary and child
// writer of one round of mgpu_glob_round (glob_runtime.cpp).
//
// The reference's mglob runs BranchAndBound with the handlers IntVarHandler,
// LinearHandler, QuadHandler (SimpleTransformer.cpp:940-963) and, with the
// option brancher=maxvio, MaxVioBrancher (Glob.cpp:134-192).  After a node's
// presolve (K2, QuadHandler::presolveNode) and LP (K3R + K3 with the node's
// rewritten McCormick / secant rows), PCBProcessor decides:
//   * shouldPrune_ (PCBProcessor.cpp:400-523): the engine-status switch and
//     the bound test against the incumbent (solAbs_tol / solRel_tol 1e-6);
//   * isFeasible: IntVarHandler::isFeasible (IntVarHandler.cpp:54-84) and
//     QuadHandler::isFeasible (QuadHandler.cpp:904-953: every original
//     quadratic constraint's activity within aTol_ 1e-6 / rTol_ 1e-7, and a
//     quadratic objective's value against the relaxation's);
//   * otherwise MaxVioBrancher::findBranches (MaxVioBrancher.cpp): candidates
//     from IntVarHandler (IntVarHandler.cpp:86-110: dd = x - floor x,
//     ud = ceil x - x) then QuadHandler (QuadHandler.cpp:473-614: y = x^2
//     violated from above, y = x0 x1 violated per LinBil::isViolated, a
//     variable at its bounds is not a candidate), merged per variable (the
//     later handler takes over when its distance sum is >= the earlier
//     one's; the distances stay the earlier handler's, because the merge's
//     setDist resolves to the empty BrCand::setDist), score 0.8 min + 0.2 max (x 0.1 for the
//     original variables: every candidate here), the first maximum in
//     variable order; up branch first when dd > ud.  IntVarHandler branches
//     at floor / ceil (IntVarHandler.cpp:133-175), QuadHandler at the value
//     itself (QuadHandler.cpp:422-471).
// One thread per node: the decision is a few hundred flops of sequential,
// order-dependent sums (the CPU restatement, oracle/glob.py, adds in the
// same order, so decisions and scores are bit-identical); the per-variable
// candidate sums live in a [node][var] scratch.
#include "glob_internal.h"

namespace mgpu {
namespace {

constexpr double kQATol = 1e-6;    // QuadHandler aTol_ (QuadHandler.cpp:61)
constexpr double kQRTol = 1e-7;    // QuadHandler rTol_ (:67)
constexpr double kQBTol = 1e-8;    // QuadHandler bTol_ (:62), isAtBnds_
constexpr double kBilATol = 1e-5;  // LinBil aTol_ (LinBil.cpp:28)
constexpr double kBilRTol = 1e-4;  // LinBil rTol_
constexpr double kIntTol = 1e-6;   // IntVarHandler intTol_

__device__ __forceinline__ bool at_bnds(double v, double l, double u) {
  return fabs(v - l) < kQBTol || fabs(v - u) < kQBTol;
}

__global__ __launch_bounds__(256) void glob_decide(GlobIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= io.nb) return;
  if (io.only != nullptr && io.only[b] == 0) return;
  const int nv = io.nv;
  const double *x = io.x + (size_t)b * nv;
  const double *lb = io.wlb + (size_t)b * nv;
  const double *ub = io.wub + (size_t)b * nv;
  io.depth_in[b] = io.in_depth[b];
  const int st = io.status[b];
  const double val = io.obj[b];
  int dec = 0;
  int bvar = -1, bup = 0, bint = 0;
  double bval = 0.0;
  if (io.kinf[b] != 0) {
    dec = io.kinf[b] == 1 ? 1 : 4;   // presolveNode infeasible / K2 failure
  } else if (st == 2 || st == 3 || st == 8 || st == 10 || st == 11) {
    dec = 1;
  } else if (st == 5) {
    dec = 2;
  } else if (!(st == 0 || st == 1 || st == 6)) {
    dec = 4;
  } else if (val >= io.inc - io.abs_tol || val >= io.inc - fabs(io.inc) * io.rel_tol) {
    dec = 2;
  } else {
    // isFeasible: integrality, then the original quadratic constraints and
    // a quadratic objective (QuadHandler::isFeasible)
    bool feas = true;
    for (int j = 0; j < nv && feas; ++j) {
      const uint8_t t = io.vtype[j];
      if ((t == kBinary || t == kInteger) && fabs(x[j] - floor(x[j] + 0.5)) > kIntTol)
        feas = false;
    }
    for (int c = 0; c < io.nfun && feas; ++c) {
      const int q0 = io.qptr[c], q1 = io.qptr[c + 1];
      if (q0 == q1) continue;          // linear: LinearHandler's
      double act = 0.0;
      for (int t = io.lptr[c]; t < io.lptr[c + 1]; ++t) act += io.lval[t] * x[io.lvar[t]];
      for (int t = q0; t < q1; ++t) act += io.qval[t] * x[io.qv1[t]] * x[io.qv2[t]];
      if (c == io.ncon) {              // the objective
        act += io.obj_const;
        const double vio = fabs(val - act);
        if (vio > fabs(act) * kQRTol && vio > kQATol) feas = false;
        continue;
      }
      const double cub = io.cub[c], clb = io.clb[c];
      if (act > cub + kQATol && (cub == 0.0 || act > cub + fabs(cub) * kQRTol)) feas = false;
      if (act < clb - kQATol && (clb == 0.0 || act < clb - fabs(clb) * kQRTol)) feas = false;
    }
    if (feas) {
      dec = 3;
    } else {
      // candidates per variable: IntVarHandler's, then QuadHandler's
      double *id = io.cand + (size_t)b * nv * 4, *iu = id + nv, *qd = iu + nv, *qu = qd + nv;
      for (int j = 0; j < nv; ++j) id[j] = iu[j] = qd[j] = qu[j] = -1.0;  // -1: none
      for (int j = 0; j < nv; ++j) {
        const uint8_t t = io.vtype[j];
        const double v = x[j];
        if ((t == kBinary || t == kInteger) && fabs(floor(v + 0.5) - v) > kIntTol) {
          id[j] = v - floor(v);
          iu[j] = ceil(v) - v;
        }
      }
      // distances are >= 0; a later candidate of the same variable adds its
      // distances to the earlier ones (new + existing, :507-512)
      auto add_q = [&](int j, double d, double u) {
        if (qd[j] < 0.0) {
          qd[j] = d;
          qu[j] = u;
        } else {
          qd[j] = d + qd[j];
          qu[j] = u + qu[j];
        }
      };
      for (int k = 0; k < io.nsq; ++k) {
        const int j = io.sq[2 * k], y = io.sq[2 * k + 1];
        const double x0 = x[j], yv = x[y];
        if (yv - x0 * x0 > fabs(yv) * kQRTol && yv - x0 * x0 > kQATol) {
          const double dd = (yv - x0 * x0) / sqrt(1.0 + (lb[j] + x0) * (lb[j] + x0));
          const double ud = (yv - x0 * x0) / sqrt(1.0 + (ub[j] + x0) * (ub[j] + x0));
          add_q(j, dd, ud);
        }
      }
      for (int k = 0; k < io.nbil; ++k) {
        const int j0 = io.bil[3 * k], j1 = io.bil[3 * k + 1], y = io.bil[3 * k + 2];
        const double v0 = x[j0], v1 = x[j1], yv = x[y];
        const double pr = v1 * v0;
        if (!(fabs(pr - yv) > kBilATol && fabs(pr - yv) > fabs(yv) * kBilRTol)) continue;
        if (!at_bnds(v0, lb[j0], ub[j0])) {
          double dd, ud;
          if (v0 * v1 > yv) {
            dd = (-yv + v0 * v1) / sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1]);
            ud = (-yv + v0 * v1) / sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1]);
          } else {
            dd = (yv - v0 * v1) / sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1]);
            ud = (yv - v0 * v1) / sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1]);
          }
          add_q(j0, dd, ud);
        }
        if (!at_bnds(v1, lb[j1], ub[j1])) {
          double dd, ud;
          if (v0 * v1 > yv) {
            dd = (-yv + v1 * v0) / sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0]);
            ud = (-yv + v1 * v0) / sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0]);
          } else {
            dd = (yv - v1 * v0) / sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0]);
            ud = (yv - v1 * v0) / sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0]);
          }
          add_q(j1, dd, ud);
        }
      }
      // MaxVioBrancher::findCandidates_ merge + findBestCandidate_
      double best = -INFINITY;
      for (int j = 0; j < nv; ++j) {
        const bool hi = id[j] >= 0.0, hq = qd[j] >= 0.0;
        if (!hi && !hq) continue;
        double d, u;
        int isint;
        if (hi && hq) {
          // the later handler (QuadHandler) takes the candidate when its
          // distance sum is >= IntVarHandler's (MaxVioBrancher.cpp:129-133);
          // the distances stay IntVarHandler's: the merge calls setDist
          // through a BrCandPtr, and BrCand::setDist is an empty non-virtual
          // (BrCand.cpp:44-46; a reference quirk, kept)
          isint = (id[j] + iu[j] <= qd[j] + qu[j]) ? 0 : 1;
          d = id[j];
          u = iu[j];
        } else if (hi) {
          isint = 1;
          d = id[j];
          u = iu[j];
        } else {
          isint = 0;
          d = qd[j];
          u = qu[j];
        }
        const double lo = d < u ? d : u, hv = d < u ? u : d;
        const double sc = 0.1 * (0.8 * lo + 0.2 * hv);
        if (sc > best) {
          best = sc;
          bvar = j;
          bint = isint;
          bup = d > u ? 1 : 0;
        }
      }
      if (bvar < 0) {
        dec = 5;   // no candidate (the reference hands the node to an NLP engine)
      } else {
        dec = 0;
        bval = x[bvar];
      }
    }
  }
  io.dec[b] = dec;
  io.bvar[b] = bvar;
  io.bval[b] = bval;
  io.bup[b] = (int8_t)bup;
  io.bint[b] = (int8_t)bint;
}

// One block: decision counts, the children's exclusive prefix (2 per
// branched node), LP count and pivots, the best feasible node (lowest
// objective, lowest index on ties).  Chunked: thread t owns nodes
// [t*C, (t+1)*C).
__global__ __launch_bounds__(1024) void glob_summary(GlobIO io) {
  __shared__ int s_cnt[1024];
  __shared__ double s_best[1024];
  __shared__ int s_bidx[1024];
  __shared__ long long s_piv[1024];
  __shared__ int s_lps[1024];
  __shared__ int s_dec[1024][6];
  __shared__ int s_bi[1024];
  const int t = threadIdx.x, nb = io.nb;
  const int C = (nb + 1023) / 1024;
  const int b0 = t * C, b1 = b0 + C < nb ? b0 + C : nb;
  int cnt = 0, lps = 0, bi = 0;
  long long piv = 0;
  int dc[6] = {0, 0, 0, 0, 0, 0};
  double best = INFINITY;
  int bidx = -1;
  for (int b = b0; b < b1; ++b) {
    const int d = io.dec[b];
    dc[d] += 1;
    if (d == 0) {
      cnt += 2;
      bi += io.bint[b];
    }
    if (io.kinf[b] == 0) {
      lps += 1;
      piv += io.iters[b];
    }
    if (d == 3 && io.obj[b] < best) {
      best = io.obj[b];
      bidx = b;
    }
  }
  s_cnt[t] = cnt;
  s_best[t] = best;
  s_bidx[t] = bidx;
  s_piv[t] = piv;
  s_lps[t] = lps;
  s_bi[t] = bi;
  for (int k = 0; k < 6; ++k) s_dec[t][k] = dc[k];
  __syncthreads();
  if (t == 0) {
    GlobOut o{};
    int run = 0;
    o.best = INFINITY;
    o.best_idx = -1;
    for (int u = 0; u < 1024; ++u) {
      const int c = s_cnt[u];
      s_cnt[u] = run;
      run += c;
      for (int k = 0; k < 6; ++k) o.ndec[k] += s_dec[u][k];
      o.lps += s_lps[u];
      o.pivots += s_piv[u];
      o.br_int += s_bi[u];
      if (s_bidx[u] >= 0 && s_best[u] < o.best) {
        o.best = s_best[u];
        o.best_idx = s_bidx[u];
      }
    }
    o.nchild = run;
    *io.out = o;
  }
  __syncthreads();
  int run = s_cnt[t];
  for (int b = b0; b < b1; ++b) {
    io.pos[b] = run;
    if (io.dec[b] == 0) run += 2;
  }
}

// One wave per branched node: two children at base + pos[b], the preferred
// one last (the top of the stack is processed first), each the node's
// tightened box with the branching bound, its rewritten rows, its LP value
// as the bound and depth + 1.
__global__ __launch_bounds__(256) void glob_children(GlobIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb || io.dec[b] != 0) return;
  const int nv = io.nv, R = io.R, j = io.bvar[b];
  const double v = io.bval[b];
  const bool isint = io.bint[b] != 0;
  const double dn = isint ? floor(v) : v, up = isint ? ceil(v) : v;
  for (int c = 0; c < 2; ++c) {
    // stack: c = 0 the other branch, c = 1 the preferred one (on top);
    // reference order: c = 0 the down child, c = 1 the up child, at the
    // slots the host assigned
    const bool upc = io.child_slots != nullptr ? c == 1 : (c == 1) == (io.bup[b] != 0);
    const size_t s = io.child_slots != nullptr ? (size_t)io.child_slots[io.pos[b] + c]
                                               : (size_t)io.base + io.pos[b] + c;
    for (int k = lane; k < nv; k += 64) {
      double l = io.wlb[(size_t)b * nv + k], u = io.wub[(size_t)b * nv + k];
      if (k == j) {
        if (upc) l = up;
        else u = dn;
      }
      io.plb[s * nv + k] = l;
      io.pub[s * nv + k] = u;
    }
    for (int k = lane; k < R; k += 64) io.prows[s * R + k] = io.wrows[(size_t)b * R + k];
    // the node's tangent cuts go down to both children
    for (int k = lane; k < io.T; k += 64)
      io.ptan[s * io.T + k] = io.wvals[(size_t)b * (R + io.T) + R + k];
    if (io.pws_head != nullptr) {   // the node's optimal basis for both children
      for (int k = lane; k < io.m; k += 64)
        io.pws_head[s * io.m + k] = io.wo_head[(size_t)b * io.m + k];
      for (int k = lane; k < io.N; k += 64)
        io.pws_st[s * io.N + k] = io.wo_st[(size_t)b * io.N + k];
      if (lane == 0) io.pws_ok[s] = 1;
    }
    if (lane == 0) {
      io.pnlb[s] = io.obj[b];
      io.pdepth[s] = io.depth_in[b] + 1;
    }
  }
}

// reference order: the round's nodes from their pool slots (one wave per node)
__global__ __launch_bounds__(256) void glob_gather(GlobIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  const size_t sl = (size_t)io.sel[b];
  const int nv = io.nv, R = io.R, T = io.T;
  for (int k = lane; k < nv; k += 64) {
    io.glb[(size_t)b * nv + k] = io.plb[sl * nv + k];
    io.gub[(size_t)b * nv + k] = io.pub[sl * nv + k];
  }
  for (int k = lane; k < R; k += 64) io.grows[(size_t)b * R + k] = io.prows[sl * R + k];
  for (int k = lane; k < T; k += 64) io.gtan[(size_t)b * T + k] = io.ptan[sl * T + k];
  if (io.pws_head != nullptr) {
    for (int k = lane; k < io.m; k += 64) io.ghead[(size_t)b * io.m + k] = io.pws_head[sl * io.m + k];
    for (int k = lane; k < io.N; k += 64) io.gst[(size_t)b * io.N + k] = io.pws_st[sl * io.N + k];
    if (lane == 0) io.gok[b] = io.pws_ok[sl];
  }
  if (lane == 0) io.gdepth[b] = io.pdepth[sl];
}

// parent-basis warm starts: the warm call solves the nodes with a basis
// (skip_a), the cold call (slack basis) the others (skip2; flag marks them
// for glob_merge)
__global__ __launch_bounds__(256) void glob_skips(GlobIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= io.nb) return;
  const bool inf = io.kinf[b] != 0, ok = io.gok[b] != 0;
  io.skip_a[b] = inf || !ok ? 1 : 0;
  io.skip2[b] = inf || ok ? 1 : 0;
  io.flag[b] = !inf && !ok ? 1 : 0;
}

// One wave per node: the LP record [R row state | T tangent values] from
// K2's rows and the tangent slots the node inherited.
__global__ __launch_bounds__(256) void glob_pack(GlobIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb) return;
  const int R = io.R, T = io.T;
  double *w = io.wvals + (size_t)b * (R + T);
  for (int k = lane; k < R; k += 64) w[k] = io.wrows[(size_t)b * R + k];
  for (int k = lane; k < T; k += 64) w[R + k] = io.in_tan[(size_t)b * T + k];
}

constexpr double kInf = __builtin_inf();

// QuadHandler::findLinPt_ (QuadHandler.cpp:238-285): golden-section search
// for the point of y = x^2 nearest to (xv, yv), the reference's operations
// in its order (sqrt of a negative y is NaN: the loop does not run and
// addCut_'s tests fail, as there).
__device__ double find_lin_pt(double xv, double yv) {
  const double alfa = 0.618, errlim = 1e-4;
  double a, b;
  if (xv > 0) {
    a = sqrt(yv);
    b = xv;
  } else {
    a = xv;
    b = -sqrt(yv);
  }
  double mu = a + alfa * (b - a);
  double la = b - alfa * (b - a);
  double mu_val = (mu - xv) * (mu - xv) + (mu * mu - yv) * (mu * mu - yv);
  double la_val = (la - xv) * (la - xv) + (la * la - yv) * (la * la - yv);
  while ((b - a) > errlim) {
    if (mu_val < la_val) {
      a = la;
      la = mu;
      la_val = mu_val;
      mu = a + alfa * (b - a);
      mu_val = (mu - xv) * (mu - xv) + (mu * mu - yv) * (mu * mu - yv);
    } else {
      b = mu;
      mu = la;
      mu_val = la_val;
      la = b - alfa * (b - a);
      la_val = (la - xv) * (la - xv) + (la * la - yv) * (la * la - yv);
    }
  }
  return la;
}

// QuadHandler::separate's squares (QuadHandler.cpp:1671-1689) for the nodes
// PCBProcessor would branch (decision 0) or hand to the NLP engine (5): for
// each square whose LP point lies below y = x^2 (x^2 - y > rTol |y| and >
// aTol), the tangent at findLinPt_'s point when addCut_ accepts it
// (2 xl x - y - xl^2 > 1e-5 and 2 xl x - y > xl^2 (1 + 1e-4), :819-840),
// into the square's first free slot.  flag[b]: cuts added (the node is
// re-solved, SepaResolve); skip2 = !flag for that LP call.  One thread per
// node (the search is sequential).
__global__ __launch_bounds__(256) void glob_separate(GlobIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= io.nb) return;
  int cuts = 0;
  const int d = io.dec[b];
  if (d == 0 || d == 5) {
    const double *x = io.x + (size_t)b * io.nv;
    double *tan = io.wvals + (size_t)b * (io.R + io.T) + io.R;
    for (int k = 0; k < io.nsq; ++k) {
      const double xv = x[io.sq[2 * k]], yv = x[io.sq[2 * k + 1]];
      if (!(xv * xv - yv > kQRTol * fabs(yv) && fabs(xv * xv - yv) > kQATol)) continue;
      const double xl = find_lin_pt(xv, yv), yl = xl * xl;
      if (!(2 * xl * xv - yv - yl > 1e-5 && 2 * xl * xv - yv > yl * (1 + 1e-4))) continue;
      for (int t = 0; t < io.S; ++t) {
        double *slot = tan + 2 * (k * io.S + t);
        if (slot[1] == kInf) {
          slot[0] = 2 * xl;
          slot[1] = xl * xl;
          ++cuts;
          break;
        }
      }
    }
  }
  io.flag[b] = cuts > 0 ? 1 : 0;
  io.skip2[b] = cuts > 0 ? 0 : 1;
  if (cuts > 0) {
    atomicAdd(io.acc, (unsigned long long)cuts);
    atomicAdd(io.acc + 1, 1ull);
  }
}

// The re-solved nodes' LP results replace the earlier ones (iterations add
// up); one wave per node.
__global__ __launch_bounds__(256) void glob_merge(GlobIO io) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= io.nb || io.flag[b] == 0) return;
  double *x = io.x + (size_t)b * io.nv;
  for (int k = lane; k < io.nv; k += 64) x[k] = io.x2[(size_t)b * io.nv + k];
  if (lane == 0) {
    io.status[b] = io.st2[b];
    io.obj[b] = io.obj2[b];
    io.iters[b] += io.it2[b];
  }
}

// ---- LinearHandler::presolveNode on the node's relaxation -----------------
// PCBProcessor::presolveNode_ (PCBProcessor.cpp:134-175) runs the handlers'
// presolveNode in order; LinearHandler's (LinearHandler.cpp:1592-1602) is
// simplePresolve in node mode over EVERY row of the relaxation (:1605-1653):
// the linear rows and QuadHandler's secant / McCormick rows as the node
// inherited them, and the tangent cuts.  Weights of |a| <= 1e-9 are absent
// (LinearFunction::addTerm, LinearFunction.cpp:89-95): they neither count in
// the sums nor put their row in the variable's constraint set
// (Problem::changeConstraint keeps that set, Problem.cpp:273-303, which
// changeBFlag_ walks, LinearHandler.cpp:1229-1234).  One thread per node,
// the reference's operations in its order (-ffp-contract=off).
constexpr double kLfTol = 1e-9, kLinETol = 1e-8, kLinInfty = 1e20, kLinIntTol = 1e-6;

struct LinNode {
  const GlobIO *io;
  double *lb, *ub;
  uint8_t *flag;
  const double *rows, *tan;
  unsigned nintmods;
  __device__ double rec(int src) const { return src < io->R ? rows[src] : tan[src - io->R]; }
  __device__ double w(int t) const {
    const int s = io->ltsrc[t];
    return s < 0 ? io->ltval[t] : rec(s);
  }
  __device__ bool is_int(int j) const { return io->vtype[j] <= 1; }
  // changeBFlag_
  __device__ void change_bflag(int j) {
    for (int p = io->lcptr[j]; p < io->lcptr[j + 1]; ++p) {
      const int t = io->lcterm[p];
      if (fabs(w(t)) > kLfTol) flag[io->ltrow[t]] = 1;
    }
  }
};

// getLfBnds_ (LinearHandler.cpp:1237-1258) over terms [t0, t1) (obj: loidx)
template <bool OBJ>
__device__ void lin_lf_bnds(const LinNode &s, int t0, int t1, double *lo, double *up) {
  double l = 0, u = 0;
  for (int t = t0; t < t1; ++t) {
    const double c = OBJ ? s.io->loval[t] : s.w(t);
    if (!OBJ && fabs(c) <= kLfTol) continue;
    const int j = OBJ ? s.io->loidx[t] : s.io->ltvar[t];
    const double vl = s.lb[j], vu = s.ub[j];
    if (c > 0) {
      l += c * vl;
      u += c * vu;
    } else {
      l += c * vu;
      u += c * vl;
    }
  }
  *lo = l;
  *up = u;
}

// getSingLfBnds_ (LinearHandler.cpp:1261-1319)
template <bool OBJ>
__device__ void lin_sing_bnds(const LinNode &s, int t0, int t1, double *lo, double *up) {
  double l = 0, u = 0;
  bool lo_sing = false, up_sing = false, lo_fin = true, up_fin = true;
  for (int t = t0; t < t1; ++t) {
    const double c = OBJ ? s.io->loval[t] : s.w(t);
    if (!OBJ && fabs(c) <= kLfTol) continue;
    const int j = OBJ ? s.io->loidx[t] : s.io->ltvar[t];
    const double vl = s.lb[j], vu = s.ub[j];
    if (c > kLinETol) {
      if (vu < kLinInfty && up_fin) u += c * vu;
      else if (up_sing) { up_sing = false; u = kInf; up_fin = false; }
      else up_sing = true;
      if (vl > -kLinInfty && lo_fin) l += c * vl;
      else if (lo_sing) { lo_sing = false; l = -kInf; lo_fin = false; }
      else lo_sing = true;
    } else if (c < -kLinETol) {
      if (vu < kLinInfty && lo_fin) l += c * vu;
      else if (lo_sing) { lo_sing = false; l = -kInf; lo_fin = false; }
      else lo_sing = true;
      if (vl > -kLinInfty && up_fin) u += c * vl;
      else if (up_sing) { up_sing = false; u = kInf; up_fin = false; }
      else up_sing = true;
    }
  }
  *lo = l;
  *up = u;
}

// updateLfBoundsFromLb_ (FROM_LB, LinearHandler.cpp:1048-1134) and
// updateLfBoundsFromUb_ (:1137-1226); side = the row's lb (ub), act = uu (ll)
template <bool OBJ, bool FROM_LB>
__device__ void lin_update(LinNode &s, int t0, int t1, double side, double act, bool sing,
                           bool *changed, bool count_int) {
  for (int t = t0; t < t1; ++t) {
    const double c = OBJ ? s.io->loval[t] : s.w(t);
    const int j = OBJ ? s.io->loidx[t] : s.io->ltvar[t];
    double vlb = s.lb[j], vub = s.ub[j];
    // FROM_LB: c > 0 raises the lower bound, c < 0 lowers the upper one;
    // from the upper side the other way round
    const bool raise = FROM_LB ? c > kLinETol : c < -kLinETol;
    const bool lower = FROM_LB ? c < -kLinETol : c > kLinETol;
    if (raise && (!sing || vub >= kLinInfty)) {
      if (vub >= kLinInfty) vub = 0.;
      double nlb = (side - act) / c + vub;
      if (nlb > vlb + kLinETol) {
        if (nlb > s.ub[j] - kLinETol) nlb = s.ub[j];
        s.change_bflag(j);
        s.lb[j] = nlb;
        if (count_int && s.is_int(j)) s.nintmods++;
        *changed = true;
      }
    } else if (lower && (!sing || vlb <= -kLinInfty)) {
      if (vlb <= -kLinInfty) vlb = 0.;
      double nub = (side - act) / c + vlb;
      if (nub < vub - kLinETol) {
        if (nub < s.lb[j] + kLinETol) nub = s.lb[j];
        s.change_bflag(j);
        s.ub[j] = nub;
        if (count_int && s.is_int(j)) s.nintmods++;
        *changed = true;
      }
    }
  }
}

// linBndTighten_ (LinearHandler.cpp:952-1045, node mode); true: infeasible
__device__ bool lin_row(LinNode &s, int i, bool *changed) {
  const GlobIO &io = *s.io;
  const int t0 = io.lrptr[i], t1 = io.lrptr[i + 1];
  const double lb = io.lrlo[i];
  const double ub = io.lrhsrc[i] < 0 ? io.lrhi[i] : s.rec(io.lrhsrc[i]);
  double ll, uu, sll = -kInf, suu = kInf;
  *changed = false;
  lin_lf_bnds<false>(s, t0, t1, &ll, &uu);
  if (ll < -kLinInfty || uu > kLinInfty) lin_sing_bnds<false>(s, t0, t1, &sll, &suu);
  if (ll > ub + kLinETol) return true;
  if (uu < lb - kLinETol) return true;
  if (lb > -kLinInfty) {
    if (uu < kLinInfty) lin_update<false, true>(s, t0, t1, lb, uu, false, changed, true);
    else if (suu < kLinInfty) lin_update<false, true>(s, t0, t1, lb, suu, true, changed, true);
  }
  if (*changed) {
    lin_lf_bnds<false>(s, t0, t1, &ll, &uu);
    if (ll < -kLinInfty || uu > kLinInfty) lin_sing_bnds<false>(s, t0, t1, &sll, &suu);
  }
  if (ub < kLinInfty) {
    if (ll > -kLinInfty) lin_update<false, false>(s, t0, t1, ub, ll, false, changed, true);
    else if (sll > -kLinInfty) lin_update<false, false>(s, t0, t1, ub, sll, true, changed, true);
  }
  return false;
}

__global__ __launch_bounds__(64) void glob_linear(GlobIO io) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= io.nb) return;
  const int nv = io.nv, M = io.M;
  LinNode s;
  s.io = &io;
  s.lb = io.flb + (size_t)b * nv;
  s.ub = io.fub + (size_t)b * nv;
  s.flag = io.fflag + (size_t)b * M;
  s.rows = io.frows + (size_t)b * io.R;
  s.tan = io.T > 0 ? io.ftan + (size_t)b * io.T : nullptr;
  s.nintmods = 0;
  for (int j = 0; j < nv; ++j) {
    s.lb[j] = io.flb_in[(size_t)b * nv + j];
    s.ub[j] = io.fub_in[(size_t)b * nv + j];
  }
  for (int i = 0; i < M; ++i) s.flag[i] = 1;
  // simplePresolve: sweeps while changed, at most 10, past the second only
  // while an integer bound moved; varBndsFromCons_ / varBndsFromObj_'s
  // verdicts are dropped there (:1630-1640), checkBounds_ decides
  bool changed = true, infeas = false;
  unsigned iters = 1;
  while (changed && iters <= 10 && (iters <= 2 || s.nintmods > 0) && !infeas) {
    s.nintmods = 0;
    changed = false;
    ++iters;
    // varBndsFromCons_ (:493-541): each flagged row once per sweep
    for (int i = 0; i < M; ++i) {
      if (!s.flag[i]) continue;
      s.flag[i] = 0;
      bool tch;
      if (lin_row(s, i, &tch)) break;
      if (tch) changed = true;
    }
    // varBndsFromObj_ (:544-597) with a solution in the pool
    if (io.has_inc && io.nobj > 0) {
      bool tch = true;
      for (long guard = 0; tch && guard <= 100000; ++guard) {
        double ll, uu, sll = kInf, suu = kInf;
        tch = false;
        lin_lf_bnds<true>(s, 0, io.nobj, &ll, &uu);
        if (ll < -kLinInfty || uu > kLinInfty) lin_sing_bnds<true>(s, 0, io.nobj, &sll, &suu);
        if (ll > io.inc_ub + kLinETol) break;
        if (ll > -kLinInfty)
          lin_update<true, false>(s, 0, io.nobj, io.inc_ub, ll, false, &tch, false);
        else if (sll > -kLinInfty)
          lin_update<true, false>(s, 0, io.nobj, io.inc_ub, sll, true, &tch, false);
        if (tch) changed = true;
      }
    }
    // tightenInts_ (:415-490)
    for (int j = 0; j < nv; ++j) {
      if (!s.is_int(j)) continue;
      const double l = s.lb[j], u = s.ub[j];
      if (l > -kLinInfty && fabs(l - floor(l + 0.5)) > kLinIntTol) {
        s.change_bflag(j);
        s.lb[j] = ceil(l);
        changed = true;
      }
      if (u < kLinInfty && fabs(u - floor(u + 0.5)) > kLinIntTol) {
        s.ub[j] = floor(u);
        s.change_bflag(j);
        changed = true;
      }
    }
    // checkBounds_ (:328-359)
    infeas = io.cons_bad != 0;
    for (int j = 0; j < nv && !infeas; ++j) infeas = s.lb[j] > s.ub[j] + kLinETol;
  }
  io.finf[b] = infeas ? 1 : 0;
}

// a node the linear presolve found infeasible is pruned before the LP
// (PCBProcessor::process, :208-213): K2's verdict for it becomes infeasible
__global__ __launch_bounds__(256) void glob_linear_verdict(GlobIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < io.nb && io.finf[b] != 0) const_cast<int32_t *>(io.kinf)[b] = 1;
}

}  // namespace

hipError_t launch_glob_decide(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_decide, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_pack(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_pack, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_separate(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_separate, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_merge(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_merge, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_gather(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_gather, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_skips(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_skips, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_children(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_children, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_summary(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_summary, dim3(1), dim3(1024), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_linear(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_linear, dim3((io.nb + 63) / 64), dim3(64), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_linear_verdict(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_linear_verdict, dim3((io.nb + 255) / 256), dim3(256), 0, stream, io);
  return hipGetLastError();
}

hipError_t launch_glob_round_tail(const GlobIO &io, hipStream_t stream) {
  if (io.nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(glob_summary, dim3(1), dim3(1024), 0, stream, io);
  hipLaunchKernelGGL(glob_children, dim3((io.nb + 3) / 4), dim3(256), 0, stream, io);
  return hipGetLastError();
}

}  // namespace mgpu
