"""TEST INFRASTRUCTURE ONLY (imported by tests/ and bench.py's cpu_baseline
leg, never by the product path): a CPU restatement of one round of the
batched spatial branch-and-bound (mgpu_glob_round,
minotaur_amd/csrc/glob_runtime.cpp + glob_tree.hip), built from the C
restatements of K2 (oracle.quad_fbbt, bit-identical to the reference's
QuadHandler::presolveNode) and of the per-node-rows LP (oracle.
dual_simplex_rows, K3R + K3's pivots), plus the decision below in the same
arithmetic order as the GPU kernel (sequential sums, no fused multiply-add),
so the two trees agree round for round.

Reference semantics restated (file:line under /root/reference/src/base):
* PCBProcessor::shouldPrune_ (PCBProcessor.cpp:400-523): engine-status
  switch, bound test with solAbs_tol / solRel_tol 1e-6;
* IntVarHandler::isFeasible (IntVarHandler.cpp:54-84), QuadHandler::
  isFeasible (QuadHandler.cpp:904-953; aTol_ 1e-6, rTol_ 1e-7);
* candidates: IntVarHandler::getBranchingCandidates (IntVarHandler.cpp:
  86-110), QuadHandler::getBranchingCandidates (QuadHandler.cpp:473-614;
  LinBil::isViolated, LinBil.cpp:64-82, aTol 1e-5, rTol 1e-4; isAtBnds_
  bTol_ 1e-8, :897-902);
* MaxVioBrancher::findCandidates_ / findBestCandidate_ (MaxVioBrancher.cpp:
  merge per variable -- the later handler takes the candidate when its
  distance sum is >= the earlier one's, but the distances stay the earlier
  handler's: the merge calls setDist through a BrCandPtr, and
  BrCand::setDist is an empty non-virtual (BrCand.cpp:44-46) -- score
  0.1 (0.8 min + 0.2 max), first maximum, up first when dd > ud);
* children: IntVarHandler::getBranches at floor / ceil, QuadHandler::
  getBranches at the value (QuadHandler.cpp:422-471);
* separation of the squares (QuadHandler::separate, QuadHandler.cpp:
  1658-1689; findLinPt_ :238-285, addCut_ / addTangent_ :805-840): a node
  that would branch (or has no candidate) and whose LP point lies below
  y = x^2 (x^2 - y > rTol |y| and > aTol) gets the tangent at the nearest
  point of the parabola when it cuts the point off by the margins of addCut_;
  the node is then re-solved (PCBProcessor.cpp:267-280, SepaResolve) and
  decided again, until no cut is added.  The cuts go into the node's
  tangent slots (``tan_slots`` per square, quad.relaxation_lp) and are
  inherited by its children; the reference adds them to the one global
  relaxation.
Parity with the reference's own glob solver is unpinned (it needs Ipopt /
filterSQP and its cut loop); the GPU tree is pinned against this
restatement and its incumbents against the QCQP itself.
"""
from __future__ import annotations

import math

import numpy as np

import oracle
from oracle import WarmStart

BINARY, INTEGER = 0, 1


class _GStats:
    def __init__(self):
        self.rounds = self.nodes = 0
        self.ndec = [0] * 6
        self.lps = self.pivots = 0
        self.br_int = self.br_cont = 0
        self.cuts = self.resolves = 0
        self.obbt_lps = 0
        self.sb_lps = 0
        self.open = self.last_batch = 0
        self.incumbent = math.inf


def _at_bnds(v, l, u):
    return abs(v - l) < 1e-8 or abs(v - u) < 1e-8


def decide(qp, kinf, st, val, x, lb, ub, inc):
    """One node: (decision, bvar, bval, bup, bint) as glob_decide."""
    nv = qp.nv
    if kinf != 0:
        return (1 if kinf == 1 else 4), -1, 0.0, 0, 0
    if st in (2, 3, 8, 10, 11):
        return 1, -1, 0.0, 0, 0
    if st == 5:
        return 2, -1, 0.0, 0, 0
    if st not in (0, 1, 6):
        return 4, -1, 0.0, 0, 0
    if val >= inc - 1e-6 or val >= inc - abs(inc) * 1e-6:
        return 2, -1, 0.0, 0, 0
    vt = qp.vtype
    feas = True
    for j in range(nv):
        if vt[j] in (BINARY, INTEGER) and abs(x[j] - math.floor(x[j] + 0.5)) > 1e-6:
            feas = False
            break
    nfun = qp.ncon + (1 if qp.has_obj else 0)
    c = 0
    while feas and c < nfun:
        q0, q1 = int(qp.qptr[c]), int(qp.qptr[c + 1])
        if q0 != q1:
            act = 0.0
            for t in range(int(qp.lptr[c]), int(qp.lptr[c + 1])):
                act += float(qp.lval[t]) * x[qp.lvar[t]]
            for t in range(q0, q1):
                act += float(qp.qval[t]) * x[qp.qv1[t]] * x[qp.qv2[t]]
            if c == qp.ncon:
                act += float(qp.obj_const)
                vio = abs(val - act)
                if vio > abs(act) * 1e-7 and vio > 1e-6:
                    feas = False
            else:
                cub, clb = float(qp.cub[c]), float(qp.clb[c])
                if act > cub + 1e-6 and (cub == 0.0 or act > cub + abs(cub) * 1e-7):
                    feas = False
                if act < clb - 1e-6 and (clb == 0.0 or act < clb - abs(clb) * 1e-7):
                    feas = False
        c += 1
    if feas:
        return 3, -1, 0.0, 0, 0
    # MaxVio over the merged candidates: score 0.1 (0.8 min + 0.2 max), the
    # first maximum, up first when dd > ud
    best, bvar, bup, bint = -math.inf, -1, 0, 0
    for j, isint, d, u in candidates(qp, x, lb, ub):
        lo, hv = (d, u) if d < u else (u, d)
        sc = 0.1 * (0.8 * lo + 0.2 * hv)
        if sc > best:
            best, bvar, bint, bup = sc, j, isint, (1 if d > u else 0)
    if bvar < 0:
        return 5, -1, 0.0, 0, 0
    return 0, bvar, float(x[bvar]), bup, bint


QA_TOL, QR_TOL = 1e-6, 1e-7   # QuadHandler aTol_, rTol_ (QuadHandler.cpp:60-67)


def candidates(qp, x, lb, ub):
    """The branching candidates of IntVarHandler and QuadHandler merged per
    variable as MaxVioBrancher / StrongBrancher::findCandidates_ merge them
    (the later handler takes a candidate when its distance sum is >=, the
    distances stay the earlier handler's: BrCand::setDist is an empty
    non-virtual): [(var, isint, ddist, udist)] ascending by variable (the
    candidate sets' order, CompareVarBrCand, Types.cpp:23-27)."""
    nv, vt = qp.nv, qp.vtype
    idd, iud, qd, qu = {}, {}, {}, {}
    for j in range(nv):
        v = x[j]
        if vt[j] in (BINARY, INTEGER) and abs(math.floor(v + 0.5) - v) > 1e-6:
            idd[j] = v - math.floor(v)
            iud[j] = math.ceil(v) - v

    def add_q(j, d, u):
        if j not in qd:
            qd[j], qu[j] = d, u
        else:
            qd[j], qu[j] = d + qd[j], u + qu[j]

    for k in range(qp.nsq):
        j, y = int(qp.sq_x[k]), int(qp.sq_y[k])
        x0, yv = x[j], x[y]
        if yv - x0 * x0 > abs(yv) * 1e-7 and yv - x0 * x0 > 1e-6:
            dd = (yv - x0 * x0) / math.sqrt(1.0 + (lb[j] + x0) * (lb[j] + x0))
            ud = (yv - x0 * x0) / math.sqrt(1.0 + (ub[j] + x0) * (ub[j] + x0))
            add_q(j, dd, ud)
    for k in range(qp.nbil):
        j0, j1, y = int(qp.bil_x0[k]), int(qp.bil_x1[k]), int(qp.bil_y[k])
        v0, v1, yv = x[j0], x[j1], x[y]
        pr = v1 * v0
        if not (abs(pr - yv) > 1e-5 and abs(pr - yv) > abs(yv) * 1e-4):
            continue
        if not _at_bnds(v0, lb[j0], ub[j0]):
            if v0 * v1 > yv:
                dd = (-yv + v0 * v1) / math.sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1])
                ud = (-yv + v0 * v1) / math.sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1])
            else:
                dd = (yv - v0 * v1) / math.sqrt(1.0 + v0 * v0 + lb[j1] * lb[j1])
                ud = (yv - v0 * v1) / math.sqrt(1.0 + v0 * v0 + ub[j1] * ub[j1])
            add_q(j0, dd, ud)
        if not _at_bnds(v1, lb[j1], ub[j1]):
            if v0 * v1 > yv:
                dd = (-yv + v1 * v0) / math.sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0])
                ud = (-yv + v1 * v0) / math.sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0])
            else:
                dd = (yv - v1 * v0) / math.sqrt(1.0 + v1 * v1 + lb[j0] * lb[j0])
                ud = (yv - v1 * v0) / math.sqrt(1.0 + v1 * v1 + ub[j0] * ub[j0])
            add_q(j1, dd, ud)
    out = []
    for j in range(nv):
        hi, hq = j in idd, j in qd
        if hi and hq:
            out.append((j, 0 if idd[j] + iud[j] <= qd[j] + qu[j] else 1, idd[j], iud[j]))
        elif hi:
            out.append((j, 1, idd[j], iud[j]))
        elif hq:
            out.append((j, 0, qd[j], qu[j]))
    return out


def _keep(a):
    return a if abs(a) > 1e-9 else 0.0   # LinearFunction::addTerm (LinearFunction.cpp:89-95)


def br_mod(qp, rec, lb, ub, x, j, isint, down):
    """Handler::getBrMod of candidate j on copies of the node's box and row
    record: IntVarHandler (IntVarHandler.cpp:113-130) floor / ceil of x_j;
    QuadHandler (QuadHandler.cpp:616-692) x_j itself, plus the rows of the
    violated terms of x_j rebuilt for the branch's box: the secant of its
    square (getNewSqLf_ over [lb, x_j] or [x_j, ub]) and, per violated
    bilinear holding x_j, rows 1 and 3 (down) or 0 and 2 (up) from
    getNewBilLf_ with x_j's bound at its value -- with x_j the bilinear's
    second factor the arguments come swapped, so row 3 / 2 then carries the
    other upper-envelope formula, as in the reference."""
    lb, ub, rec = lb.copy(), ub.copy(), np.array(rec, dtype=np.float64)
    v = float(x[j])
    if isint:
        if down:
            ub[j] = math.floor(v)
        else:
            lb[j] = math.ceil(v)
        return lb, ub, rec
    nsq = qp.nsq
    for k in range(nsq):
        if int(qp.sq_x[k]) != j:
            continue
        y = int(qp.sq_y[k])
        vio = v * v - x[y]
        if vio > QA_TOL and vio > abs(x[y]) * QR_TOL:
            lo_, hi_ = (lb[j], v) if down else (v, ub[j])
            rec[2 * k + 1] = -hi_ * lo_
            rec[2 * k] = _keep(-1. * (hi_ + lo_)) if abs(hi_ + lo_) > 1e-5 else 0.0
    for k in range(qp.nbil):
        X0, X1 = int(qp.bil_x0[k]), int(qp.bil_x1[k])
        if j != X0 and j != X1:
            continue
        y = int(qp.bil_y[k])
        xv = x[X0] * x[X1]
        vio = abs(xv - x[y])
        if not (vio > 1e-5 and vio > abs(x[y]) * 1e-4):
            continue
        a, b = (X0, X1) if j == X0 else (X1, X0)    # getNewBilLf_'s x0, x1
        xa = x[a]
        if down:
            lb0, ub0 = lb[a], xa
        else:
            lb0, ub0 = xa, ub[a]
        lb1, ub1 = lb[b], ub[b]

        def row(t):
            # getNewBilLf_ (QuadHandler.cpp:730-763): coefficients of a, b, rhs
            if t == 0:
                return lb1, lb0, lb0 * lb1
            if t == 1:
                return ub1, ub0, ub0 * ub1
            if t == 2:
                return -1.0 * ub1, -1.0 * lb0, -lb0 * ub1
            return -1.0 * lb1, -1.0 * ub0, -ub0 * lb1
        o0 = 2 * nsq + 12 * k
        for t in ((1, 3) if down else (0, 2)):
            ca, cb, rhs = row(t)
            cx0, cx1 = (ca, cb) if a == X0 else (cb, ca)
            o = o0 + 3 * t
            rec[o], rec[o + 1], rec[o + 2] = _keep(cx0), _keep(cx1), rhs
    lb[j] = v if not down else lb[j]
    ub[j] = v if down else ub[j]
    return lb, ub, rec


SB_CANDS, SB_ITER, SB_THRESH, SB_ETOL = 20, 50, 5, 1e-6   # reliabilitySetup(20, 50, 5), Glob.cpp:171-181


def _sb_prune(chcutoff, change, st):
    """StrongBrancher::shouldPrune_ (StrongBrancher.cpp:461-497): (prune, reliable)."""
    if st in (3, 2, 5):
        return True, True
    if st in (1, 0):
        return change > chcutoff - SB_ETOL, True
    if st == 6:
        return False, True
    return False, False


def _score(up, down):
    """getScore_ (StrongBrancher.cpp:381-389)."""
    return down * 0.8 + up * 0.2 if up > down else up * 0.8 + down * 0.2


def find_lin_pt(xval, yval):
    """QuadHandler::findLinPt_ (QuadHandler.cpp:238-285): the point of y = x^2
    nearest to (xval, yval) by golden-section search, in the reference's
    operation order (sqrt of a negative y is NaN there: no cut follows)."""
    alfa, errlim = 0.618, 1e-4
    sy = math.sqrt(yval) if yval >= 0.0 else math.nan
    if xval > 0:
        a, b = sy, xval
    else:
        a, b = xval, -sy
    mu = a + alfa * (b - a)
    la = b - alfa * (b - a)
    mu_val = (mu - xval) * (mu - xval) + (mu * mu - yval) * (mu * mu - yval)
    la_val = (la - xval) * (la - xval) + (la * la - yval) * (la * la - yval)
    while (b - a) > errlim:
        if mu_val < la_val:
            a = la
            la = mu
            la_val = mu_val
            mu = a + alfa * (b - a)
            mu_val = (mu - xval) * (mu - xval) + (mu * mu - yval) * (mu * mu - yval)
        else:
            b = mu
            mu = la
            mu_val = la_val
            la = b - alfa * (b - a)
            la_val = (la - xval) * (la - xval) + (la * la - yval) * (la * la - yval)
    return la, la * la


def separate(qp, x, tan, R, S):
    """The squares part of QuadHandler::separate on one node: fills the first
    free tangent slot of each square whose cut addCut_ accepts (record
    ``tan`` = the node's full row record, tangent part at R); returns the
    number of cuts added."""
    cuts = 0
    for k in range(qp.nsq):
        j, y = int(qp.sq_x[k]), int(qp.sq_y[k])
        xval, yval = float(x[j]), float(x[y])
        if xval * xval - yval > QR_TOL * abs(yval) and abs(xval * xval - yval) > QA_TOL:
            xl, yl = find_lin_pt(xval, yval)
            if 2 * xl * xval - yval - yl > 1e-5 and 2 * xl * xval - yval > yl * (1 + 1e-4):
                for t in range(S):
                    o = R + 2 * (k * S + t)
                    if tan[o + 1] == math.inf:
                        tan[o] = 2 * xl
                        tan[o + 1] = xl * xl
                        cuts += 1
                        break
    return cuts


class _Heap:
    """TreeManager's bfs NodeHeap order (NodeHeap.cpp:24-47, as
    glob_runtime.cpp's gheap_greater): the smallest bound within 1e-6 on top,
    then the shallower node, then the larger id."""

    def __init__(self):
        self.items = []

    @staticmethod
    def _key(n):
        return n

    def push(self, node):
        self.items.append(node)

    def pop(self):
        def better(a, b):   # a comes out before b
            if a['lb'] > b['lb'] + 1e-6:
                return False
            if a['lb'] < b['lb'] - 1e-6:
                return True
            if a['depth'] != b['depth']:
                return a['depth'] < b['depth']
            return a['id'] > b['id']
        best = 0
        for i in range(1, len(self.items)):
            if better(self.items[i], self.items[best]):
                best = i
        return self.items.pop(best)

    def __len__(self):
        return len(self.items)


class CpuGlobContext:
    """mgpu_glob_config / _init / _round / _best on the CPU."""

    def __init__(self, qp, tan_slots=0):
        from minotaur_amd.quad import relaxation_lp, tangent_record
        self.qp = qp
        self.S = tan_slots if qp.nsq > 0 else 0
        self.R = qp.nrow_state
        self.rows0 = oracle.quad_root_rows(qp)
        self.p, self.nr = relaxation_lp(qp, self.rows0, self.S)
        self.tan0 = tangent_record(qp, self.S)
        self.order, self.warm, self.qt, self.lin, self.obbt = 0, 0, 1, 0, 0
        self.brancher = 0

    def glob_config(self, order=0, warm=0, qt=1, lin=0, obbt=0):
        self.order, self.warm, self.qt, self.lin, self.obbt = order, warm, qt, lin, obbt

    def glob_brancher(self, kind=0):
        """0 MaxVioBrancher, 1 Glob's relstronger (StrongBrancher with
        reliabilitySetup(20, 50, 5), Glob.cpp:171-181; batch 1, order 2,
        warm 1, lin 1)."""
        self.brancher = kind

    def _lp1(self, lb, ub, rec, ws, iter_limit=10000):
        """One node LP from the engine's basis ws = (head, st) or the slack
        basis: (status, value, pivots, x, basis out)."""
        W = None if ws is None else WarmStart(ws[0][None], ws[1][None], None, None)
        st, obj, it, x, ho, so = oracle.dual_simplex_rows(self.p, lb[None], ub[None], self.nr,
                                                          np.asarray(rec)[None], ws=W,
                                                          iter_limit=iter_limit, want_x=True,
                                                          want_ws=True)
        return int(st[0]), float(obj[0]), int(it[0]), x[0].copy(), (ho[0].copy(), so[0].copy())

    def _presolve(self, lb, ub, rec, first=False):
        """PCBProcessor::presolveNode_ / Handler::getStrongerMods: the
        handlers' presolveNode in order (LinearHandler's when lin, then
        QuadHandler's K2).  Returns (infeasible, lb, ub, rec)."""
        lb, ub = lb.copy()[None], ub.copy()[None]
        if self.lin and self._linear(lb, ub, [rec])[0]:
            return True, lb[0], ub[0], rec
        qt = 1 if (self.qt or first) else 0
        o = oracle.quad_fbbt(self.qp, lb, ub, self.inc, qt, np.asarray(rec)[None, :self.R])
        if int(o.infeas[0]) != 0:
            if int(o.infeas[0]) != 1:
                raise RuntimeError('glob round: engine problem in K2')
            return True, o.lb[0], o.ub[0], rec
        rec = np.array(rec, dtype=np.float64)
        rec[:self.R] = o.rows[0]
        return False, o.lb[0].copy(), o.ub[0].copy(), rec

    def _after_solve(self, info, obj, x):
        """StrongBrancher::updateAfterSolve (StrongBrancher.cpp:589-643): the
        pseudocost of the branching that made this node."""
        if info is None:
            return
        j = info['var']
        if info['int']:
            oldval, newval = info['act'], x[j]
            c = (obj - info['plb']) / (abs(newval - oldval) + SB_ETOL)
            down = newval < oldval
        else:
            down = info['act'] < 0
            c = (obj - info['plb']) / ((info['dd'] if down else info['ud']) + SB_ETOL)
        if c < 0.0 or math.isinf(c) or math.isnan(c):
            c = 0.0
        self._upd_pc(j, c, down)

    def _upd_pc(self, j, c, down):
        """updatePCost_ (:645-650)."""
        if down:
            self.pd[j] = (self.pd[j] * self.td[j] + c) / (self.td[j] + 1)
            self.td[j] += 1
        else:
            self.pu[j] = (self.pu[j] * self.tu[j] + c) / (self.tu[j] + 1)
            self.tu[j] += 1

    def _strong(self, lb, ub, rec, x, objval, eng):
        """StrongBrancher::findBranches (StrongBrancher.cpp:184-264) on one
        node.  Returns (kind, payload, engine basis): ('branch', (var, isint,
        dd, ud, up_first)), ('prune', None), ('mod', (lb, ub, rec)) or
        ('nocand', None)."""
        qp = self.qp
        cands = candidates(qp, x, lb, ub)
        if not cands:
            return 'nocand', None, eng
        rel = [c for c in cands if self.tu[c[0]] >= SB_THRESH and self.td[c[0]] >= SB_THRESH]
        unrel = [c for c in cands if not (self.tu[c[0]] >= SB_THRESH and self.td[c[0]] >= SB_THRESH)]
        maxchange = self.inc - objval
        best, bc = -math.inf, None
        dirs = {}      # setDir per candidate (BrVarCand's default: UpBranch, BrVarCand.cpp:31)

        def pcscore(c):
            j = c[0]
            chd, chu = c[2] * self.pd[j], c[3] * self.pu[j]
            return chd, chu, _score(chu, chd)

        for c in rel:                      # findBestCandidate_ :93-108
            chd, chu, sc = pcscore(c)
            if sc > best:
                best, bc = sc, c
                dirs[c[0]] = not (chu > chd)
        # sortUnrelCands_ (:429-459): vio = score / (max(times) + 1); the
        # smallest of the top maxCands_
        vio = [_score(c[3], c[2]) / (max(self.td[c[0]], self.tu[c[0]]) + 1) for c in unrel]
        minscore = sorted(vio, reverse=True)[:SB_CANDS][-1] if unrel else 0.0
        status, mod = 'none', None
        cnt = i = 0
        for c in unrel:                    # :115-145
            if cnt >= SB_CANDS:
                break
            if vio[i] >= minscore:
                cnt += 1
                res = []
                for down in (True, False):   # strongBranch_ :499-587: down, then up
                    blb, bub, brec = br_mod(qp, rec, lb, ub, x, c[0], c[1], down)
                    inf, blb, bub, brec = self._presolve(blb, bub, brec)
                    if inf:
                        res.append((2, self._last_val))
                        continue
                    st, ob, it, _, wo = self._lp1(blb, bub, brec, eng, SB_ITER)
                    self.tot.lps += 1
                    self.tot.sb_lps += 1
                    self.lplog.append((st, ob, it))
                    self._last_val = ob
                    if st in (0, 6):
                        eng = wo
                    res.append((st, ob))
                (sd, od), (su, ou) = res
                chu, chd = max(ou - objval, 0.0), max(od - objval, 0.0)
                # useStrongBranchInfo_ (:652-689)
                pdn, rd = _sb_prune(maxchange, chd, sd)
                pup, ru = _sb_prune(maxchange, chu, su)
                if not (rd and ru):
                    chu = chd = 0.0
                elif pup and pdn:
                    status = 'prune'
                elif pup:
                    status, mod = 'mod', br_mod(qp, rec, lb, ub, x, c[0], c[1], True)
                elif pdn:
                    status, mod = 'mod', br_mod(qp, rec, lb, ub, x, c[0], c[1], False)
                else:
                    j = c[0]
                    self._upd_pc(j, abs(chd) / (abs(c[2]) + SB_ETOL), True)
                    self._upd_pc(j, abs(chu) / (abs(c[3]) + SB_ETOL), False)
                sc = _score(chu, chd)
                if status != 'none':
                    break
                if sc > best:
                    best, bc = sc, c
                    dirs[c[0]] = not (chu > chd)
            i += 1
        if status == 'prune':
            return 'prune', None, eng
        if status == 'mod':
            return 'mod', mod, eng
        for jx, c in enumerate(unrel):     # :149-169
            if vio[jx] < minscore or jx >= i:
                chd, chu, sc = pcscore(c)
                if sc > best:
                    best, bc = sc, c
                    dirs[c[0]] = not (chu > chd)
        if best == 0 and not rel:          # :170-180
            bc = unrel[int(np.argmax(vio))]
        if bc is None:
            return 'nocand', None, eng
        return 'branch', (bc[0], bc[1], bc[2], bc[3], dirs.get(bc[0], True)), eng

    def _process_rs(self, nd, nid):
        """PCBProcessor::process (PCBProcessor.cpp:178-353) on one node with
        the StrongBrancher: presolve, then solve / prune / updateAfterSolve /
        feasible / root OBBT / separate / findBranches, re-solving after a
        separation cut, OBBT or a brancher modification.  Returns (decision,
        children as node tuples)."""
        qp = self.qp
        lb, ub, rec = nd[0].copy(), nd[1].copy(), np.array(nd[2], dtype=np.float64)
        info = nd[7] if len(nd) > 7 else None
        first = self.tot.nodes == 0
        inf, lb, ub, rec = self._presolve(lb, ub, rec, first)
        if inf:
            return 1, []
        eng = None if nd[5] is None else (nd[5], nd[6])
        it_ = 0
        root = nid == 0
        while True:
            it_ += 1
            st, obj, piv, x, wo = self._lp1(lb, ub, rec, eng)
            self.tot.lps += 1
            self.tot.pivots += piv
            self.lplog.append((st, obj, piv))
            self._last_val = obj
            if st in (0, 6):
                eng = wo
            d = decide(qp, 0, st, obj, x, lb, ub, self.inc)[0]
            if d in (1, 2, 4):
                if d == 4:
                    raise RuntimeError('glob round: engine problem')
                return d, []
            if it_ == 1:
                self._after_solve(info, obj, x)
            if d == 3:
                if obj < self.inc:
                    self.inc = obj
                    self.best_x = x.copy()
                return 3, []
            if it_ == 1 and root and self.obbt:
                ch, feas, nlb, nub, nrec, nl = self._root_obbt(lb.copy(), ub.copy(), rec, x)
                self.tot.obbt_lps += nl
                if ch:
                    lb, ub, rec = nlb, nub, nrec
                    if not feas:
                        continue
            if self.S > 0:
                nc = separate(qp, x, rec, self.R, self.S)
                if nc:
                    self.tot.cuts += nc
                    self.tot.resolves += 1
                    continue
            ws_children = eng
            kind, pay, eng = self._strong(lb, ub, rec, x, obj, eng)
            if kind == 'nocand':
                return 5, []
            if kind == 'prune':
                return 1, []
            if kind == 'mod':
                lb, ub, rec = pay
                inf, lb, ub, rec = self._presolve(lb, ub, rec)
                if inf:
                    return 1, []
                continue
            j, isint, dd, ud, up_first = pay
            v = float(x[j])
            self.brlog.append((j, v))
            if isint:
                self.tot.br_int += 1
            else:
                self.tot.br_cont += 1
            kids = []
            for upc in (False, True):
                clb, cub = lb.copy(), ub.copy()
                if upc:
                    clb[j] = math.ceil(v) if isint else v
                else:
                    cub[j] = math.floor(v) if isint else v
                act = v if isint else (1.0 if upc else -1.0)
                kids.append((clb, cub, rec.copy(), obj, nd[4] + 1, ws_children[0], ws_children[1],
                             {'var': j, 'int': isint, 'act': act, 'dd': dd, 'ud': ud, 'plb': obj}))
            down_first = True
            if isint:   # IntVarHandler::getBranches (:133-190): guided dive, else the direction
                down_first = not up_first
                if math.isfinite(self.inc) and not math.isnan(self.best_x[j]):
                    down_first = self.best_x[j] < v
            return 0, kids if down_first else kids[::-1]

    def _rel_feasible(self, rec, x):
        """QuadHandler::isFeasibleToRelaxation_ (QuadHandler.cpp:955-981):
        x against every row of the relaxation with record rec (weights of
        |a| <= 1e-9 absent, terms ascending), aTol 1e-6 / rTol 1e-7."""
        q = self.nr.node_problem(self.p, rec)
        for i in range(q.m):
            act = 0.0
            for k in range(q.rowptr[i], q.rowptr[i + 1]):
                a = float(q.val[k])
                if abs(a) > 1e-9:
                    act += a * x[q.colidx[k]]
            cub, clb = float(q.rhi[i]), float(q.rlo[i])
            if act > cub + 1e-6 and (cub == 0 or act > cub + abs(cub) * 1e-7):
                return False
            if act < clb - 1e-6 and (clb == 0 or act < clb - abs(clb) * 1e-7):
                return False
        return True

    def _root_obbt(self, lb, ub, rec, x):
        """QuadHandler::postSolveRootNode (QuadHandler.cpp:1397-1547): the
        chained bound LPs of tightenLP_ (minotaur_amd/obbt.py obbt_chained,
        pinned bit for bit against the reference, over this module's CPU
        chain step oracle.chain_solve), then the rows rewritten for the new
        box.  Returns (changed, feasible, lb, ub, rec, bound LPs)."""
        from minotaur_amd import obbt
        R = self.R
        _, nlb, nub, mods, log = obbt.obbt_chained(oracle.chain_solve, self.qp, rec[:R], x,
                                                   lb=lb, ub=ub, incumbent=self.inc)
        if not mods:
            return False, True, lb, ub, rec, len(log)
        rec = rec.copy()
        rec[:R] = oracle.quad_update_rows(self.qp, nlb, nub, rec[:R])
        return True, self._rel_feasible(rec, x), nlb, nub, rec, len(log)

    def _linear(self, LB, UB, recs):
        """LinearHandler::presolveNode (LinearHandler.cpp:1592-1653) on each
        node's relaxation: the C restatement of simplePresolve (node mode,
        pinned bit for bit against the reference's LinearHandler) over the
        rows with the node's record applied, |a| <= 1e-9 dropped and terms
        ascending (LinearFunction::addTerm), the incumbent's objective bound
        once one is known.  Tightens LB / UB in place; returns infeasible."""
        from minotaur_amd.problem import from_rows
        nb = LB.shape[0]
        linf = np.zeros(nb, dtype=np.int32)
        for b in range(nb):
            q = self.nr.node_problem(self.p, recs[b])
            rows = [[(int(q.colidx[k]), float(q.val[k])) for k in range(q.rowptr[i], q.rowptr[i + 1])]
                    for i in range(q.m)]
            qn = from_rows(q.name, q.n, rows, q.rlo, q.rhi, q.vlb, q.vub, q.vtype, q.obj,
                           q.obj_const)
            r = oracle.linear_fbbt(qn, LB[b:b + 1], UB[b:b + 1],
                                   self.inc if math.isfinite(self.inc) else None)
            LB[b], UB[b] = r.lb[0], r.ub[0]
            linf[b] = int(r.infeas[0])
        return linf

    def glob_init(self, capacity, incumbent=math.inf):
        qp = self.qp
        self.cap = capacity
        st, obj, x, y, it, ws = oracle.dual_simplex_root(self.p)
        # the root inverse: nodes refactor by column replacement (K3R / K3L)
        self.ws = WarmStart(ws.head, ws.st, ws.binv, None) if st == 0 else None
        root = (qp.vlb.astype(np.float64).copy(), qp.vub.astype(np.float64).copy(),
                np.concatenate([self.rows0, self.tan0]), -math.inf, 0)
        # a node: (lb, ub, record, bound, depth[, basis head, statuses])
        self.pool = [root + (None, None)]
        self.heap = _Heap()
        if self.order == 2:
            self.heap.push({'lb': -math.inf, 'depth': 0, 'id': 0, 'node': self.pool.pop()})
            self.next_id = 1
        self.inc = incumbent
        self.best_x = np.full(qp.nv, np.nan)
        self.lplog = []        # (status, value, pivots) of every node LP in order
        self.brlog = []        # (variable, value) of every branching in order
        self.tot = _GStats()
        self.tot.incumbent = incumbent
        # StrongBrancher's pseudocosts (initialize_, :391-401) and the engine's
        # last solution value (strongBranch_ reads it after a presolve verdict)
        self.pu, self.pd = np.zeros(qp.nv), np.zeros(qp.nv)
        self.tu, self.td = np.zeros(qp.nv, dtype=np.int64), np.zeros(qp.nv, dtype=np.int64)
        self._last_val = 0.0
        self.tot.open = 1

    def _lp(self, lb, ub, vals, heads, sts):
        """The node LPs: warm 0 from the root basis; warm 1 from each node's
        parent basis refactored for its rows (None: the slack basis).
        Returns status, obj, iters, x and the final bases (warm 1)."""
        B = lb.shape[0]
        if self.warm != 1:
            st, obj, it, x = oracle.dual_simplex_rows(self.p, lb, ub, self.nr, vals,
                                                      ws=self.ws, want_x=True)
            return st.copy(), obj.copy(), it.copy(), x.copy(), None, None
        m, N = self.p.m, self.p.n + self.p.m
        st = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros((B, self.p.n))
        ho = np.zeros((B, m), dtype=np.int32)
        so = np.zeros((B, N), dtype=np.int8)
        warm = [b for b in range(B) if heads[b] is not None]
        cold = [b for b in range(B) if heads[b] is None]
        for idx, w in ((warm, True), (cold, False)):
            if not idx:
                continue
            f = np.asarray(idx)
            ws = WarmStart(np.stack([heads[b] for b in idx]), np.stack([sts[b] for b in idx]),
                           None, None) if w else None
            r = oracle.dual_simplex_rows(self.p, lb[f], ub[f], self.nr, vals[f], ws=ws,
                                         want_x=True, want_ws=True)
            st[f], obj[f], it[f], x[f], ho[f], so[f] = r
        return st, obj, it, x, ho, so

    def glob_round(self, batch, incumbent=math.inf):
        qp = self.qp
        if incumbent < self.inc:
            self.inc = incumbent
        heap = self.order == 2
        if self.brancher == 1:
            return self._round_rs(batch)
        if heap:
            nodes, ids = [], []
            while len(nodes) < batch and len(self.heap):
                top = self.heap.pop()
                if top['lb'] > self.inc - 1e-6 or \
                        abs(self.inc - top['lb']) / (abs(self.inc) + 1e-6) * 100.0 < 1e-6:
                    continue
                nodes.append(top['node'])
                ids.append(top['id'])
            nb = len(nodes)
        else:
            nb = min(batch, len(self.pool))
            if len(self.pool) + nb > self.cap:
                nb = self.cap - len(self.pool)
            if nb <= 0 and self.pool:
                raise RuntimeError('glob pool full')
            base = len(self.pool) - nb
            nodes = self.pool[base:]
            del self.pool[base:]
        if nb <= 0:
            self.tot.open = 0
            return self.tot
        R = self.R
        LB = np.stack([nd[0] for nd in nodes])
        UB = np.stack([nd[1] for nd in nodes])
        RW = np.stack([nd[2][:R] for nd in nodes])
        # the handlers' presolveNode in order (PCBProcessor.cpp:148-167):
        # LinearHandler's on the node's relaxation rows, then QuadHandler's
        linf = self._linear(LB, UB, [nd[2] for nd in nodes]) if self.lin else np.zeros(nb, np.int32)
        qt = 1 if (self.qt or self.tot.nodes == 0) else 0
        o = oracle.quad_fbbt(qp, LB, UB, self.inc, qt, RW)
        kinf_all = np.where(linf != 0, 1, o.infeas).astype(np.int32)
        # the node records: K2's rows, then the tangent slots the node inherited
        vals = np.concatenate([o.rows, np.stack([nd[2][R:] for nd in nodes])], axis=1)
        heads = [nd[5] if self.warm == 1 else None for nd in nodes]
        sts = [nd[6] if self.warm == 1 else None for nd in nodes]
        live = [b for b in range(nb) if int(kinf_all[b]) == 0]
        st = np.full(nb, 12, dtype=np.int32)
        obj = np.full(nb, math.inf)
        it = np.zeros(nb, dtype=np.int32)
        x = np.zeros((nb, qp.nv))
        wh, wst = [None] * nb, [None] * nb
        if live:
            f = np.asarray(live)
            r = self._lp(o.lb[f], o.ub[f], vals[f], [heads[b] for b in live],
                         [sts[b] for b in live])
            st[f], obj[f], it[f], x[f] = r[0], r[1], r[2], r[3]
            for b in live:
                self.lplog.append((int(st[b]), float(obj[b]), int(it[b])))
            if self.warm == 1:
                for t, b in enumerate(live):
                    wh[b], wst[b] = r[4][t], r[5][t]
        best, bidx = math.inf, -1
        children = []
        ndec = [0] * 6
        decs = []
        for b in range(nb):
            kinf = int(kinf_all[b])
            if kinf == 0:
                self.tot.lps += 1
            decs.append(decide(qp, kinf, int(st[b]), float(obj[b]), x[b], o.lb[b], o.ub[b],
                               self.inc))
        # root OBBT (PCBProcessor.cpp:256-280): the root neither pruned nor
        # feasible at its first solve; re-solved when its point leaves the
        # tightened relaxation, decided again either way
        if self.obbt and self.tot.nodes == 0 and nb == 1 and decs[0][0] in (0, 5):
            ch, feas, nlb, nub, rec, nl = self._root_obbt(o.lb[0].copy(), o.ub[0].copy(),
                                                          vals[0], x[0])
            self.tot.obbt_lps += nl
            if ch:
                o.lb[0], o.ub[0], vals[0] = nlb, nub, rec
                if not feas:
                    r = self._lp(o.lb[:1], o.ub[:1], vals[:1],
                                 [wh[0] if self.warm == 1 else None],
                                 [wst[0] if self.warm == 1 else None])
                    st[0], obj[0], x[0] = r[0][0], r[1][0], r[3][0]
                    it[0] += r[2][0]
                    if self.warm == 1:
                        wh[0], wst[0] = r[4][0], r[5][0]
                    self.tot.lps += 1
                    self.lplog.append((int(st[0]), float(obj[0]), int(r[2][0])))
                decs[0] = decide(qp, 0, int(st[0]), float(obj[0]), x[0], o.lb[0], o.ub[0],
                                 self.inc)
        # the separation loop (PCBProcessor.cpp:267-280): tangents for the
        # squares of the nodes that would branch, re-solve (warm 1: from the
        # node's last basis), decide again
        while self.S > 0:
            flagged = []
            for b in range(nb):
                if decs[b][0] in (0, 5):
                    c = separate(qp, x[b], vals[b], R, self.S)
                    if c:
                        self.tot.cuts += c
                        flagged.append(b)
            if not flagged:
                break
            f = np.asarray(flagged)
            r = self._lp(o.lb[f], o.ub[f], vals[f],
                         [wh[b] if self.warm == 1 else None for b in flagged],
                         [wst[b] if self.warm == 1 else None for b in flagged])
            for t, b in enumerate(flagged):
                st[b], obj[b], x[b] = r[0][t], r[1][t], r[3][t]
                it[b] += r[2][t]
                if self.warm == 1:
                    wh[b], wst[b] = r[4][t], r[5][t]
                self.tot.lps += 1
                self.tot.resolves += 1
                decs[b] = decide(qp, 0, int(st[b]), float(obj[b]), x[b], o.lb[b], o.ub[b],
                                 self.inc)
        kids = []
        for b in range(nb):
            kinf = int(kinf_all[b])
            if kinf == 0:
                self.tot.pivots += int(it[b])
            dec, bv, bval, bup, bint = decs[b]
            ndec[dec] += 1
            if dec == 3 and obj[b] < best:
                best, bidx = float(obj[b]), b
            if dec == 0:
                self.brlog.append((int(bv), float(bval)))
                if bint:
                    self.tot.br_int += 1
                else:
                    self.tot.br_cont += 1
                dn = math.floor(bval) if bint else bval
                up = math.ceil(bval) if bint else bval
                made = {}
                for upc in (False, True):
                    lb, ub = o.lb[b].copy(), o.ub[b].copy()
                    if upc:
                        lb[bv] = up
                    else:
                        ub[bv] = dn
                    made[upc] = (lb, ub, vals[b].copy(), float(obj[b]), nodes[b][4] + 1,
                                 wh[b], wst[b])
                if heap:
                    # QuadHandler::getBranches: down, up; IntVarHandler: the
                    # guided dive's side first with an incumbent, else the
                    # candidate's preferred direction
                    down_first = True
                    if bint:
                        down_first = bup == 0
                        if math.isfinite(self.inc) and not math.isnan(self.best_x[bv]):
                            down_first = self.best_x[bv] < bval
                    order = (False, True) if down_first else (True, False)
                    for upc in order:
                        kids.append(made[upc])
                else:
                    for c in range(2):
                        upc = (c == 1) == (bup != 0)
                        children.append(made[upc])
        if heap:
            for k in kids:
                self.heap.push({'lb': k[3], 'depth': k[4], 'id': self.next_id, 'node': k})
                self.next_id += 1
        else:
            self.pool.extend(children)
        if bidx >= 0 and best < self.inc:
            self.inc = best
            self.best_x = x[bidx].copy()
        self.tot.rounds += 1
        self.tot.nodes += nb
        for k in range(6):
            self.tot.ndec[k] += ndec[k]
        self.tot.open = len(self.heap) if heap else len(self.pool)
        self.tot.last_batch = nb
        self.tot.incumbent = self.inc
        if ndec[4]:
            raise RuntimeError('glob round: engine problem')
        return self.tot

    def _round_rs(self, batch):
        """A round with the StrongBrancher: one node (batch 1, reference
        order, parent-basis warm starts), processed as the reference does."""
        # lin 1: a brancher modification reaches p_, whose box QuadHandler
        # propagates, only through LinearHandler's copyBndsFromRel_
        # (PCBProcessor.cpp:299-305 applies it to the relaxation), so one box
        # per node restates the reference only with the linear presolve on
        if batch != 1 or self.order != 2 or self.warm != 1 or self.lin != 1:
            raise ValueError('relstronger: batch 1, order 2, warm 1, lin 1')
        while len(self.heap):
            top = self.heap.pop()
            if top['lb'] > self.inc - 1e-6 or \
                    abs(self.inc - top['lb']) / (abs(self.inc) + 1e-6) * 100.0 < 1e-6:
                continue
            break
        else:
            self.tot.open = 0
            return self.tot
        d, kids = self._process_rs(top['node'], top['id'])
        self.tot.ndec[d] += 1
        for k in kids:
            self.heap.push({'lb': k[3], 'depth': k[4], 'id': self.next_id, 'node': k})
            self.next_id += 1
        self.tot.rounds += 1
        self.tot.nodes += 1
        self.tot.open = len(self.heap)
        self.tot.last_batch = 1
        self.tot.incumbent = self.inc
        return self.tot

    def glob_best(self):
        return self.inc, self.best_x.copy()
