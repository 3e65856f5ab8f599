"""Root OBBT with batched bound LPs.

Restates QuadHandler::postSolveRootNode (src/base/QuadHandler.cpp:1397-1547)
and tightenLP_ (:2218-2297) with the LP work moved to the GPU:

* ``select_vars`` — the itmp marks of postSolveRootNode from the root LP
  solution (:1410-1512): which variables get their lower (1), upper (2) or
  both (3) bounds tightened;
* ``relaxation_lp`` — the relaxation that tightenLP_ clones (rel->clone,
  :2230): the original constraints with every product replaced by its aux
  y, the secant / McCormick rows (row state of K2), the linearised
  objective, plus the objective cutoff row  f(x) <= cub - c  (:2236-2246);
* ``obbt`` — solves EVERY bound LP the sequential loop could ask for in one
  batch (``Context.lp_bound``, K3 with per-LP objective +-x_j warm-started
  from the root basis) and then replays the loop in variable order on the
  host: setItmpFromSol_ (:2173-2216) may cancel later LPs but never adds
  one, so the batch is a superset and the replay picks the same LPs, takes
  getBndByLP_'s value (:2080-2109) and applies updatePBounds_ (:3248-3320).

The reference solves the LPs one after the other, each warm-started from the
previous one; the batch warm-starts all from the root basis.  Optimal values
agree to LP tolerance (1e-6, the north-star bar); at degenerate optima the
primal vertex fed to setItmpFromSol_ can differ, which the tests check
against the same replay over the CPU oracle's LPs.

* ``obbt_chained`` — the exact mode: tightenLP_'s loop as the reference runs
  it with HipLPEngine as bte_, one bound LP at a time on the GPU, each from
  the previous LP's optimal basis (bte_->load drops the warm start, so the
  first LP starts from the slack basis; a basis survives only ProvenOptimal /
  EngineIterationLimit, HipLPEngine::solve), the reduced costs of that basis
  rebuilt in the kernel for the new objective (mgpu_lp_solve with ws_d =
  NULL).  Same LPs, same vertices, so the same setItmpFromSol_ decisions and
  the same final bounds as the reference's postSolveRootNode.
"""
from __future__ import annotations

import dataclasses

import math

import numpy as np

from .problem import LinProblem, from_rows

MAX_VIO = 1e-3        # QuadHandler.cpp:1408
ALLOWED_GAP = 0.01    # :2183
B_TOL, R_TOL = 1e-8, 1e-7


def relaxation_lp(qp, rows, lb=None, ub=None, cutoff=math.inf) -> LinProblem:
    """The relaxation over p_'s variables as a LinProblem (linear rows only);
    ``cutoff`` < inf appends the objective cutoff row last."""
    lb = qp.vlb if lb is None else lb
    ub = qp.vub if ub is None else ub
    ymap = {}
    for k in range(qp.nsq):
        ymap[(int(qp.sq_x[k]), int(qp.sq_x[k]))] = int(qp.sq_y[k])
    for k in range(qp.nbil):
        ymap[(int(qp.bil_x0[k]), int(qp.bil_x1[k]))] = int(qp.bil_y[k])

    def lin_of(f):
        terms = [(int(qp.lvar[t]), float(qp.lval[t])) for t in range(qp.lptr[f], qp.lptr[f + 1])]
        terms += [(ymap[(int(qp.qv1[t]), int(qp.qv2[t]))], float(qp.qval[t]))
                  for t in range(qp.qptr[f], qp.qptr[f + 1])]
        return terms

    R, rlo, rhi = [], [], []
    for c in range(qp.ncon):
        R.append(lin_of(c))
        rlo.append(qp.clb[c])
        rhi.append(qp.cub[c])
    o = 0
    for k in range(qp.nsq):
        R.append([(int(qp.sq_y[k]), 1.0), (int(qp.sq_x[k]), rows[o])])
        rlo.append(-math.inf)
        rhi.append(rows[o + 1])
        o += 2
    for k in range(qp.nbil):
        for t in range(4):
            R.append([(int(qp.bil_x0[k]), rows[o]), (int(qp.bil_x1[k]), rows[o + 1]),
                      (int(qp.bil_y[k]), -1.0 if t < 2 else 1.0)])
            rlo.append(-math.inf)
            rhi.append(rows[o + 2])
            o += 3
    obj = np.zeros(qp.nv)
    oconst = 0.0
    if qp.has_obj:
        for j, a in lin_of(qp.ncon):
            obj[j] += a
        oconst = qp.obj_const
    if cutoff < math.inf:
        R.append([(j, float(obj[j])) for j in np.nonzero(obj)[0]])
        rlo.append(-math.inf)
        rhi.append(cutoff - oconst)
    return from_rows(f'{qp.name}-rel', qp.nv, R, rlo, rhi, lb, ub, qp.vtype, obj, oconst)


def select_vars(qp, x, lb, ub):
    """itmp marks of postSolveRootNode (QuadHandler.cpp:1410-1512) from the
    root relaxation solution x, with the variables' current bounds."""
    itmp = np.zeros(qp.nv, dtype=np.int64)
    for k in range(qp.nsq):
        y, x0 = int(qp.sq_y[k]), int(qp.sq_x[k])
        yv, xv = x[y], x[x0]
        vio1 = abs(xv * xv - yv)
        if vio1 > MAX_VIO and vio1 > 0.1 * abs(yv):
            if ub[x0] - lb[x0] >= 2:
                itmp[x0] = 3
            if ub[y] - lb[y] >= 2:
                vio1 = yv - lb[y]
                itmp[y] = 3 if (vio1 > MAX_VIO and vio1 > 0.1 * lb[y]) else 2

    def mark(v):
        if ub[v] - lb[v] >= 2 and itmp[v] != 3:
            vio1 = x[v] - lb[v]
            vio2 = ub[v] - x[v]
            if vio1 > MAX_VIO and vio1 > 0.1 * abs(lb[v]):
                if vio2 > MAX_VIO and vio2 > 0.1 * abs(ub[v]):
                    itmp[v] = 3
                else:
                    itmp[v] = 3 if itmp[v] == 2 else 1
            elif vio2 > MAX_VIO and vio2 > abs(ub[v]):
                itmp[v] = 3 if itmp[v] == 1 else 2

    for k in range(qp.nbil):
        y, x0, x1 = int(qp.bil_y[k]), int(qp.bil_x0[k]), int(qp.bil_x1[k])
        yv = x[y]
        vio1 = abs(x[x0] * x[x1] - yv)
        if vio1 > MAX_VIO and vio1 > 0.1 * abs(yv):
            mark(x0)
            mark(x1)
            mark(y)
    return itmp


def _set_itmp_from_sol(itmp, xs, lb, ub):
    """setItmpFromSol_, QuadHandler.cpp:2173-2216 (all variables, in order)."""
    for v in range(itmp.size):
        t = itmp[v]
        if t == 0:
            continue
        l, u, xv = lb[v], ub[v], xs[v]
        if t == 1:
            if (xv - l) / (u - l) <= ALLOWED_GAP:
                itmp[v] = 0
        elif t == 2:
            if (u - xv) / (u - l) <= ALLOWED_GAP:
                itmp[v] = 0
        else:
            if (xv - l) / (u - l) <= ALLOWED_GAP:
                itmp[v] = 2
            if (u - xv) / (u - l) <= ALLOWED_GAP:
                itmp[v] = 1


def _update_pbounds(v, nlb, nub, vtype, lb, ub, mods):
    """updatePBounds_, QuadHandler.cpp:3248-3320; returns -1 if infeasible."""
    if vtype[v] <= 3:
        nub = float(np.floor(nub))   # (inf stays inf)
        nlb = float(np.ceil(nlb))
    L, U = lb[v], ub[v]
    if nlb > U + B_TOL or nub < L - B_TOL:
        return -1
    if (nlb > L + B_TOL and nub < U - B_TOL and (L == -math.inf or nlb > L + R_TOL * abs(L))
            and (U == math.inf or nub < U - R_TOL * abs(U))):
        lb[v], ub[v] = nlb, nub
        mods.append((2, v, nlb, nub))
    elif nlb > L + B_TOL and (L == -math.inf or nlb > L + R_TOL * abs(L)):
        lb[v] = nlb
        mods.append((0, v, nlb, 0.0))
    elif nub < U - B_TOL and (U == math.inf or nub < U - R_TOL * abs(U)):
        ub[v] = nub
        mods.append((1, v, nub, 0.0))
    return 0


def bound_lp_batch(itmp):
    """Every bound LP the sequential loop could solve: min x_v for itmp 1/3,
    max x_v (min -x_v) for itmp 2/3 (3 may decay to 2 before v's turn)."""
    cols, signs = [], []
    for v in np.nonzero(itmp)[0]:
        if itmp[v] in (1, 3):
            cols.append(int(v)); signs.append(1.0)
        if itmp[v] in (2, 3):
            cols.append(int(v)); signs.append(-1.0)
    return np.asarray(cols, dtype=np.int32), np.asarray(signs)


def replay(qp, itmp0, lb, ub, results):
    """tightenLP_'s variable loop (QuadHandler.cpp:2250-2293) over solved
    bound LPs.  results[(v, sign)] = (status, obj, x).  Returns
    (infeasible, lb, ub, mods, n_lp_used)."""
    itmp = itmp0.copy()
    lb = np.array(lb, dtype=np.float64)
    ub = np.array(ub, dtype=np.float64)
    mods, used = [], 0

    def bnd(v, sign):
        st, ob, xs = results[(v, sign)]
        if st in (0, 6, 4):                   # optimal, iteration limit, unbounded
            return ob, False, xs
        return math.inf, True, xs             # infeasible / cutoff

    for v in range(qp.nv):
        t = itmp[v]
        if t == 0:
            continue
        nlb, nub = -math.inf, math.inf
        if t in (1, 3):
            used += 1
            b, inf, xs = bnd(v, 1.0)
            if inf:
                continue
            nlb = b       # (v->setItmp(itmp - 1) marks the LP clone's variable only)
            _set_itmp_from_sol(itmp, xs, lb, ub)
        if t == 2:
            used += 1
            b, inf, xs = bnd(v, -1.0)
            if inf:
                continue
            nub = -b
            _set_itmp_from_sol(itmp, xs, lb, ub)
        if _update_pbounds(v, nlb, nub, qp.vtype, lb, ub, mods) < 0:
            return True, lb, ub, mods, used
    return False, lb, ub, mods, used


def obbt(ctx, qp, rows, x_root, ws, lb=None, ub=None, incumbent=math.inf, iter_limit=0):
    """Root OBBT on the GPU: (infeasible, lb, ub, mods, n_batch_lps, n_used).
    ``ctx`` must have ``relaxation_lp(qp, rows, lb, ub, cutoff)`` loaded and
    ``ws`` its root basis."""
    lb = qp.vlb if lb is None else lb
    ub = qp.vub if ub is None else ub
    itmp = select_vars(qp, x_root, lb, ub)
    cols, signs = bound_lp_batch(itmp)
    if cols.size == 0:
        return False, np.array(lb), np.array(ub), [], 0, 0
    r = ctx.lp_bound(cols, signs, lb, ub, ws, iter_limit, want_x=True)
    res = {(int(c), float(s)): (int(r.status[i]), float(r.obj[i]), r.x[i])
           for i, (c, s) in enumerate(zip(cols, signs))}
    inf, nlb, nub, mods, used = replay(qp, itmp, lb, ub, res)
    return inf, nlb, nub, mods, int(cols.size), used


def _bound_objective(p, v, sign):
    """lp->changeObj(x_v or -x_v, 0.0) (QuadHandler.cpp:2258-2278)."""
    c = np.zeros(p.n)
    c[v] = sign
    return dataclasses.replace(p, name=f'{p.name}-obj{v}{"+" if sign > 0 else "-"}', obj=c,
                               obj_const=0.0)


class GpuChain:
    """One bound LP on the GPU the way HipLPEngine::solve runs it: the loaded
    problem's objective, warm basis (head, st, binv) without reduced costs
    (rebuilt in K3 / K3L for this objective), x and the final basis back."""

    def __init__(self, ctx, iter_limit=0):
        self.ctx, self.iter_limit = ctx, iter_limit

    def __call__(self, p, ws):
        from .runtime import WarmStart
        self.ctx.load(p)
        o = self.ctx.lp_solve(p.vlb[None], p.vub[None], ws=ws, iter_limit=self.iter_limit,
                              want_x=True, want_ws=True)
        st = int(o.status[0])
        wo = None
        if st in (0, 6):
            wo = WarmStart(o.ws.head[0], o.ws.st[0], None, o.ws.binv[0])
        return st, float(o.obj[0]), o.x[0], wo


def obbt_chained(solve, qp, rows, x_root, lb=None, ub=None, incumbent=math.inf):
    """tightenLP_ (QuadHandler.cpp:2218-2297) one bound LP at a time, each
    warm-started from the last optimal basis.  ``solve(p, ws) -> (status,
    obj, x, ws_out)`` solves LinProblem p (ws None: slack basis; ws_out None
    unless optimal / iteration limit): ``GpuChain(ctx)`` on the device, or a
    CPU restatement in tests.  Returns (infeasible, lb, ub, mods, log) with
    log[k] = (col, sign, status, value) of every LP solved, in order."""
    lb = np.array(qp.vlb if lb is None else lb, dtype=np.float64)
    ub = np.array(qp.vub if ub is None else ub, dtype=np.float64)
    itmp = select_vars(qp, x_root, lb, ub)
    # the clone: bounds frozen at load, cutoff row when an incumbent is known
    rel = relaxation_lp(qp, rows, lb.copy(), ub.copy(), incumbent)
    mods, log = [], []
    ws = None

    def bnd(v, sign):
        nonlocal ws
        st, ob, xs, wo = solve(_bound_objective(rel, v, sign), ws)
        if wo is not None:
            ws = wo
        log.append((v, sign, st, ob))
        if st in (0, 6, 4):            # getBndByLP_ (:2080-2109)
            return ob, False, xs
        return math.inf, True, xs

    for v in range(qp.nv):
        t = itmp[v]
        if t == 0:
            continue
        nlb, nub = -math.inf, math.inf
        if t in (1, 3):
            b, inf, xs = bnd(v, 1.0)
            if inf:
                continue
            nlb = b
            _set_itmp_from_sol(itmp, xs, lb, ub)
        if t == 2:
            b, inf, xs = bnd(v, -1.0)
            if inf:
                continue
            nub = -b
            _set_itmp_from_sol(itmp, xs, lb, ub)
        if _update_pbounds(v, nlb, nub, qp.vtype, lb, ub, mods) < 0:
            return True, lb, ub, mods, log
    return False, lb, ub, mods, log
