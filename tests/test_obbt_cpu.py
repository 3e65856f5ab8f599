"""CPU: root OBBT host logic (minotaur_amd/obbt.py) over the C oracle's
bound LPs.  The bound LPs themselves are pinned to scipy HiGHS; the replay
of QuadHandler::tightenLP_ is checked for validity (a feasible point of the
original problem is never cut off) and for using only batched LPs."""
import math

import numpy as np
import pytest

import oracle
from minotaur_amd import obbt
from minotaur_amd.quad import random_qcqp


def _setup(seed, cutoff=math.inf):
    qp = random_qcqp(seed, nv0=8, ncon=4)
    rows = oracle.quad_root_rows(qp)
    p = obbt.relaxation_lp(qp, rows, cutoff=cutoff)
    st, ob, x, y, it, ws = oracle.dual_simplex_root(p)
    assert st == 0
    return qp, rows, p, x, ws


@pytest.mark.parametrize('seed', [0, 1, 2, 3])
def test_bound_lps_match_highs(seed):
    qp, rows, p, x, ws = _setup(seed)
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    cols, signs = obbt.bound_lp_batch(itmp)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ws)
    for k in range(cols.size):
        c = np.zeros(p.n)
        c[cols[k]] = signs[k]
        hs, ho = oracle.highs_obj(p, c)
        assert hs == st[k]
        if st[k] == 0:
            assert abs(ho - ob[k]) <= 1e-6 * max(1.0, abs(ho))
            assert abs(signs[k] * xs[k][cols[k]] - ob[k]) <= 1e-9 * max(1.0, abs(ob[k]))


@pytest.mark.parametrize('seed', [0, 1, 2, 3, 4, 5])
def test_obbt_replay_keeps_feasible_point(seed):
    qp, rows, p, x, ws = _setup(seed)
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    cols, signs = obbt.bound_lp_batch(itmp)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ws)
    res = {(int(c), float(s)): (int(st[i]), float(ob[i]), xs[i])
           for i, (c, s) in enumerate(zip(cols, signs))}
    inf, lb, ub, mods, used = obbt.replay(qp, itmp, qp.vlb, qp.vub, res)
    assert not inf
    assert used <= cols.size
    assert np.all(lb >= qp.vlb) and np.all(ub <= qp.vub)
    tol = 1e-6 * (1 + np.abs(qp.xstar))
    assert np.all(lb <= qp.xstar + tol) and np.all(qp.xstar <= ub + tol)
    for kind, v, a, b in mods:
        assert kind in (0, 1, 2)


def test_select_vars_marks():
    """itmp marks follow postSolveRootNode: a violated square with a wide
    x gets 3; narrow ranges (< 2) are never marked."""
    qp, rows, p, x, ws = _setup(1)
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    assert set(np.unique(itmp)) <= {0, 1, 2, 3}
    narrow = (qp.vub - qp.vlb) < 2
    assert np.all(itmp[narrow] == 0)


@pytest.mark.parametrize('seed', [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize('cut', [False, True])
def test_chained_obbt_restatement(seed, cut):
    """obbt_chained over the C oracle (one bound LP at a time, each from the
    previous optimal basis with rebuilt reduced costs): every LP's value is
    HiGHS's, the flagged LPs are a subset of the batch, the feasible point
    survives.  (The GPU test pins it to the reference's own tightenLP_.)"""
    qp = random_qcqp(seed, nv0=8, ncon=4)
    rows = oracle.quad_root_rows(qp)
    p0 = obbt.relaxation_lp(qp, rows)
    st, ob, x, y, it, ws = oracle.dual_simplex_root(p0)
    assert st == 0
    inc = ob + 1.0 + abs(ob) if cut else math.inf
    inf, lb, ub, mods, log = obbt.obbt_chained(oracle.chain_solve, qp, rows, x, incumbent=inc)
    assert not inf and log
    p = obbt.relaxation_lp(qp, rows, cutoff=inc)
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    cols, signs = obbt.bound_lp_batch(itmp)
    flagged = set(zip(cols.tolist(), signs.tolist()))
    for v, s, st_k, val in log:
        assert (v, s) in flagged
        c = np.zeros(p.n)
        c[v] = s
        hs, ho = oracle.highs_obj(p, c)
        assert hs == st_k
        if st_k == 0:
            assert abs(ho - val) <= 1e-6 * max(1.0, abs(ho))
    assert np.all(lb >= qp.vlb) and np.all(ub <= qp.vub)
    if not cut:   # (a cutoff may legitimately remove the known feasible point)
        tol = 1e-6 * (1 + np.abs(qp.xstar))
        assert np.all(lb <= qp.xstar + tol) and np.all(qp.xstar <= ub + tol)


def test_chain_solve_rebuilds_reduced_costs():
    """A warm basis handed over without reduced costs is re-priced for the
    new objective: the same optimum as from the slack basis."""
    qp = random_qcqp(2, nv0=8, ncon=4)
    rows = oracle.quad_root_rows(qp)
    p = obbt.relaxation_lp(qp, rows)
    st, ob, x, ws = oracle.chain_solve(p, None)
    assert st == 0 and ws is not None and ws.d is None
    q = obbt._bound_objective(p, int(qp.sq_x[0]), -1.0)
    a = oracle.chain_solve(q, ws)
    b = oracle.chain_solve(q, None)
    assert a[0] == b[0] == 0
    assert abs(a[1] - b[1]) <= 1e-9 * max(1.0, abs(b[1]))
