"""GPU: the batched spatial branch-and-bound (mgpu_glob_*: K2 from the
parents' rows, K3R + K3 on each node's own rows, the glob decision and MaxVio
branching over IntVarHandler and QuadHandler candidates, children on an HBM
stack) equals its CPU restatement (oracle/glob_tree.py: the C restatements of
K2 and of the per-node-rows LP, the same decision arithmetic) round for
round -- nodes, decisions, branchings, LP solves and pivots, open nodes --
and ends on the same incumbent bits and point."""
import math

import numpy as np
import pytest

from minotaur_amd import glob as mglob
from minotaur_amd.quad import random_qcqp

pytestmark = pytest.mark.gpu

CASES = [(0, 5, 3), (1, 8, 5), (2, 6, 4), (2, 8, 5), (3, 8, 5), (4, 6, 4), (5, 8, 5),
         (0, 8, 5)]


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize('batch', [1, 16, 256])
@pytest.mark.parametrize('seed,nv0,ncon', CASES)
def test_glob_tree_matches_cpu_restatement(ctx, seed, nv0, ncon, batch):
    from glob_tree import CpuGlobContext
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    mglob.setup(ctx, qp)
    cpu = CpuGlobContext(qp)
    ctx.glob_init(1 << 15)
    cpu.glob_init(1 << 15)
    for _ in range(60 if batch == 1 else 25):
        sg, sc = ctx.glob_round(batch), cpu.glob_round(batch)
        assert (sg.rounds, sg.nodes, list(sg.ndec), sg.br_int, sg.br_cont, sg.lps, sg.pivots,
                sg.open) == (sc.rounds, sc.nodes, list(sc.ndec), sc.br_int, sc.br_cont,
                             sc.lps, sc.pivots, sc.open)
        assert sg.incumbent == sc.incumbent or (math.isinf(sg.incumbent) and
                                                math.isinf(sc.incumbent))
        if sg.open == 0:
            break
    og, xg = ctx.glob_best()
    oc, xc = cpu.glob_best()
    assert og == oc or (math.isinf(og) and math.isinf(oc))
    if math.isfinite(og):
        assert np.array_equal(xg, xc)


@pytest.mark.parametrize('seed,nv0,ncon', [(2, 16, 10), (0, 16, 10)])
def test_glob_tree_beyond_64_rows_matches_cpu(ctx, seed, nv0, ncon):
    """A relaxation past one wave of rows (m 78..90): the node LPs run on K3L
    with their rows in HBM and the root basis refactored inside the kernel;
    the tree still equals the CPU restatement round for round."""
    from glob_tree import CpuGlobContext
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    p, nr = mglob.setup(ctx, qp)
    assert p.m > 64
    cpu = CpuGlobContext(qp)
    ctx.glob_init(1 << 14)
    cpu.glob_init(1 << 14)
    for _ in range(8):
        sg, sc = ctx.glob_round(64), cpu.glob_round(64)
        assert (sg.nodes, list(sg.ndec), sg.br_int, sg.br_cont, sg.lps, sg.pivots, sg.open) == \
            (sc.nodes, list(sc.ndec), sc.br_int, sc.br_cont, sc.lps, sc.pivots, sc.open)
        assert sg.incumbent == sc.incumbent or (math.isinf(sg.incumbent) and
                                                math.isinf(sc.incumbent))
        if sg.open == 0:
            break


def test_glob_tree_closes(ctx):
    """A complete tree at batch 1024: every node decided, the stack empties,
    the incumbent is feasible for the QCQP's original constraints."""
    qp = random_qcqp(0, nv0=8, ncon=5, squares=False)
    obj, x, st, secs = mglob.solve(ctx, qp, batch=1024, capacity=1 << 18)
    assert st.open == 0 and st.nodes == sum(st.ndec) and st.ndec[4] == 0
    assert math.isfinite(obj)
    for c in range(qp.ncon):
        act = sum(qp.lval[t] * x[qp.lvar[t]] for t in range(qp.lptr[c], qp.lptr[c + 1]))
        act += sum(qp.qval[t] * x[qp.qv1[t]] * x[qp.qv2[t]]
                   for t in range(qp.qptr[c], qp.qptr[c + 1]))
        assert qp.clb[c] - 1e-5 <= act <= qp.cub[c] + 1e-5


def _qcqp_value(qp, x, f):
    v = sum(qp.lval[t] * x[qp.lvar[t]] for t in range(qp.lptr[f], qp.lptr[f + 1]))
    return v + sum(qp.qval[t] * x[qp.qv1[t]] * x[qp.qv2[t]] for t in range(qp.qptr[f], qp.qptr[f + 1]))


@pytest.mark.parametrize('seed,nv0,ncon', CASES + [(6, 10, 6), (7, 10, 6), (9, 8, 5)])
def test_glob_incumbent_sound(ctx, seed, nv0, ncon):
    """VERDICT r3 #4's soundness bar: where the tree ends with an incumbent,
    it is a QCQP-feasible point of the ORIGINAL constraints (products
    evaluated, not their auxiliaries), its objective is the incumbent, and
    the incumbent is no better than the HiGHS optimum of the root McCormick
    relaxation (a valid lower bound of the QCQP).  The tree also reports
    how many nodes closed with no branching candidate (the reference's
    NoCandToBranch, where it would call an NLP engine: DESIGN §8)."""
    from scipy.optimize import linprog
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    p, _ = mglob.setup(ctx, qp)
    obj, x, st, _ = mglob.solve(ctx, qp, batch=1024, capacity=1 << 18, loaded=True)
    assert st.open == 0 and st.ndec[4] == 0
    # the root relaxation's optimum (HiGHS) bounds the QCQP from below
    A = np.zeros((p.m, p.n))
    for r in range(p.m):
        for t in range(p.rowptr[r], p.rowptr[r + 1]):
            A[r, p.colidx[t]] += p.val[t]
    lo, hi = np.asarray(p.rlo), np.asarray(p.rhi)
    ub_rows = np.isfinite(hi)
    lb_rows = np.isfinite(lo)
    r = linprog(p.obj, A_ub=np.vstack([A[ub_rows], -A[lb_rows]]),
                b_ub=np.concatenate([hi[ub_rows], -lo[lb_rows]]),
                bounds=list(zip(p.vlb, [None if math.isinf(u) else u for u in p.vub])),
                method='highs')
    assert r.status == 0
    root_lb = r.fun + p.obj_const
    if not math.isfinite(obj):
        assert x is None
        return
    assert obj >= root_lb - 1e-6 * max(1.0, abs(root_lb)), (obj, root_lb)
    assert x is not None
    for c in range(qp.ncon):
        act = _qcqp_value(qp, x, c)
        assert qp.clb[c] - 1e-5 <= act <= qp.cub[c] + 1e-5, (c, act)
    assert np.all(x[:qp.nv0] >= qp.vlb[:qp.nv0] - 1e-9) and np.all(x[:qp.nv0] <= qp.vub[:qp.nv0] + 1e-9)
    ints = qp.vtype[:qp.nv0] != 4   # Binary / Integer (problem.CONTINUOUS = 4)
    assert np.all(np.abs(x[:qp.nv0][ints] - np.round(x[:qp.nv0][ints])) <= 1e-6)
    if qp.has_obj:
        val = _qcqp_value(qp, x, qp.ncon) + qp.obj_const
        assert abs(val - obj) <= 1e-5 * max(1.0, abs(obj)), (val, obj)
    print(f"seed {seed}: incumbent {obj:.6g}, root bound {root_lb:.6g}, nodes {st.nodes}, "
          f"no-candidate closures {st.ndec[5]}")
