"""GPU parity of path warm starts (mgpu_lp_solve_path: the batched tree's
warm mode 2 — a node's basis is its pivot path from the shared root basis,
the reference's NodeIncRelaxer semantics of starting every child from its
parent's optimal basis) against oracle/lp_dual.c orc_dual_simplex_path_batch.

Bar: statuses, own pivot counts, objective bits, primal vectors and the
output paths (length, pivots, column statuses) equal the restatement's on
parent and child boxes; objectives equal HiGHS within 1e-6 on a sample.
"""
import math
import os

import numpy as np
import pytest

import oracle
from minotaur_amd.problem import LinProblem, random_boxes, random_mkp, random_problem
from minotaur_amd.runtime import PATH_INHERIT, PATH_MAX

pytestmark = pytest.mark.gpu

INST = os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd', 'instances')


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _cases():
    return {'tls4_oa': LinProblem.load(os.path.join(INST, 'tls4_oa.npz')),
            'tls4_lin': LinProblem.load(os.path.join(INST, 'tls4_lin.npz')),
            'mkp': random_mkp(1, 40, 5), 'random1': random_problem(1)}


def _root(p):
    from minotaur_amd.runtime import WarmStart
    st, _, _, _, _, ows = oracle.dual_simplex_root(p)
    if st != 0:
        pytest.skip('root LP not optimal')
    return WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T)), ows


def _both(ctx, p, LB, UB, k, path, st, ws, ows, cap, inherit):
    g, gk, gp, gs = ctx.lp_solve_path(LB, UB, ws, k, path, st, inherit)
    o = oracle.dual_simplex_path(p, LB, UB, ows, k, path, st, cap, inherit)
    assert np.array_equal(g.status, o[0])
    assert np.array_equal(g.iters, o[2])
    ok = o[0] == 0
    assert np.array_equal(g.obj[ok].view(np.int64), o[1][ok].view(np.int64))
    assert np.array_equal(g.x[ok].view(np.int64), o[3][ok].view(np.int64))
    assert np.array_equal(gk, o[4])
    for b in np.nonzero(gk > 0)[0]:
        assert np.array_equal(gp[b, :gk[b]], o[5][b, :gk[b]])
        assert np.array_equal(gs[b], o[6][b])
    return g, gk, gp, gs


def _children(p, LB, UB, x, status, k, path, st):
    """Both children of every optimal node with a fractional integer column
    (the first one), each carrying its parent's final path."""
    ints = np.isin(p.vtype, (0, 1))
    cl, cu, ck, cp, cs = [], [], [], [], []
    for b in np.nonzero(status == 0)[0]:
        fr = np.nonzero(ints & (np.abs(x[b] - np.round(x[b])) > 1e-6))[0]
        if fr.size == 0:
            continue
        j, v = fr[0], x[b][fr[0]]
        for up in (0, 1):
            lo, hi = LB[b].copy(), UB[b].copy()
            if up:
                lo[j] = math.ceil(v)
            else:
                hi[j] = math.floor(v)
            cl.append(lo)
            cu.append(hi)
            ck.append(k[b])
            cp.append(path[b])
            cs.append(st[b])
    return np.array(cl), np.array(cu), np.array(ck), np.array(cp), np.array(cs)


@pytest.mark.parametrize('name', ['tls4_oa', 'tls4_lin', 'mkp', 'random1'])
def test_path_parents_and_children_vs_oracle(ctx, name):
    p = _cases()[name]
    ctx.load(p)
    ws, ows = _root(p)
    cap = ctx.oracle_pfi()
    assert cap == PATH_MAX
    LB, UB = random_boxes(p, 3000, 31)
    f = oracle.linear_fbbt(p, LB, UB, None)
    keep = f.infeas == 0
    LB, UB = f.lb[keep], f.ub[keep]
    B, N = LB.shape[0], p.n + p.m
    k0 = np.zeros(B, np.int32)
    g, gk, gp, gs = _both(ctx, p, LB, UB, k0, np.zeros((B, PATH_MAX), np.uint32),
                          np.zeros((B, N), np.int8), ws, ows, cap, PATH_INHERIT)
    # k = 0 is the shared warm start itself: the same solves as K3P's
    s2, o2, i2, _ = oracle.dual_simplex(p, LB, UB, ows, pfi=cap)
    assert np.array_equal(g.status, s2) and np.array_equal(g.iters, i2)
    # children from their parents' paths, then grandchildren
    for gen in range(2):
        CL, CU, CK, CP, CS = _children(p, LB, UB, g.x, g.status, gk, gp, gs)
        if CL.shape[0] == 0:
            break
        g, gk, gp, gs = _both(ctx, p, CL, CU, CK, CP, CS, ws, ows, cap, PATH_INHERIT)
        LB, UB = CL, CU
        for b in np.nonzero(g.status == 0)[0][:20]:
            hs, ho = oracle.highs(p, LB[b], UB[b])
            assert hs == 0 and abs(ho - g.obj[b]) <= 1e-6 * max(1.0, abs(ho))
    if name == 'tls4_oa':
        assert (CK > 0).mean() > 0.5      # most children inherit a path


def test_path_inherit_cap_and_overflow(ctx):
    """inherit 4 hands only short paths on; a small eta cap sends child LPs
    whose replayed path fills the file into the dense continuation."""
    p = _cases()['tls4_oa']
    ctx.load(p)
    ws, ows = _root(p)
    LB, UB = random_boxes(p, 2000, 32)
    B, N = LB.shape[0], p.n + p.m
    g, gk, gp, gs = _both(ctx, p, LB, UB, np.zeros(B, np.int32),
                          np.zeros((B, PATH_MAX), np.uint32), np.zeros((B, N), np.int8), ws,
                          ows, PATH_MAX, 4)
    assert gk.max() <= 4
    ctx.set_lp_pfi(12)
    try:
        g, gk, gp, gs = _both(ctx, p, LB, UB, np.zeros(B, np.int32),
                              np.zeros((B, PATH_MAX), np.uint32), np.zeros((B, N), np.int8),
                              ws, ows, 12, 12)
        CL, CU, CK, CP, CS = _children(p, LB, UB, g.x, g.status, gk, gp, gs)
        c, _, _, _ = _both(ctx, p, CL, CU, CK, CP, CS, ws, ows, 12, 12)
        assert (c.iters + CK > 12).any()      # the continuation ran
    finally:
        ctx.set_lp_pfi(PATH_MAX)
