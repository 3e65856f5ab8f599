"""GPU parity of K3L (lp_large.hip: the batched dual simplex for relaxations
with more rows than a wave has lanes; one node per workgroup, B^-1 in HBM)
through the C ABI.

Bar: K3L restates oracle/lp_dual.c pivot for pivot with the oracle's
summation orders, so statuses and iteration counts equal the oracle's and
objectives are BIT-identical (the objective is a sequential sum, as in the
oracle); optimal objectives are within 1e-6 of HiGHS (north star).  The
golden LPs (m <= 64) are forced through K3L (mgpu_set_lp_variant(2)); the
knapsack outer-approximation LPs with f = 64 and 256 terms (m = 257 and 1025
rows: SURVEY §8d configs 3 and 5) take the K3L path on their own."""
import math

import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, cases, load_lp
from minotaur_amd.problem import knapsack_oa, random_boxes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


class forced:
    """Run a block with one LP kernel forced, restoring auto afterwards."""

    def __init__(self, ctx, v):
        self.ctx, self.v = ctx, v

    def __enter__(self):
        self.ctx.set_lp_variant(self.v)

    def __exit__(self, *a):
        self.ctx.set_lp_variant(0)


@pytest.mark.parametrize('name', cases('lp_'))
def test_k3l_cold_bitwise_vs_oracle(ctx, name):
    p, g = load_lp(name)
    ctx.load(p)
    with forced(ctx, 2):
        r = ctx.lp_solve(g['lb'], g['ub'])
    assert_lp_matches(r.status, r.obj, g)
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, it)
    assert np.array_equal(r.obj, obj)


@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random0', 'random3'])
def test_k3l_warm_from_root_bitwise(ctx, name):
    p, g = load_lp(name)
    ctx.load(p)
    with forced(ctx, 2):
        root, ws = ctx.root_solve()
        r = ctx.lp_solve(g['lb'], g['ub'], ws)
    rs, robj, x, y, it, ows = oracle.dual_simplex_root(p)
    assert root.status[0] == rs and root.iters[0] == it and root.obj[0] == robj
    assert np.array_equal(ws.head, ows.head) and np.array_equal(ws.st, ows.st)
    assert np.array_equal(ws.binv_rows(), ows.binv)
    assert_lp_matches(r.status, r.obj, g)
    st, obj, its, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows)
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, its)
    assert np.array_equal(r.obj, obj)
    # K3 on the same nodes: same pivots, objective to rounding of its tree sum
    with forced(ctx, 1):
        k3 = ctx.lp_solve(g['lb'], g['ub'], ws)
    assert np.array_equal(k3.status, r.status) and np.array_equal(k3.iters, r.iters)


def test_k3l_iteration_limit_skip_and_warm_out(ctx):
    p, g = load_lp('tls4')
    ctx.load(p)
    with forced(ctx, 2):
        r = ctx.lp_solve(g['lb'][:8], g['ub'][:8], iter_limit=3)
        skip = np.array([1, 0, 1, 0, 0, 0, 0, 1], dtype=np.int32)
        r2 = ctx.lp_solve(g['lb'][:8], g['ub'][:8], skip=skip)
        full = ctx.lp_solve(g['lb'][:8], g['ub'][:8], want_ws=True)
        opt = full.status == 0
        again = ctx.lp_solve(g['lb'][:8][opt], g['ub'][:8][opt],
                             type(full.ws)(full.ws.head[opt], full.ws.st[opt], full.ws.d[opt],
                                           full.ws.binv[opt]))
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'][:8], g['ub'][:8], iter_limit=3)
    assert np.array_equal(r.status, st) and np.array_equal(r.iters, it)
    assert np.all(r2.status[skip == 1] == 12)
    assert np.array_equal(r2.status[skip == 0], full.status[skip == 0])
    assert np.all(again.status == 0) and np.all(again.iters == 0)
    assert np.array_equal(again.obj, full.obj[opt])


def test_k3l_bound_lps_bitwise(ctx):
    p, g = load_lp('tls4')
    ctx.load(p)
    _, _, _, _, _, ows = oracle.dual_simplex_root(p)
    with forced(ctx, 2):
        root, ws = ctx.root_solve()
        cols = np.arange(0, p.n, 7, dtype=np.int32)
        cols = np.concatenate([cols, cols])
        signs = np.concatenate([np.ones(cols.size // 2), -np.ones(cols.size // 2)])
        r = ctx.lp_bound(cols, signs, ws=ws)
    st, obj, it, _ = oracle.lp_bound(p, cols, signs, ws=ows)
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, it)
    assert np.array_equal(r.obj, obj)


@pytest.mark.parametrize('f,N,nodes', [(64, 256, 256), (256, 1024, 48)])
def test_k3l_large_m_knapsack_oa(ctx, f, N, nodes):
    """m = 1 + 4 f rows: root from the slack basis, then node boxes warm-started
    from the root optimum, against the oracle (bitwise) and HiGHS (1e-6)."""
    p = knapsack_oa(f=f, N=N)
    assert p.m == 1 + 4 * f and p.m > 64
    ctx.load(p)
    root, ws = ctx.root_solve()              # auto: K3L (m > 64)
    rs, robj, _, _, rit, ows = oracle.dual_simplex_root(p)
    hs, hobj = oracle.highs(p)
    assert root.status[0] == rs == hs == 0
    assert root.iters[0] == rit and root.obj[0] == robj
    assert abs(root.obj[0] - hobj) <= 1e-6 * max(1.0, abs(hobj))
    LB, UB = random_boxes(p, nodes, 4242 + f)
    r = ctx.lp_solve(LB, UB, ws)
    st, obj, its, _ = oracle.dual_simplex(p, LB, UB, ows, nthreads=8)
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, its)
    assert np.array_equal(r.obj, obj)
    assert (r.iters > 0).any()
    for b in range(0, nodes, max(1, nodes // 8)):
        hs, hobj = oracle.highs(p, LB[b], UB[b])
        assert r.status[b] == hs
        if hs == 0:
            assert abs(r.obj[b] - hobj) <= 1e-6 * max(1.0, abs(hobj))
        else:
            assert math.isinf(r.obj[b])
