"""GPU parity of K3P (product-form dual simplex for a batch that shares one
warm start, repo:minotaur_amd/csrc/lp_pfi.hip) through the C ABI.

K3P restates oracle/lp_dual.c's product-form mode (``pfi=k``: B^{-1} kept as
k eta columns on the shared root inverse; an LP that needs more than k pivots
is continued by the dense K3 from its basis and explicit inverse).  So
statuses, pivot counts and objective bits equal the oracle's (the objective is
summed sequentially, as the oracle does); against HiGHS the north-star bar of
1e-6 holds.  Covered: the bench's node boxes (tls4-lin, column slots S = 3), the
golden warm-start cases, the overflow path (small eta caps force most LPs
through the dense re-solve), iteration limits, skips, bound LPs (OBBT
objectives), primal vectors, and instances with S = 1 and S = 4.
"""
import math
import os

import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, load_lp
from minotaur_amd.problem import LinProblem, random_boxes, random_mkp, random_problem
from minotaur_amd.runtime import LP_PFI_BIG
from minotaur_amd.runtime import LP_PFI_MAX as KCAP

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


class k3p:
    """LP calls inside run on K3P (variant 3: K3P or a loud error) with an
    eta-file cap of kmax; auto mode and the default cap afterwards."""

    def __init__(self, ctx, kmax=KCAP):
        self.ctx, self.kmax = ctx, kmax

    def __enter__(self):
        self.ctx.set_lp_variant(3)
        self.ctx.set_lp_pfi(self.kmax)

    def __exit__(self, *a):
        self.ctx.set_lp_variant(0)
        self.ctx.set_lp_pfi(KCAP)


def _tls4():
    return LinProblem.load(os.path.join(HERE, '..', 'minotaur_amd', 'instances', 'tls4_lin.npz'))


def _close(a, b, tol=1e-9):
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isfinite(a), np.isfinite(b))
    fin = np.isfinite(a)
    return np.all(np.abs(a[fin] - b[fin]) <= tol * np.maximum(1, np.abs(b[fin])))


def _root(p):
    """The oracle's root optimum as the shared warm start of both sides (the
    ABI wants B^-1 column-major), so GPU and oracle start from the same bits."""
    from minotaur_amd.runtime import WarmStart
    st, _, _, _, _, ows = oracle.dual_simplex_root(p)
    if st != 0:
        pytest.skip('root LP not optimal')
    ws = WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T))
    return ws, ows


def _check(ctx, p, LB, UB, kmax, iter_limit=0, want_x=False):
    ws, ows = _root(p)
    with k3p(ctx, kmax):
        r = ctx.lp_solve(LB, UB, ws, iter_limit=iter_limit, want_x=want_x)
    st, obj, its, x = oracle.dual_simplex(p, LB, UB, ows, nthreads=8, pfi=kmax,
                                          iter_limit=iter_limit or 10000, want_x=want_x)
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, its)
    assert _close(r.obj, obj)
    ok = st == 0
    assert np.array_equal(r.obj[ok].view(np.int64), obj[ok].view(np.int64))   # oracle bits
    if want_x:
        ok = st == 0
        assert np.allclose(r.x[ok], x[ok], rtol=1e-9, atol=1e-9)
    return r, its


@pytest.mark.parametrize('kmax', [KCAP, 8, 3])
def test_k3p_bench_boxes_vs_oracle(ctx, kmax):
    """The bench's node boxes; a small kmax sends many LPs through the overflow
    list to the dense K3 (the oracle runs the same two-stage solve)."""
    p = _tls4()
    ctx.load(p)
    LB, UB = random_boxes(p, 6007, 20261015)
    f = oracle.linear_fbbt(p, LB, UB, None)
    keep = f.infeas == 0
    r, its = _check(ctx, p, f.lb[keep], f.ub[keep], kmax)
    if kmax <= 8:
        assert (its > kmax).any()   # the overflow path ran
    # north-star bar against HiGHS on a sample
    for b in np.nonzero(r.status == 0)[0][:40]:
        hs, ho = oracle.highs(p, f.lb[keep][b], f.ub[keep][b])
        assert hs == 0 and abs(ho - r.obj[b]) <= 1e-6 * max(1.0, abs(ho))


@pytest.mark.parametrize('kmax', [LP_PFI_BIG, 40, KCAP, 24, 16, 9])
def test_k3p_tls4_oa_deep_boxes_vs_oracle(ctx, kmax):
    """Config 2's OA-LP boxes: 10.7 pivots from the root basis on average,
    18 % above 16 (the 16-eta build for caps <= 16, the 32-eta build up to
    32, the 48-eta build above)."""
    p = LinProblem.load(os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd',
                                     'instances', 'tls4_oa.npz'))
    ctx.load(p)
    LB, UB = random_boxes(p, 6007, 20261017)
    f = oracle.linear_fbbt(p, LB, UB, 3.5)
    keep = f.infeas == 0
    _, its = _check(ctx, p, f.lb[keep], f.ub[keep], kmax)
    assert (its > 16).any()


@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random0', 'random3', 'random5'])
def test_k3p_golden_warm_from_root(ctx, name):
    p, g = load_lp(name)
    if p.m > 64 or p.n + p.m > 256:
        pytest.skip('outside K3P')
    ctx.load(p)
    ws, ows = _root(p)
    with k3p(ctx):
        r = ctx.lp_solve(g['lb'], g['ub'], ws)
    assert_lp_matches(r.status, r.obj, g)
    st, obj, its, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows, pfi=KCAP)
    assert np.array_equal(r.status, st) and np.array_equal(r.iters, its)
    assert _close(r.obj, obj)


def test_k3p_primal_vectors_and_iteration_limit(ctx):
    p = _tls4()
    ctx.load(p)
    LB, UB = random_boxes(p, 1024, 7)
    _check(ctx, p, LB, UB, KCAP, want_x=True)
    _check(ctx, p, LB, UB, KCAP, iter_limit=3)
    _check(ctx, p, LB, UB, 4, iter_limit=6)


def test_k3p_skip_and_empty_box(ctx):
    p = _tls4()
    ctx.load(p)
    LB, UB = random_boxes(p, 64, 11)
    LB[5, 3], UB[5, 3] = 1.0, 0.0     # empty box: infeasible before any pivot
    skip = (np.arange(64) % 7 == 0).astype(np.int32)
    root, ws = ctx.root_solve()
    with k3p(ctx):
        r = ctx.lp_solve(LB, UB, ws, skip=skip)
        full = ctx.lp_solve(LB, UB, ws)
    assert np.all(r.status[skip == 1] == 12) and np.all(np.isinf(r.obj[skip == 1]))
    assert np.array_equal(r.status[skip == 0], full.status[skip == 0])
    assert full.status[5] == 2 and full.iters[5] == 0


@pytest.mark.parametrize('kind,n,m,seed', [('mkp', 6, 16, 3), ('mkp', 40, 8, 1),
                                           ('mkp', 120, 8, 2), ('rand', 200, 40, 1),
                                           ('rand', 60, 60, 4)])
def test_k3p_column_slot_counts(ctx, kind, n, m, seed):
    """S = ceil((n + m) / 64) from 1 to 4 column slots per lane."""
    p = (random_mkp(seed, n, m) if kind == 'mkp'
         else random_problem(seed, n=n, m=m, density=min(0.15, 4.0 / m)))
    assert p.n + p.m <= 256 and p.m <= 64
    ctx.load(p)
    LB, UB = random_boxes(p, 777, seed)
    _check(ctx, p, LB, UB, KCAP, want_x=True)
    _check(ctx, p, LB, UB, 5)


def test_k3p_bound_lps_vs_oracle(ctx):
    """Bound LPs (QuadHandler::tightenLP_ objectives +-x_j) on one box."""
    p = _tls4()
    ctx.load(p)
    ws, ows = _root(p)
    cols = np.repeat(np.arange(p.n, dtype=np.int32), 2)
    signs = np.tile([1.0, -1.0], p.n)
    with k3p(ctx):
        g = ctx.lp_bound(cols, signs, ws=ws, want_x=True)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ows, pfi=KCAP)
    assert np.array_equal(g.status, st) and np.array_equal(g.iters, it)
    assert _close(g.obj, ob)
    for k in np.nonzero(st == 0)[0][::17]:
        c = np.zeros(p.n)
        c[cols[k]] = signs[k]
        hs, ho = oracle.highs_obj(p, c)
        assert hs == 0 and abs(ho - g.obj[k]) <= 1e-6 * max(1.0, abs(ho))


def test_k3p_refuses_what_it_cannot_run(ctx):
    """Variant 3 with a per-node warm start or a warm start out fails loudly."""
    from minotaur_amd.runtime import MgpuError
    p, g = load_lp('knapsack')
    ctx.load(p)
    root, ws = ctx.root_solve()
    with k3p(ctx), pytest.raises(MgpuError):
        ctx.lp_solve(g['lb'], g['ub'], ws, want_ws=True)
    with k3p(ctx), pytest.raises(MgpuError):
        ctx.lp_solve(g['lb'], g['ub'])      # slack basis: nothing shared


def test_k3p_device_path_matches_host(ctx):
    import torch
    from minotaur_amd.runtime import WarmStart
    p = _tls4()
    ctx.load(p)
    root, ws = ctx.root_solve()
    LB, UB = random_boxes(p, 4096, 5)
    with k3p(ctx):
        host = ctx.lp_solve(LB, UB, ws)
        dev = torch.device('cuda', 0)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        wsd = WarmStart(t(ws.head), t(ws.st), t(ws.d), t(ws.binv))
        B = LB.shape[0]
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        ob = torch.zeros(B, dtype=torch.float64, device=dev)
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        ctx.lp_solve_dev(t(LB), t(UB), st, ob, it, ws=wsd)
        ctx.sync()
    assert np.array_equal(st.cpu().numpy(), host.status)
    assert np.array_equal(it.cpu().numpy(), host.iters)
    assert np.array_equal(ob.cpu().numpy(), host.obj)
    assert math.isfinite(float(ob.cpu().numpy()[host.status == 0].sum()))
