"""GPU parity of K3 (batched bounded dual simplex) through the C ABI.

Bar (north star): LP status identical and relaxation objective within 1e-6
of the golden HiGHS values; additionally the kernel restates the oracle's
dual simplex step for step, so statuses and iteration counts must equal the
oracle's exactly and objectives agree to ~1e-9.
"""
import math
import os

import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, cases, load_lp
from minotaur_amd.problem import LinProblem, random_boxes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _close(a, b, tol=1e-9):
    a, b = np.asarray(a), np.asarray(b)
    fin = np.isfinite(a) & np.isfinite(b)
    assert np.array_equal(np.isfinite(a), np.isfinite(b))
    return np.all(np.abs(a[fin] - b[fin]) <= tol * np.maximum(1, np.abs(b[fin])))


@pytest.mark.parametrize('name', cases('lp_'))
def test_lp_cold_matches_highs_and_oracle(ctx, name):
    p, g = load_lp(name)
    ctx.load(p)
    r = ctx.lp_solve(g['lb'], g['ub'])
    assert_lp_matches(r.status, r.obj, g)
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, it)
    assert _close(r.obj, obj)


@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random0', 'random3', 'random5'])
def test_lp_warm_from_root(ctx, name):
    p, g = load_lp(name)
    ctx.load(p)
    root, ws = ctx.root_solve()
    rs, robj, x, y, it, ows = oracle.dual_simplex_root(p)
    assert root.status[0] == rs and root.iters[0] == it and abs(root.obj[0] - robj) < 1e-9
    # same optimal basis as the oracle (binv is column-major in the ABI)
    assert np.array_equal(ws.head, ows.head) and np.array_equal(ws.st, ows.st)
    assert np.allclose(ws.binv_rows(), ows.binv, rtol=1e-9, atol=1e-12)
    assert np.allclose(ws.d, ows.d, rtol=1e-9, atol=1e-12)
    r = ctx.lp_solve(g['lb'], g['ub'], ws)
    assert_lp_matches(r.status, r.obj, g)
    st, obj, its, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows, pfi=ctx.oracle_pfi())
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, its)
    assert _close(r.obj, obj)
    # the dense K3 on the same shared warm start: the oracle's dense mode
    ctx.set_lp_variant(1)
    try:
        r = ctx.lp_solve(g['lb'], g['ub'], ws)
    finally:
        ctx.set_lp_variant(0)
    st, obj, its, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows)
    assert np.array_equal(r.status, st) and np.array_equal(r.iters, its)
    assert _close(r.obj, obj)


def test_amplosiut_known_answers(ctx):
    p, g = load_lp('lp0')
    ctx.load(p)
    r = ctx.lp_solve(g['lb'], g['ub'])
    assert r.status[0] == 0 and abs(r.obj[0] + 8.42857) < 1e-5
    # testOsiWarmStart: re-solve from the optimal basis takes 0 iterations
    root, ws = ctx.root_solve()
    r2 = ctx.lp_solve(p.vlb[None], p.vub[None], ws)
    assert r2.status[0] == 0 and r2.iters[0] == 0 and abs(r2.obj[0] - root.obj[0]) < 1e-12
    p, g = load_lp('lp_eg0')
    ctx.load(p)
    assert ctx.lp_solve(g['lb'], g['ub']).status[0] == 2


def test_lp_iteration_limit_and_skip(ctx):
    p, g = load_lp('tls4')
    ctx.load(p)
    r = ctx.lp_solve(g['lb'][:8], g['ub'][:8], iter_limit=3)
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'][:8], g['ub'][:8], iter_limit=3)
    assert np.array_equal(r.status, st) and np.array_equal(r.iters, it)
    skip = np.array([1, 0, 1, 0, 0, 0, 0, 1], dtype=np.int32)
    r2 = ctx.lp_solve(g['lb'][:8], g['ub'][:8], skip=skip)
    assert np.all(r2.status[skip == 1] == 12)
    full = ctx.lp_solve(g['lb'][:8], g['ub'][:8])
    assert np.array_equal(r2.status[skip == 0], full.status[skip == 0])


def test_lp_per_node_warm_start_roundtrip(ctx):
    """Per-node warm starts out -> in: every node re-solves in 0 pivots."""
    p, g = load_lp('knapsack')
    ctx.load(p)
    r = ctx.lp_solve(g['lb'], g['ub'], want_ws=True, want_x=True)
    opt = r.status == 0
    r2 = ctx.lp_solve(g['lb'][opt], g['ub'][opt],
                      type(r.ws)(r.ws.head[opt], r.ws.st[opt], r.ws.d[opt], r.ws.binv[opt]))
    assert np.all(r2.status == 0) and np.all(r2.iters == 0)
    assert _close(r2.obj, r.obj[opt], 1e-12)
    # primal solution satisfies the rows and the box
    A = p.dense()
    for b in np.nonzero(opt)[0][:50]:
        ax = A @ r.x[b]
        assert np.all(ax >= p.rlo - 1e-6) and np.all(ax <= p.rhi + 1e-6)
        assert np.all(r.x[b] >= g['lb'][b] - 1e-6) and np.all(r.x[b] <= g['ub'][b] + 1e-6)


def test_lp_large_batch_vs_oracle(ctx):
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    p = LinProblem.load(os.path.join(here, '..', 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    ctx.load(p)
    root, ws = ctx.root_solve()
    LB, UB = random_boxes(p, 5003, 31337)
    r = ctx.lp_solve(LB, UB, ws)
    _, _, _, _, _, ows = oracle.dual_simplex_root(p)
    st, obj, its, _ = oracle.dual_simplex(p, LB, UB, ows, nthreads=8, pfi=ctx.oracle_pfi())
    assert np.array_equal(r.status, st)
    assert np.array_equal(r.iters, its)
    assert _close(r.obj, obj)


def test_lp_device_path(ctx):
    import torch
    p, g = load_lp('tls4')
    ctx.load(p)
    host = ctx.lp_solve(g['lb'], g['ub'])
    dev = torch.device('cuda', 0)
    B = g['lb'].shape[0]
    lb = torch.from_numpy(g['lb']).to(dev)
    ub = torch.from_numpy(g['ub']).to(dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    obj = torch.zeros(B, dtype=torch.float64, device=dev)
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.lp_solve_dev(lb, ub, st, obj, it)
    ctx.sync()
    assert np.array_equal(st.cpu().numpy(), host.status)
    assert np.array_equal(it.cpu().numpy(), host.iters)
    assert np.array_equal(obj.cpu().numpy(), host.obj)


@pytest.mark.parametrize('name', ['tls4', 'mkp'])
def test_strong_branching_children_match_oracle(name):
    """mgpu_strong_branch (ReliabilityBrancher::strongBranch_, :469-506): the
    2k child LPs (down ub = floor(v) / up lb = ceil(v) per candidate, all from
    the node's optimal basis, iteration cap 25 as ReliabilityBrancher.cpp:101
    or none) equal the ORACLE's solves of the same child boxes from the same
    basis (oracle.dual_simplex in the arithmetic the context runs: statuses,
    pivot counts, objectives within 1e-9), and the uncapped optima equal
    HiGHS within 1e-6."""
    import os
    from minotaur_amd.problem import LinProblem, random_mkp
    from minotaur_amd.runtime import Context, WarmStart
    if name == 'tls4':
        p = LinProblem.load(os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd',
                                         'instances', 'tls4_lin.npz'))
    else:
        p = random_mkp(7, 40, 6)
    st0, _, x, _, _, ows = oracle.dual_simplex_root(p)
    assert st0 == 0
    ws = WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T))
    ints = np.nonzero(np.isin(p.vtype, (0, 1)))[0]
    frac = ints[np.abs(x[ints] - np.round(x[ints])) > 1e-6]
    cand = frac[:20] if frac.size else ints[:8]     # maxStrongCands_ = 20 (:43-67)
    vals = np.where(np.abs(x[cand] - np.round(x[cand])) > 1e-6, x[cand], x[cand] + 0.5)
    LB = np.repeat(p.vlb[None], 2 * cand.size, axis=0)
    UB = np.repeat(p.vub[None], 2 * cand.size, axis=0)
    for c, (j, v) in enumerate(zip(cand, vals)):
        UB[2 * c, j] = np.floor(v)
        LB[2 * c + 1, j] = np.ceil(v)
    ctx = Context(0)
    try:
        ctx.load(p)
        for lim in (25, 0):
            st, ob, it = ctx.strong_branch(p.vlb, p.vub, cand, vals, ws, lim)
            so, oo, io, _ = oracle.dual_simplex(p, LB, UB, ows, iter_limit=lim or 10000,
                                                pfi=ctx.oracle_pfi())
            assert np.array_equal(st, so) and np.array_equal(it, io)
            ok = np.isfinite(oo)
            assert np.array_equal(np.isfinite(ob), ok)
            assert np.all(np.abs(ob[ok] - oo[ok]) <= 1e-9 * np.maximum(1.0, np.abs(oo[ok])))
            if lim:
                assert it.max() <= 25
            else:
                for c in range(2 * cand.size):
                    hs, ho = oracle.highs(p, LB[c], UB[c])
                    assert hs == st[c]
                    if hs == 0:
                        assert abs(ob[c] - ho) <= 1e-6 * max(1.0, abs(ho))
    finally:
        ctx.close()


def test_failed_reload_leaves_no_problem():
    """A failed mgpu_load_lp invalidates the context's problem (no kernel may
    run on freed or stale buffers): the next mgpu_fbbt / mgpu_lp_solve
    returns MGPU_ERR_STATE (-3) until a load succeeds."""
    import ctypes
    from minotaur_amd.runtime import Context, MgpuError
    p = LinProblem.load(os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd',
                                     'instances', 'tls4_lin.npz'))
    ctx = Context(0)
    try:
        ctx.load(p)
        ctx.fbbt(p.vlb[None], p.vub[None])
        bad = np.array(p.colidx, dtype=np.int32)
        bad[3] = p.n + 7                                   # column out of range
        k = [np.ascontiguousarray(a) for a in (p.rowptr, bad, p.val, p.rlo, p.rhi, p.vlb, p.vub,
                                               p.vtype.astype(np.int32), p.obj)]
        rc = ctx.lib.mgpu_load_lp(ctx.h, p.n, p.m, *[a.ctypes.data_as(ctypes.c_void_p)
                                                      for a in k], 0.0)
        assert rc == -1
        with pytest.raises(MgpuError, match='rc=-3'):
            ctx.fbbt(p.vlb[None], p.vub[None])
        with pytest.raises(MgpuError, match='rc=-3'):
            ctx.lp_solve(p.vlb[None], p.vub[None])
        ctx.load(p)                                        # a good load restores it
        g = ctx.fbbt(p.vlb[None], p.vub[None])
        o = oracle.linear_fbbt(p, p.vlb[None], p.vub[None])
        assert np.array_equal(g.lb, o.lb) and np.array_equal(g.ub, o.ub)
    finally:
        ctx.close()


def test_default_iteration_limit_is_osilp_default():
    """iter_limit 0 = OsiLPEngine's maxIterLimit_ 10000 (OsiLPEngine.cpp:99),
    < 0 = none: on LPs far below the cap all three agree with the oracle at
    its default 10000, and a small explicit cap gives status 6 at exactly
    that pivot count."""
    from minotaur_amd.problem import knapsack_oa
    from minotaur_amd.runtime import Context
    p = knapsack_oa(f=40, N=64)       # m = 161: K3L from the slack basis
    LB, UB = random_boxes(p, 32, 3)
    ctx = Context(0)
    try:
        ctx.load(p)
        so, oo, io, _ = oracle.dual_simplex(p, LB, UB)
        for lim in (0, 10000, -1):
            g = ctx.lp_solve(LB, UB, iter_limit=lim)
            assert np.array_equal(g.status, so) and np.array_equal(g.iters, io)
            assert np.array_equal(g.obj, oo)
        cap = int(max(2, io.max() // 2))
        g = ctx.lp_solve(LB, UB, iter_limit=cap)
        s2, o2, i2, _ = oracle.dual_simplex(p, LB, UB, iter_limit=cap)
        assert np.array_equal(g.status, s2) and np.array_equal(g.iters, i2)
        assert np.any(g.status == 6) and np.all(g.iters[g.status == 6] == cap)
    finally:
        ctx.close()


@pytest.mark.parametrize('variant', [0, 2])
@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random3'])
def test_warm_basis_without_reduced_costs(ctx, name, variant):
    """ws_d = NULL: a basis saved under one objective, solved under another
    (HipLPEngine after changeObj, the chained OBBT): K3 (variant 0 routes a
    d-less warm start to it) and K3L rebuild y = c_B' B^-1 and d = c - A'y
    as the oracle's compute_duals does -- statuses, pivots and objective
    bits equal the oracle's."""
    import dataclasses
    from minotaur_amd.runtime import WarmStart
    p, g = load_lp(name)
    ctx.load(p)
    root, ws = ctx.root_solve()
    rng = np.random.default_rng(7)
    q = dataclasses.replace(p, obj=np.round(rng.normal(size=p.n), 3))
    ctx.load(q)
    lb, ub = g['lb'][:64], g['ub'][:64]
    ctx.set_lp_variant(variant)
    try:
        r = ctx.lp_solve(lb, ub, WarmStart(ws.head, ws.st, None, ws.binv), want_x=True)
    finally:
        ctx.set_lp_variant(0)
    ows = oracle.WarmStart(ws.head, ws.st, ws.binv_rows(), None)
    st, obj, it, _ = oracle.dual_simplex(q, lb, ub, ows)
    assert np.array_equal(r.status, st) and np.array_equal(r.iters, it)
    assert np.array_equal(r.obj, obj)


@pytest.mark.parametrize('variant', [0, 2])
@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random3'])
def test_single_lp_route_device_slots(ctx, name, variant):
    """mgpu_lp_solve1 (HipLPEngine's route): warm starts in device slots,
    box in / results out through the pinned block.  A chain of LPs, each
    from the previous one's slot, equals mgpu_lp_solve with the same warm
    starts through the host bit for bit (status, pivots, objective, x), the
    slot holds the same basis, rc is d with basic columns zeroed; ws_d = 0
    rebuilds d as a d-less host warm start does."""
    from golden_io import bits_equal
    from minotaur_amd.runtime import WarmStart
    p, g = load_lp(name)
    ctx.load(p)
    ctx.set_lp_variant(variant)
    slots = []
    try:
        prev, hws = -1, None
        for b in range(12):
            lb, ub = g['lb'][b], g['ub'][b]
            out = ctx.ws_alloc()
            slots.append(out)
            st, obj, it, x, rc = ctx.lp_solve1(lb, ub, prev, True, out)
            r = ctx.lp_solve(lb[None], ub[None], hws, want_x=True, want_ws=True)
            assert (st, it) == (int(r.status[0]), int(r.iters[0]))
            assert bits_equal(np.array([obj]), r.obj)
            if st in (0, 6):
                assert bits_equal(x, r.x[0])
                w = ctx.ws_read(out)
                assert np.array_equal(w.head, r.ws.head[0]) and np.array_equal(w.st, r.ws.st[0])
                assert bits_equal(w.d, r.ws.d[0]) and bits_equal(w.binv, r.ws.binv[0])
                assert bits_equal(rc, np.where(w.st == 3, 0.0, w.d))
                prev = out
                hws = WarmStart(r.ws.head[0], r.ws.st[0], r.ws.d[0], r.ws.binv[0])
        # a basis under a new objective: rebuilt reduced costs both ways
        q = p.__class__(**{**p.__dict__, 'obj': -p.obj})
        ctx.load(q)
        st, obj, it, x, rc = ctx.lp_solve1(p.vlb, p.vub, prev, False, -1)
        r = ctx.lp_solve(p.vlb[None], p.vub[None],
                         WarmStart(hws.head, hws.st, None, hws.binv), want_x=True)
        assert (st, it) == (int(r.status[0]), int(r.iters[0]))
        assert bits_equal(np.array([obj]), r.obj)
        # a slot written from the host reads back
        ctx.load(p)
        s2 = ctx.ws_alloc()
        slots.append(s2)
        ctx.ws_write(s2, hws)
        w = ctx.ws_read(s2)
        assert np.array_equal(w.head, hws.head) and bits_equal(w.binv, hws.binv)
    finally:
        ctx.set_lp_variant(0)
        for s in slots:
            ctx.ws_free(s)
