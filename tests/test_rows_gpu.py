"""GPU parity of the per-node rows path (the batched glob path): K2 rewrites
the secant / McCormick rows of every node (QuadHandler::upSqCon_ /
upBilCon_, QuadHandler.cpp:3322-3419) and the node LPs take them
(OsiLPEngine::changeConstraint, OsiLPEngine.cpp:206-243) through
mgpu_lp_solve_rows: K3R refactors the warm basis for each node's matrix,
then K3 solves.

Bar: statuses and pivot counts identical to the oracle's node-rows mode
(oracle.dual_simplex_rows: invert_basis + compute_duals + the dual simplex
restatement), objectives within 1e-9; HiGHS within 1e-6 on every node; the
rows come from K2 on the device (bit-identical to the reference QuadHandler,
tests/test_quad_gpu.py) and, where oracle/_ref is built, the oracle LP run
on the reference QuadHandler's own rows gives the same objectives."""
import math

import numpy as np
import pytest

import oracle
from minotaur_amd.quad import random_qcqp, random_quad_boxes, relaxation_lp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _setup(ctx, seed, nv0=14, ncon=8):
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon)
    ctx.load_quad(qp)
    rows0 = ctx.quad_rows()
    p, nr = relaxation_lp(qp, rows0)
    st, obj, _, _, _, ws = oracle.dual_simplex_root(p)
    assert st == 0
    ctx.load(p)
    ctx.set_node_rows(nr)
    return qp, rows0, p, nr, ws


def _close(a, b, tol):
    return abs(a - b) <= tol * (1.0 + abs(b))


@pytest.mark.parametrize('seed', [3, 7])
@pytest.mark.parametrize('warm', [True, False])
def test_rows_lp_matches_oracle_and_highs(ctx, seed, warm):
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, seed)
    LB, UB = random_quad_boxes(qp, 2000, 100 + seed)
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    w = WarmStart(ws.head, ws.st, None, None) if warm else None
    r = ctx.lp_solve_rows(q.lb, q.ub, q.rows, ws=w, skip=q.infeasible, want_x=True)
    so, oo, io, xo = oracle.dual_simplex_rows(p, q.lb, q.ub, nr, q.rows, ws=w, nthreads=8,
                                              want_x=True)
    live = q.infeasible == 0
    assert live.sum() > 100
    assert np.all(r.status[~live] == 12)
    assert np.array_equal(r.status[live], so[live])
    assert np.array_equal(r.iters[live], io[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)
    assert np.allclose(r.x[opt], xo[opt], rtol=1e-9, atol=1e-8)
    for b in np.nonzero(live)[0][::9]:
        hs, hv = oracle.highs(nr.node_problem(p, q.rows[b]), q.lb[b], q.ub[b])
        assert hs == r.status[b], b
        if hs == 0:
            assert _close(r.obj[b], hv, 1e-6), (b, r.obj[b], hv)


def test_rows_dev_pipeline_k2_to_lp(ctx):
    """K2 -> per-node LP on one stream with device pointers only: the LP
    reads K2's rows_out in place (no host copy between them)."""
    import torch
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, 7)
    LB, UB = random_quad_boxes(qp, 3000, 17)
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    try:
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        B = LB.shape[0]
        lb, ub = t(LB), t(UB)
        rows_in = t(np.tile(rows0, (B, 1)))
        lb2, ub2, rows2 = torch.empty_like(lb), torch.empty_like(ub), torch.empty_like(rows_in)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx.quad_fbbt_dev(lb, ub, rows_in, lb2, ub2, rows2, inf, nm, qt=1)
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        obj = torch.zeros(B, dtype=torch.float64, device=dev)
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        wsd = WarmStart(t(ws.head.astype(np.int32)), t(ws.st.astype(np.int8)), None, None)
        ctx.lp_solve_rows_dev(lb2, ub2, rows2, st, obj, it, ws=wsd, skip=inf)
        ctx.sync()
        assert ctx.last_kernel_ms('refactor') > 0.0 and ctx.last_kernel_ms('lp') > 0.0
        o = oracle.quad_fbbt(qp, LB, UB, None, 1, rows0)
        assert np.array_equal(inf.cpu().numpy(), o.infeas)
        so, oo, io, _ = oracle.dual_simplex_rows(p, o.lb, o.ub, nr, o.rows,
                                                 ws=WarmStart(ws.head, ws.st, None, None),
                                                 nthreads=8)
        live = o.infeas == 0
        assert np.array_equal(st.cpu().numpy()[live], so[live])
        assert np.array_equal(it.cpu().numpy()[live], io[live])
        opt = live & (so == 0)
        assert np.allclose(obj.cpu().numpy()[opt], oo[opt], rtol=1e-9, atol=1e-9)
    finally:
        ctx.reset_stream()
        torch.cuda.set_stream(torch.cuda.default_stream(dev))


@pytest.mark.skipif(not oracle.have_ref(), reason='oracle/_ref (reference build) absent')
def test_rows_lp_on_reference_quadhandler_rows(ctx):
    """The rows the reference's own QuadHandler writes (oracle/_ref) feed the
    oracle LP; the GPU path (K2 rows -> K3R -> K3) gives the same values."""
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, 3)
    LB, UB = random_quad_boxes(qp, 400, 5)
    ref = oracle.ref_quad_fbbt(qp, LB, UB, None, 1, oracle.ref_quad_root_rows(qp))
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    w = WarmStart(ws.head, ws.st, None, None)
    r = ctx.lp_solve_rows(q.lb, q.ub, q.rows, ws=w, skip=q.infeasible)
    so, oo, io, _ = oracle.dual_simplex_rows(p, ref.lb, ref.ub, nr, ref.rows, ws=w)
    live = ref.infeas == 0
    assert np.array_equal(q.infeasible, ref.infeas)
    assert np.array_equal(r.status[live], so[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)


def test_rows_singular_basis_falls_back_to_slack(ctx):
    """A warm basis that is singular for a node's matrix: K3R drops it for
    the slack basis exactly as the oracle's invert_basis failure does."""
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, 3)
    LB, UB = random_quad_boxes(qp, 64, 9)
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    vals = q.rows.copy()
    # zero every rewritten coefficient of node 0..31: a basis holding two
    # McCormick rows' x columns may become singular
    vals[:32] = 0.0
    head = ws.head.copy()
    w = WarmStart(head, ws.st, None, None)
    r = ctx.lp_solve_rows(q.lb, q.ub, vals, ws=w, skip=q.infeasible)
    so, oo, io, _ = oracle.dual_simplex_rows(p, q.lb, q.ub, nr, vals, ws=w)
    live = q.infeasible == 0
    assert np.array_equal(r.status[live], so[live])
    assert np.array_equal(r.iters[live], io[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)


def test_rows_errors(ctx):
    from minotaur_amd.quad import NodeRows
    from minotaur_amd.runtime import MgpuError
    qp, rows0, p, nr, ws = _setup(ctx, 3)
    bad = NodeRows(nr.stride, nr.coef_pos.copy(), nr.coef_src.copy(), nr.row_idx, nr.lo_src,
                   nr.hi_src)
    bad.coef_pos[1] = bad.coef_pos[0]          # repeated entry
    with pytest.raises(MgpuError):
        ctx.set_node_rows(bad)
    with pytest.raises(MgpuError):             # the failed call cleared the map
        ctx.lp_solve_rows(p.vlb[None], p.vub[None], rows0[None])
    ctx.set_node_rows(nr)
    r = ctx.lp_solve_rows(np.zeros((0, p.n)), np.zeros((0, p.n)), np.zeros((0, nr.stride)))
    assert r.status.shape == (0,)
    ctx.load(p)                                # a reload clears the map
    with pytest.raises(MgpuError):
        ctx.lp_solve_rows(p.vlb[None], p.vub[None], rows0[None])


def test_lp_refactor_single_basis(ctx):
    """mgpu_lp_refactor (what HipLPEngine runs after changeConstraint): the
    kept basis refactored for the loaded matrix equals numpy's inverse of the
    basis matrix and the oracle LP from that basis takes the same pivots;
    a singular basis comes back as the slack basis."""
    from minotaur_amd.problem import random_problem
    from minotaur_amd.runtime import WarmStart
    p = random_problem(5, n=30, m=20)
    ctx.load(p)
    _, ws = ctx.root_solve()
    q = random_problem(5, n=30, m=20)
    q.val = q.val * (1.0 + 0.05 * np.sin(np.arange(q.nnz)))   # rows changed
    ctx.load(q)
    w, sing = ctx.lp_refactor(ws.head, ws.st)
    assert sing == 0
    A = np.hstack([q.dense(), -np.eye(q.m)])
    Bm = A[:, w.head]
    binv = w.binv.T                      # column-major -> (B^-1)[i, k]
    assert np.allclose(binv @ Bm, np.eye(q.m), atol=1e-9)
    y = np.array([q.obj[h] if h < q.n else 0.0 for h in w.head]) @ binv
    cfull = np.concatenate([q.obj, np.zeros(q.m)])
    d = cfull - A.T @ y
    nb = w.st != 3
    assert np.allclose(w.d[nb], d[nb], atol=1e-9)
    # the solve from the refactored basis = the oracle's from (head, st)
    r = ctx.lp_solve(q.vlb[None], q.vub[None], ws=WarmStart(w.head, w.st, w.d, w.binv))
    from minotaur_amd.quad import NodeRows
    none = NodeRows(1, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32),
                    np.zeros(0, np.int32), np.zeros(0, np.int32))
    so, oo, io, _ = oracle.dual_simplex_rows(q, q.vlb[None], q.vub[None], none, np.zeros((1, 1)),
                                             ws=WarmStart(ws.head, ws.st, None, None))
    assert r.status[0] == so[0] and r.iters[0] == io[0]
    assert abs(r.obj[0] - oo[0]) <= 1e-9 * max(1.0, abs(oo[0]))
    # singular: two basis positions on the same slack column
    h2 = ws.head.copy()
    h2[1] = h2[0]
    w2, sing2 = ctx.lp_refactor(h2, ws.st)
    assert sing2 == 1 and np.array_equal(w2.head, np.arange(q.n, q.n + q.m))


@pytest.mark.parametrize('seed,nv0,ncon', [(1, 16, 10), (0, 18, 12), (1, 20, 14)])
@pytest.mark.parametrize('warm', [True, False])
def test_rows_lp_beyond_64_rows(ctx, seed, nv0, ncon, warm):
    """Per-node rows past one wave of rows (m = 76..104): K3L takes the
    node's matrix into its HBM slot and, for a warm basis given as head +
    statuses, refactors it in the kernel (the oracle's invert_basis, then
    compute_duals).  Statuses and pivots equal the oracle's node-rows mode,
    objectives within 1e-9, HiGHS within 1e-6."""
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, seed, nv0=nv0, ncon=ncon)
    assert p.m > 64
    LB, UB = random_quad_boxes(qp, 300, 700 + seed)
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    w = WarmStart(ws.head, ws.st, None, None) if warm else None
    r = ctx.lp_solve_rows(q.lb, q.ub, q.rows, ws=w, skip=q.infeasible, want_x=True)
    so, oo, io, xo = oracle.dual_simplex_rows(p, q.lb, q.ub, nr, q.rows, ws=w, nthreads=8,
                                              want_x=True)
    live = q.infeasible == 0
    assert live.sum() > 30
    assert np.all(r.status[~live] == 12)
    assert np.array_equal(r.status[live], so[live])
    assert np.array_equal(r.iters[live], io[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)
    assert np.allclose(r.x[opt], xo[opt], rtol=1e-9, atol=1e-8)
    for b in np.nonzero(live)[0][::7]:
        hs, hv = oracle.highs(nr.node_problem(p, q.rows[b]), q.lb[b], q.ub[b])
        assert hs == r.status[b], b
        if hs == 0:
            assert _close(r.obj[b], hv, 1e-6), (b, r.obj[b], hv)


@pytest.mark.parametrize('seed', [3, 7, 8, 12])
def test_rows_lp_column_replacement_refactor(ctx, seed):
    """K3R given the root inverse (mgpu_lp_solve_rows ws_binv): each node's
    basis is refactored by replacing only the basic columns its rows
    changed (oracle colrep_refactor), Gauss-Jordan when a pivot is tiny.
    Statuses and pivots equal the oracle's same mode, objectives 1e-9,
    HiGHS 1e-6."""
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, seed)
    LB, UB = random_quad_boxes(qp, 3000, 300 + seed)
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    wg = WarmStart(ws.head, ws.st, None, np.ascontiguousarray(ws.binv.T))   # ABI: column-major
    wo = oracle.WarmStart(ws.head, ws.st, ws.binv, None)                    # oracle: row-major
    r = ctx.lp_solve_rows(q.lb, q.ub, q.rows, ws=wg, skip=q.infeasible, want_x=True)
    so, oo, io, xo = oracle.dual_simplex_rows(p, q.lb, q.ub, nr, q.rows, ws=wo, nthreads=8,
                                              want_x=True)
    live = q.infeasible == 0
    assert live.sum() > 100
    assert np.array_equal(r.status[live], so[live])
    assert np.array_equal(r.iters[live], io[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)
    assert np.allclose(r.x[opt], xo[opt], rtol=1e-9, atol=1e-8)
    for b in np.nonzero(live)[0][::23]:
        hs, hv = oracle.highs(nr.node_problem(p, q.rows[b]), q.lb[b], q.ub[b])
        assert hs == r.status[b], b
        if hs == 0:
            assert _close(r.obj[b], hv, 1e-6), (b, r.obj[b], hv)


@pytest.mark.parametrize('seed,nv0,ncon', [(1, 16, 10), (0, 18, 12)])
def test_rows_lp_column_replacement_beyond_64_rows(ctx, seed, nv0, ncon):
    """The column replacement inside K3L (m = 76..100): from the root inverse,
    the changed basic columns swapped in one update each; statuses and pivots
    equal the oracle's same mode, objectives 1e-9, HiGHS 1e-6."""
    from minotaur_amd.runtime import WarmStart
    qp, rows0, p, nr, ws = _setup(ctx, seed, nv0=nv0, ncon=ncon)
    assert p.m > 64
    LB, UB = random_quad_boxes(qp, 300, 900 + seed)
    q = ctx.quad_fbbt(LB, UB, rows0, qt=1)
    wg = WarmStart(ws.head, ws.st, None, np.ascontiguousarray(ws.binv.T))
    wo = oracle.WarmStart(ws.head, ws.st, ws.binv, None)
    r = ctx.lp_solve_rows(q.lb, q.ub, q.rows, ws=wg, skip=q.infeasible, want_x=True)
    so, oo, io, xo = oracle.dual_simplex_rows(p, q.lb, q.ub, nr, q.rows, ws=wo, nthreads=8,
                                              want_x=True)
    live = q.infeasible == 0
    assert live.sum() > 30
    assert np.array_equal(r.status[live], so[live])
    assert np.array_equal(r.iters[live], io[live])
    opt = live & (so == 0)
    assert np.allclose(r.obj[opt], oo[opt], rtol=1e-9, atol=1e-9)
    for b in np.nonzero(live)[0][::7]:
        hs, hv = oracle.highs(nr.node_problem(p, q.rows[b]), q.lb[b], q.ub[b])
        assert hs == r.status[b], b
        if hs == 0:
            assert _close(r.obj[b], hv, 1e-6), (b, r.obj[b], hv)
