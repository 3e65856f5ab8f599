"""GPU: batched bound LPs (mgpu_lp_bound, K3 with per-LP objective
+-x_j) and root OBBT on top of them.

Bar (LP work, north star): statuses and iteration counts identical to the
C restatement, objectives within 1e-9 of it and within 1e-6 of scipy HiGHS;
the OBBT replay over GPU LPs gives the same tightened bounds (to 1e-6) and
the same mod sequence as the replay over the oracle's LPs."""
import math

import numpy as np
import pytest

import oracle
from minotaur_amd import obbt
from minotaur_amd.quad import objective_at, random_qcqp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _setup(ctx, seed, cutoff):
    qp = random_qcqp(seed, nv0=8, ncon=4)
    rows = oracle.quad_root_rows(qp)
    if cutoff == 'mid':
        cutoff = objective_at(qp, 0.5 * (qp.vlb[:qp.nv0] + qp.vub[:qp.nv0]))
    p = obbt.relaxation_lp(qp, rows, cutoff=cutoff)
    ctx.load(p)
    r, ws = ctx.root_solve()
    ost, oob, ox, oy, oit, ows = oracle.dual_simplex_root(p)
    return qp, rows, p, r, ws, ows, ox


@pytest.mark.parametrize('cutoff', [math.inf, 'mid'])
@pytest.mark.parametrize('seed', [0, 1, 2, 3, 4, 5])
def test_bound_lps_gpu_vs_oracle(ctx, seed, cutoff):
    qp, rows, p, r, ws, ows, ox = _setup(ctx, seed, cutoff)
    if r.status[0] != 0:
        pytest.skip('root LP not optimal under this cutoff')
    x = r.x[0]
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    cols, signs = obbt.bound_lp_batch(itmp)
    if cols.size == 0:
        cols = np.arange(p.n, dtype=np.int32)
        signs = np.where(np.arange(p.n) % 2 == 0, 1.0, -1.0)
    g = ctx.lp_bound(cols, signs, ws=ws, want_x=True)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ows, pfi=ctx.oracle_pfi())
    assert np.array_equal(g.status, st)
    assert np.array_equal(g.iters, it)
    ok = st == 0
    assert np.all(np.abs(g.obj[ok] - ob[ok]) <= 1e-9 * np.maximum(1.0, np.abs(ob[ok])))
    for k in np.nonzero(ok)[0]:
        c = np.zeros(p.n)
        c[cols[k]] = signs[k]
        hs, ho = oracle.highs_obj(p, c)
        assert hs == 0 and abs(ho - g.obj[k]) <= 1e-6 * max(1.0, abs(ho))


@pytest.mark.parametrize('seed', [0, 1, 3, 4])
def test_obbt_gpu_matches_oracle_replay(ctx, seed):
    qp, rows, p, r, ws, ows, ox = _setup(ctx, seed, math.inf)
    x = r.x[0]
    inf, lb, ub, mods, nlp, used = obbt.obbt(ctx, qp, rows, x, ws)
    itmp = obbt.select_vars(qp, x, qp.vlb, qp.vub)
    cols, signs = obbt.bound_lp_batch(itmp)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ows, pfi=ctx.oracle_pfi())
    res = {(int(c), float(s)): (int(st[i]), float(ob[i]), xs[i])
           for i, (c, s) in enumerate(zip(cols, signs))}
    inf2, lb2, ub2, mods2, used2 = obbt.replay(qp, itmp, qp.vlb, qp.vub, res)
    assert inf == inf2 and used == used2 and nlp == cols.size
    assert np.allclose(lb, lb2, rtol=1e-6, atol=1e-6) and np.allclose(ub, ub2, rtol=1e-6, atol=1e-6)
    assert [(k, v) for k, v, _, _ in mods] == [(k, v) for k, v, _, _ in mods2]


def test_bound_lps_dev_path(ctx):
    import torch
    qp, rows, p, r, ws, ows, ox = _setup(ctx, 2, math.inf)
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    try:
        from minotaur_amd.runtime import WarmStart
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        wsd = WarmStart(t(ws.head), t(ws.st), t(ws.d), t(ws.binv))
        cols = np.repeat(np.arange(p.n, dtype=np.int32), 2)
        signs = np.tile([1.0, -1.0], p.n)
        B = cols.size
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        ob = torch.zeros(B, dtype=torch.float64, device=dev)
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx.lp_bound_dev(t(p.vlb), t(p.vub), t(cols), t(signs), st, ob, it, ws=wsd)
        ctx.sync()
        h = ctx.lp_bound(cols, signs, ws=ws)
        assert np.array_equal(st.cpu().numpy(), h.status)
        assert np.array_equal(ob.cpu().numpy(), h.obj)
    finally:
        ctx.reset_stream()
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
