"""GPU parity of K2 (batched QuadHandler::presolveNode) through the C ABI.

Bar: bit-exact f64 bounds and secant / McCormick row state, identical
infeasibility verdicts, mod counts and mod logs, against (a) the committed
golden vectors produced by the reference's own QuadHandler and (b) the C
oracle on larger seeded batches (ragged last wave, both node-state
variants, device-pointer path)."""
import math

import numpy as np
import pytest

import oracle
from golden_io import assert_quad_equal, bits_equal, cases, load_quad
from minotaur_amd.quad import objective_at, random_qcqp, random_quad_boxes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _inc(g):
    return math.inf if g['incumbent'] is None else g['incumbent']


@pytest.mark.parametrize('variant', [1, 2])
@pytest.mark.parametrize('name', cases('quad_'))
def test_quad_matches_reference_golden(ctx, name, variant):
    qp, g = load_quad(name)
    ctx.load_quad(qp)
    assert bits_equal(ctx.quad_rows(), g['rows_in'])
    ctx.set_fbbt_variant(variant)
    try:
        r = ctx.quad_fbbt(g['lb_in'], g['ub_in'], g['rows_in'], _inc(g), g['qt'],
                          mod_cap=g['mod_cap'])
    finally:
        ctx.set_fbbt_variant(0)
    assert_quad_equal(r.lb, r.ub, r.rows, r.infeasible, r.nmods, r.kind, r.idx, r.v1, r.v2, g)


@pytest.mark.parametrize('qt', [0, 1])
def test_quad_large_batch_vs_oracle(ctx, qt):
    qp = random_qcqp(5, nv0=16, ncon=9)
    LB, UB = random_quad_boxes(qp, 5000, 99, edge=True)   # 5000: ragged last wave
    x = 0.5 * (qp.vlb[:qp.nv0] + qp.vub[:qp.nv0])
    inc = objective_at(qp, x)
    ctx.load_quad(qp)
    rows = ctx.quad_rows()
    r = ctx.quad_fbbt(LB, UB, rows, inc, qt, mod_cap=96)
    o = oracle.quad_fbbt(qp, LB, UB, inc, qt, rows, 96)
    g = dict(lb_out=o.lb, ub_out=o.ub, rows_out=o.rows, infeas=o.infeas, nmods=o.nmods,
             mod_kind=o.kind, mod_idx=o.idx, mod_v1=o.v1, mod_v2=o.v2, mod_cap=96)
    assert_quad_equal(r.lb, r.ub, r.rows, r.infeasible, r.nmods, r.kind, r.idx, r.v1, r.v2, g)


def test_quad_dev_path_per_node_rows(ctx):
    """Device pointers, per-node row state in, chained twice (the second
    pass starts from the first pass's boxes and rows)."""
    import torch
    qp = random_qcqp(3, nv0=14, ncon=8)
    LB, UB = random_quad_boxes(qp, 777, 5, edge=True)
    ctx.load_quad(qp)
    rows0 = np.tile(ctx.quad_rows(), (LB.shape[0], 1))
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    try:
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        lb, ub, rows = t(LB), t(UB), t(rows0)
        B = LB.shape[0]
        lb2, ub2, rows2 = torch.empty_like(lb), torch.empty_like(ub), torch.empty_like(rows)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx.quad_fbbt_dev(lb, ub, rows, lb2, ub2, rows2, inf, nm, qt=1)
        lb3, ub3, rows3 = torch.empty_like(lb), torch.empty_like(ub), torch.empty_like(rows)
        inf2 = torch.zeros_like(inf)
        nm2 = torch.zeros_like(nm)
        ctx.quad_fbbt_dev(lb2, ub2, rows2, lb3, ub3, rows3, inf2, nm2, qt=0)
        ctx.sync()
        o1 = oracle.quad_fbbt(qp, LB, UB, None, 1, rows0)
        o2 = oracle.quad_fbbt(qp, o1.lb, o1.ub, None, 0, o1.rows)
        assert bits_equal(lb2.cpu().numpy(), o1.lb) and bits_equal(rows2.cpu().numpy(), o1.rows)
        assert np.array_equal(inf.cpu().numpy(), o1.infeas)
        assert bits_equal(lb3.cpu().numpy(), o2.lb) and bits_equal(ub3.cpu().numpy(), o2.ub)
        assert bits_equal(rows3.cpu().numpy(), o2.rows)
        assert np.array_equal(nm2.cpu().numpy(), o2.nmods)
        assert ctx.last_kernel_ms('quad') > 0.0
    finally:
        ctx.reset_stream()
        torch.cuda.set_stream(torch.cuda.default_stream(dev))


def test_quad_empty_and_errors(ctx):
    from minotaur_amd.runtime import MgpuError
    qp = random_qcqp(1)
    ctx.load_quad(qp)
    r = ctx.quad_fbbt(np.zeros((0, qp.nv)), np.zeros((0, qp.nv)))
    assert r.lb.shape == (0, qp.nv)
    bad = random_qcqp(1)
    bad.sq_x = bad.sq_x[::-1].copy()       # registry order violated
    with pytest.raises(MgpuError):
        ctx.load_quad(bad)
