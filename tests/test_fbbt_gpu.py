"""GPU parity of K1 (batched node FBBT) through the C ABI.

Bar: bit-exact f64 bounds, identical infeasibility verdicts, identical mod
counts and mod logs, against (a) the committed golden vectors produced by
the reference's own LinearHandler::presolveNode and (b) the C oracle on
larger seeded batches.
"""
import math

import numpy as np
import pytest

import oracle
from golden_io import assert_mods_equal, bits_equal, cases, load_fbbt
from minotaur_amd.problem import LinProblem, random_boxes, random_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _inc(g):
    return math.inf if g['incumbent'] is None else g['incumbent']


@pytest.mark.parametrize('variant', [1, 2, 3])
@pytest.mark.parametrize('name', cases())
def test_fbbt_matches_reference_golden(ctx, name, variant, monkeypatch):
    """variant 3 (persistent, lanes refilled from the node queue) runs on
    two waves here, so nearly every lane processes several nodes."""
    p, g = load_fbbt(name)
    ctx.load(p)
    ctx.set_fbbt_variant(variant)
    monkeypatch.setenv('MGPU_FBBT_WAVES', '2')
    try:
        r = ctx.fbbt(g['lb_in'], g['ub_in'], _inc(g), mod_cap=g['mod_cap'])
    finally:
        ctx.set_fbbt_variant(0)
    assert bits_equal(r.lb, g['lb_out'])
    assert bits_equal(r.ub, g['ub_out'])
    assert np.array_equal(r.infeasible, g['infeas'])
    assert np.array_equal(r.nmods, g['nmods'])
    assert_mods_equal(r.nmods, r.mod_var, r.mod_lu, r.mod_val, g, g['mod_cap'])


@pytest.mark.parametrize('variant', [4, 5, 6])
@pytest.mark.parametrize('name', cases())
def test_fbbt_group_matches_reference_golden(ctx, name, variant):
    """K1G (variants 4 / 5 / 6: 16 / 8 / 4 lanes per node, the activity
    sums added in term order from LDS product slots) against the
    reference's own presolveNode outputs: bounds bit for bit, verdicts and
    mod counts (K1G keeps no mod log)."""
    from minotaur_amd.runtime import MgpuError
    p, g = load_fbbt(name)
    if p.m > 64:
        pytest.skip('K1G keeps row flags in one 64-bit mask')
    ctx.load(p)
    ctx.set_fbbt_variant(variant)
    try:
        r = ctx.fbbt(g['lb_in'], g['ub_in'], _inc(g), mod_cap=0)
    except MgpuError as e:
        pytest.skip(str(e))
    finally:
        ctx.set_fbbt_variant(0)
    assert bits_equal(r.lb, g['lb_out'])
    assert bits_equal(r.ub, g['ub_out'])
    assert np.array_equal(r.infeasible, g['infeas'])
    assert np.array_equal(r.nmods, g['nmods'])


@pytest.mark.parametrize('variant', [4, 5, 6])
@pytest.mark.parametrize('inst', ['tls4_lin', 'tls4_oa'])
@pytest.mark.parametrize('inc', [math.inf, 20.0])
def test_fbbt_group_large_batch_vs_oracle(ctx, inst, inc, variant):
    """K1G on 20 001 random-branching boxes (ragged last wave) against the
    C restatement, with and without an incumbent."""
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    p = LinProblem.load(os.path.join(here, '..', 'minotaur_amd', 'instances', f'{inst}.npz'))
    LB, UB = random_boxes(p, 20001, 4242)
    ctx.load(p)
    ctx.set_fbbt_variant(variant)
    try:
        r = ctx.fbbt(LB, UB, inc)
    finally:
        ctx.set_fbbt_variant(0)
    o = oracle.linear_fbbt(p, LB, UB, None if math.isinf(inc) else inc, nthreads=8)
    assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)
    assert np.array_equal(r.infeasible, o.infeas)
    assert np.array_equal(r.nmods, o.nmods)


def _tls4():
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    return LinProblem.load(os.path.join(here, '..', 'minotaur_amd', 'instances',
                                        'tls4_lin.npz'))


@pytest.mark.parametrize('waves', [None, '7', '150'])
@pytest.mark.parametrize('inc', [math.inf, 20.0])
def test_fbbt_large_batch_vs_oracle(ctx, inc, waves, monkeypatch):
    """Ragged last wave (B not a multiple of 64) and many waves; with
    `waves` set, the persistent variant on that many waves (node queue
    refills)."""
    p = _tls4()
    LB, UB = random_boxes(p, 20001, 424242)
    ctx.load(p)
    if waves:
        ctx.set_fbbt_variant(3)
        monkeypatch.setenv('MGPU_FBBT_WAVES', waves)
    try:
        r = ctx.fbbt(LB, UB, inc)
    finally:
        ctx.set_fbbt_variant(0)
    o = oracle.linear_fbbt(p, LB, UB, None if math.isinf(inc) else inc, nthreads=8)
    assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)
    assert np.array_equal(r.infeasible, o.infeas)
    assert np.array_equal(r.nmods, o.nmods)


@pytest.mark.parametrize('inc', [math.inf, 20.0])
def test_fbbt_persistent_odd_bounds(ctx, inc, monkeypatch):
    """The persistent kernel on boxes whose [0,1] integer columns take the
    other values a bound can hold -- -0.0, fractions, an inverted pair,
    values just off 0 and 1 -- against the restatement, mod log entry by
    entry.  (Round 5 tried keeping such columns' bounds as bits in VGPRs with
    these values as escapes; this test pinned it, DESIGN §3 K1 has why it did
    not ship.)"""
    p = _tls4()
    LB, UB = random_boxes(p, 6000, 777)
    rng = np.random.default_rng(5)
    slots = np.nonzero(((p.vtype == 0) | (p.vtype == 1)) & (p.vlb >= 0) & (p.vub <= 1))[0]
    odd = np.array([-0.0, 0.25, 0.5, 1 - 2 ** -52, 2 ** -60, 0.999999, 1e-7, 1.0 + 2 ** -52])
    for b in range(LB.shape[0]):
        for j in rng.choice(slots, size=rng.integers(0, 6), replace=False):
            k = rng.integers(0, 4)
            if k == 0:
                LB[b, j] = odd[rng.integers(0, odd.size)]
            elif k == 1:
                UB[b, j] = odd[rng.integers(0, odd.size)]
            elif k == 2:
                LB[b, j], UB[b, j] = 1.0, 0.0
            else:
                LB[b, j] = -0.0
                UB[b, j] = -0.0 if rng.integers(0, 2) else 0.0
    ctx.load(p)
    ctx.set_fbbt_variant(3)
    monkeypatch.setenv('MGPU_FBBT_WAVES', '37')
    try:
        r = ctx.fbbt(LB, UB, inc, mod_cap=48)
    finally:
        ctx.set_fbbt_variant(0)
    o = oracle.linear_fbbt(p, LB, UB, None if math.isinf(inc) else inc, 48, nthreads=8)
    assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)
    assert np.array_equal(r.infeasible, o.infeas)
    assert np.array_equal(r.nmods, o.nmods)
    for b in range(LB.shape[0]):
        k = min(int(o.nmods[b]), 48)
        assert np.array_equal(r.mod_var[b, :k], o.mod_var[b, :k])
        assert np.array_equal(r.mod_lu[b, :k], o.mod_lu[b, :k])
        assert bits_equal(r.mod_val[b, :k], o.mod_val[b, :k])


def test_fbbt_global_variant_large_problem(ctx):
    """n=400 does not fit LDS: the global-scratch kernel runs automatically."""
    p = random_problem(77, n=400, m=300, density=0.02)
    LB, UB = random_boxes(p, 300, 5)
    ctx.load(p)
    r = ctx.fbbt(LB, UB, 0.0, mod_cap=64)
    o = oracle.linear_fbbt(p, LB, UB, 0.0, 64)
    assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)
    assert np.array_equal(r.infeasible, o.infeas)
    assert np.array_equal(r.nmods, o.nmods)
    for b in range(len(LB)):
        k = min(int(o.nmods[b]), 64)
        assert np.array_equal(r.mod_var[b, :k], o.mod_var[b, :k])
        assert np.array_equal(r.mod_lu[b, :k], o.mod_lu[b, :k])
        assert bits_equal(r.mod_val[b, :k], o.mod_val[b, :k])


def test_fbbt_device_pointers_and_aliasing(ctx):
    import torch
    p = _tls4()
    LB, UB = random_boxes(p, 1000, 99)
    ctx.load(p)
    host = ctx.fbbt(LB, UB, 20.0)
    dev = torch.device('cuda', 0)
    lb = torch.from_numpy(LB).to(dev)
    ub = torch.from_numpy(UB).to(dev)
    inf = torch.zeros(1000, dtype=torch.int32, device=dev)
    nm = torch.zeros(1000, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.fbbt_dev(lb, ub, lb, ub, inf, nm, 20.0)     # in place (aliased)
    ctx.sync()
    assert bits_equal(lb.cpu().numpy(), host.lb)
    assert bits_equal(ub.cpu().numpy(), host.ub)
    assert np.array_equal(inf.cpu().numpy(), host.infeasible)
    assert np.array_equal(nm.cpu().numpy(), host.nmods)


def test_fbbt_empty_and_single(ctx):
    p = _tls4()
    ctx.load(p)
    r = ctx.fbbt(np.zeros((0, p.n)), np.zeros((0, p.n)))
    assert r.lb.shape == (0, p.n)
    r = ctx.fbbt(p.vlb[None], p.vub[None])
    o = oracle.linear_fbbt(p, p.vlb[None], p.vub[None])
    assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)


def test_errors_are_reported_not_thrown(ctx):
    from minotaur_amd.runtime import Context, MgpuError
    c = Context(0)
    with pytest.raises(MgpuError, match='no problem loaded'):
        c.fbbt(np.zeros((1, 3)), np.ones((1, 3)))
    p = _tls4()
    bad = LinProblem(**{**p.__dict__})
    bad.colidx = p.colidx.copy()
    bad.colidx[1] = bad.colidx[0]          # duplicate column in row 0
    with pytest.raises(MgpuError, match='duplicate'):
        c.load(bad)
    c.close()
