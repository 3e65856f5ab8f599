"""Config 2 as a MINLP on the GPU: tls4's outer-approximation LP
(minotaur_amd/instances/tls4_oa.npz; minotaur_amd.problem.tls4_oa: its four
convex -sum sqrt(x y) rows, tls4.nl:203-222, as tangent rows, the 60 linear
rows unchanged).

* K1 node FBBT equals the reference's LinearHandler::presolveNode bit for
  bit (tests/golden/fbbt_tls4_oa_*.npz; also run by test_fbbt_gpu.py);
* node LPs equal HiGHS within 1e-6 and the oracle pivot for pivot (slack
  basis: K3; shared root basis: K3P);
* complete trees — MaxVio and reliability branching, depth- and best-first,
  root and parent warm starts — prove HiGHS' OA-MILP optimum (3.2, a lower
  bound on tls4's MINLP optimum 8.3) and evaluate the same tree as the CPU
  restatement oracle/bnb.py round for round.
"""
import math
import os

import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, bits_equal, load_fbbt, load_lp
from minotaur_amd import bnb
from minotaur_amd.problem import LinProblem

pytestmark = pytest.mark.gpu

INST = os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd', 'instances')
OA_MILP_OPT = 3.2          # HiGHS on tls4_oa.npz (tools/make_instances.py)


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _p():
    return LinProblem.load(os.path.join(INST, 'tls4_oa.npz'))


@pytest.mark.parametrize('name', ['tls4_oa_noinc', 'tls4_oa_inc3p5'])
def test_tls4_oa_fbbt_bit_exact_vs_reference(ctx, name):
    p, g = load_fbbt(name)
    ctx.load(p)
    r = ctx.fbbt(g['lb_in'], g['ub_in'],
                 math.inf if g['incumbent'] is None else g['incumbent'], mod_cap=g['mod_cap'])
    assert bits_equal(r.lb, g['lb_out']) and bits_equal(r.ub, g['ub_out'])
    assert np.array_equal(r.infeasible, g['infeas']) and np.array_equal(r.nmods, g['nmods'])


def test_tls4_oa_lp_vs_highs_and_oracle(ctx):
    p, g = load_lp('tls4_oa')
    ctx.load(p)
    r = ctx.lp_solve(g['lb'], g['ub'])                     # slack basis: K3
    assert_lp_matches(r.status, r.obj, g)
    so, _, io, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert np.array_equal(r.status, so) and np.array_equal(r.iters, io)
    _, _, _, _, _, ows = oracle.dual_simplex_root(p)
    from minotaur_amd.runtime import WarmStart
    ws = WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T))
    w = ctx.lp_solve(g['lb'], g['ub'], ws)                 # shared root basis: K3P
    assert_lp_matches(w.status, w.obj, g)
    so, _, io, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows, pfi=ctx.oracle_pfi())
    assert np.array_equal(w.status, so) and np.array_equal(w.iters, io)


def _sig(st):
    return (st.rounds, st.nodes, list(st.ndec), st.lps, st.pivots, st.sb_lps, st.sb_pruned,
            st.sb_modified, st.sb_pivots)


# (order, warm, brancher, batch): MaxVio trees of 10^5 nodes, reliability
# trees of 10^3 (the restatement's run time bounds the batch sizes)
TREES = [(0, 0, 0, 4096), (1, 0, 0, 4096), (1, 1, 0, 8192), (0, 2, 0, 4096), (1, 2, 0, 4096),
         (1, 0, 1, 256), (0, 0, 1, 1024), (1, 1, 1, 64)]


@pytest.mark.parametrize('order,warm,brancher,batch', TREES)
def test_tls4_oa_tree_proves_highs_optimum(ctx, order, warm, brancher, batch):
    from bnb import CpuBnbContext
    p = _p()
    hs, hobj = oracle.highs_milp(p)
    assert hs == 0 and abs(hobj - OA_MILP_OPT) <= 1e-9 and hobj <= 8.3
    ctx.load(p)
    og, xg, sg, _ = bnb.solve(ctx, batch=batch, capacity=1 << 20, order=order, warm=warm,
                              brancher=brancher)
    assert sg.open == 0 and sg.ndec[4] == 0
    assert abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))
    ints = np.isin(p.vtype, (0, 1))
    assert np.all(np.abs(xg[ints] - np.round(xg[ints])) <= 1e-6)
    pfi = ctx.oracle_pfi() if (warm != 1 and brancher == 0) else 0
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p, pfi), batch=batch, capacity=1 << 20, order=order,
                             warm=warm, brancher=brancher)
    assert _sig(sg) == _sig(sc)
    assert og == oc                  # every LP kernel sums the objective as the oracle does


def test_tls4_oa_tree_eta_cap_48_equals_restatement(ctx):
    """The complete tree the bench times (depth-first, warm 2, batch 16 384)
    with K3P's 48-eta build (mgpu_set_lp_pfi 48: caps above 32): the same
    rounds, pivots and optimum bits as the CPU restatement with pfi 48."""
    from bnb import CpuBnbContext
    from minotaur_amd.runtime import LP_PFI_BIG, LP_PFI_MAX
    p = _p()
    ctx.load(p)
    ctx.set_lp_pfi(LP_PFI_BIG)
    try:
        assert ctx.oracle_pfi() == LP_PFI_BIG
        og, _, sg, _ = bnb.solve(ctx, batch=16384, capacity=1 << 20, order=0, warm=2)
    finally:
        ctx.set_lp_pfi(LP_PFI_MAX)
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p, LP_PFI_BIG), batch=16384, capacity=1 << 20,
                             order=0, warm=2)
    assert sg.open == 0 and sg.ndec[4] == 0
    assert _sig(sg) == _sig(sc)
    assert og == oc and abs(og - OA_MILP_OPT) <= 1e-6


def test_tls4_oa_warm2_small_eta_cap_wide_rounds_equal_restatement(ctx):
    """with a small eta cap (9) and rounds of 32 768 nodes far more
    than a quarter of the basis-warm-started LPs fill the eta file; each must
    still go on from its own basis (one continuation slot per LP), as the
    oracle's product-form mode does, so the rounds equal the restatement's
    pivot for pivot."""
    from bnb import CpuBnbContext
    from minotaur_amd.runtime import LP_PFI_MAX
    p = _p()
    ctx.load(p)
    ctx.set_lp_pfi(9)
    try:
        assert ctx.oracle_pfi() == 9
        og, _, sg, _ = bnb.solve(ctx, batch=32768, capacity=1 << 20, order=0, warm=2,
                                 max_rounds=20)
    finally:
        ctx.set_lp_pfi(LP_PFI_MAX)
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p, 9), batch=32768, capacity=1 << 20, order=0,
                             warm=2, max_rounds=20)
    assert sg.lps > 32768            # at least one full-width round
    assert _sig(sg) == _sig(sc)
    assert og == oc
