"""CPU: the dual-simplex restatement (oracle/lp_dual.c) against the golden
HiGHS objectives/statuses and the reference's AMPLOsiUT known answers."""
import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, cases, load_lp


@pytest.mark.parametrize('name', cases('lp_'))
def test_oracle_lp_cold_matches_highs(name):
    p, g = load_lp(name)
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert_lp_matches(st, obj, g)


@pytest.mark.parametrize('name', ['tls4', 'knapsack', 'random0', 'random3', 'random5'])
def test_oracle_lp_warm_matches_highs(name):
    p, g = load_lp(name)
    rs, robj, x, y, it, ws = oracle.dual_simplex_root(p)
    assert rs == g['status'][0]
    st, obj, its, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ws)
    assert_lp_matches(st, obj, g)
    # warm starts need far fewer pivots than the slack basis
    st0, _, it0, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert its.sum() < it0.sum()


def test_amplosiut_known_answers():
    """AMPLOsiUT::testOsiLP / testOsiLP2 (src/testing/AMPLOsiUT.cpp:46-92)."""
    p, g = load_lp('lp0')
    st, obj, _, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert st[0] == 0 and abs(obj[0] + 8.42857) < 1e-5
    p, g = load_lp('lp_eg0')
    st, obj, _, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert st[0] == 2


def test_oracle_warm_start_resolve_is_zero_iterations():
    """AMPLOsiUT::testOsiWarmStart (:95-120): reloading the optimal basis
    re-solves in 0 iterations."""
    p, g = load_lp('lp0')
    rs, robj, x, y, it, ws = oracle.dual_simplex_root(p)
    st, obj, its, _ = oracle.dual_simplex(p, p.vlb[None], p.vub[None], ws)
    assert st[0] == 0 and its[0] == 0 and abs(obj[0] - robj) < 1e-12


def test_oracle_iteration_limit():
    p, g = load_lp('tls4')
    st, obj, it, _ = oracle.dual_simplex(p, g['lb'][:1], g['ub'][:1], None, iter_limit=3)
    assert st[0] == 6 and it[0] == 3


def test_oracle_large_m_knapsack_oa_matches_highs():
    """The restatement beyond one wave of rows (the K3L regime): the knapsack
    outer-approximation LP with f = 64 terms (m = 257), root and seeded node
    boxes warm-started from the root, against scipy HiGHS (1e-6)."""
    import math
    from minotaur_amd.problem import knapsack_oa, random_boxes
    p = knapsack_oa(f=64, N=256)
    rs, robj, x, y, it, ws = oracle.dual_simplex_root(p)
    hs, hobj = oracle.highs(p)
    assert rs == hs == 0 and abs(robj - hobj) <= 1e-6 * max(1.0, abs(hobj))
    LB, UB = random_boxes(p, 24, 4306)
    st, obj, its, _ = oracle.dual_simplex(p, LB, UB, ws)
    for b in range(24):
        hs, hobj = oracle.highs(p, LB[b], UB[b])
        assert st[b] == hs
        if hs == 0:
            assert abs(obj[b] - hobj) <= 1e-6 * max(1.0, abs(hobj))
        else:
            assert math.isinf(obj[b])
