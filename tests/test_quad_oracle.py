"""CPU: the plain-C restatement of QuadHandler::presolveNode (oracle/
quad_fbbt.c) reproduces the reference's own outputs (golden vectors from
oracle/_ref, i.e. Minotaur's QuadHandler compiled from /root/reference) bit
for bit: bounds, verdicts, mod logs and the secant / McCormick row state."""
import numpy as np
import pytest

import oracle
from golden_io import assert_quad_equal, bits_equal, cases, load_quad


@pytest.mark.parametrize('name', cases('quad_'))
def test_quad_oracle_matches_reference_golden(name):
    qp, g = load_quad(name)
    assert bits_equal(oracle.quad_root_rows(qp), g['rows_in'])
    r = oracle.quad_fbbt(qp, g['lb_in'], g['ub_in'], g['incumbent'], g['qt'], g['rows_in'],
                         g['mod_cap'])
    assert_quad_equal(r.lb, r.ub, r.rows, r.infeas, r.nmods, r.kind, r.idx, r.v1, r.v2, g)


def test_quad_fixture_coverage():
    """The fixtures exercise every outcome: infeasible and feasible nodes,
    all mod kinds (lower, upper, both, row rewrite), both tightenQuad_ modes."""
    kinds, infeas, qts = set(), set(), set()
    for name in cases('quad_'):
        _, g = load_quad(name)
        infeas |= set(np.unique(g['infeas']).tolist())
        qts.add(g['qt'])
        for b in range(len(g['nmods'])):
            kinds |= set(g['mod_kind'][b, :min(g['nmods'][b], g['mod_cap'])].tolist())
    assert {0, 1} <= infeas
    assert {0, 1, 2, 3} <= kinds
    assert qts == {0, 1}


def test_quad_rows_per_node_stride():
    """Per-node row state ([B,R]) gives the same answer as the shared form."""
    qp, g = load_quad('qcqp2')
    B = g['lb_in'].shape[0]
    a = oracle.quad_fbbt(qp, g['lb_in'], g['ub_in'], g['incumbent'], g['qt'], g['rows_in'])
    b = oracle.quad_fbbt(qp, g['lb_in'], g['ub_in'], g['incumbent'], g['qt'],
                         np.tile(g['rows_in'], (B, 1)))
    assert bits_equal(a.lb, b.lb) and bits_equal(a.rows, b.rows)


@pytest.mark.skipif(not oracle.have_ref(), reason="reference build not present")
def test_quad_oracle_matches_reference_live():
    """With the reference library built here: fresh seeds, all modes."""
    from minotaur_amd.quad import objective_at, random_qcqp, random_quad_boxes
    for s in (71, 72, 73):
        qp = random_qcqp(s, nv0=12, ncon=7, aux_bounds='free' if s == 73 else 'product')
        LB, UB = random_quad_boxes(qp, 48, 500 + s, edge=True)
        x = 0.5 * (qp.vlb[:qp.nv0] + qp.vub[:qp.nv0])
        for inc in (None, objective_at(qp, x)):
            for qt in (0, 1):
                r = oracle.ref_quad_fbbt(qp, LB, UB, inc, qt, None, 128)
                o = oracle.quad_fbbt(qp, LB, UB, inc, qt, None, 128)
                g = dict(lb_out=r.lb, ub_out=r.ub, rows_out=r.rows, infeas=r.infeas,
                         nmods=r.nmods, mod_kind=r.kind, mod_idx=r.idx, mod_v1=r.v1,
                         mod_v2=r.v2, mod_cap=128)
                assert_quad_equal(o.lb, o.ub, o.rows, o.infeas, o.nmods, o.kind, o.idx,
                                  o.v1, o.v2, g)
