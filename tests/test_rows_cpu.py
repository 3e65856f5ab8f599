"""CPU: the glob-path relaxation builder (quad.relaxation_lp) and the
oracle's node-rows mode (oracle.dual_simplex_rows), checked against scipy
HiGHS on node LPs built from the K2 oracle's rewritten rows."""
import numpy as np

import oracle
from minotaur_amd.quad import random_qcqp, random_quad_boxes, relaxation_lp
from minotaur_amd.runtime import WarmStart


def test_relaxation_layout_reads_root_rows():
    qp = random_qcqp(3, nv0=14, ncon=8)
    rows0 = oracle.quad_root_rows(qp)
    p, nr = relaxation_lp(qp, rows0)
    assert p.n == qp.nv and p.m == qp.ncon + qp.nsq + 4 * qp.nbil
    assert nr.stride == qp.nrow_state
    assert nr.coef_pos.size == qp.nsq + 8 * qp.nbil and nr.row_idx.size == qp.nsq + 4 * qp.nbil
    # the record of the root box reproduces the loaded values and bounds
    q = nr.node_problem(p, rows0)
    v = np.where(np.abs(p.val) <= 1e-9, 0.0, p.val)
    assert np.array_equal(q.val, v) and np.array_equal(q.rhi, p.rhi)
    # rewritten rows are <= rows (QuadHandler: all relaxation rows <= rhs)
    assert np.all(np.isneginf(p.rlo[nr.row_idx]))


def test_oracle_rows_mode_matches_highs():
    qp = random_qcqp(7, nv0=14, ncon=8)
    rows0 = oracle.quad_root_rows(qp)
    p, nr = relaxation_lp(qp, rows0)
    st, obj, _, _, _, ws = oracle.dual_simplex_root(p)
    assert st == 0 and abs(obj - oracle.highs(p)[1]) <= 1e-7 * (1 + abs(obj))
    LB, UB = random_quad_boxes(qp, 120, 1)
    o = oracle.quad_fbbt(qp, LB, UB, None, 1, rows0)
    w = WarmStart(ws.head, ws.st, None, None)
    s1, o1, i1, _ = oracle.dual_simplex_rows(p, o.lb, o.ub, nr, o.rows, ws=w)
    s2, o2, i2, _ = oracle.dual_simplex_rows(p, o.lb, o.ub, nr, o.rows, ws=None)
    live = np.nonzero(o.infeas == 0)[0]
    assert live.size > 20
    for b in live:
        hs, hv = oracle.highs(nr.node_problem(p, o.rows[b]), o.lb[b], o.ub[b])
        assert hs == s1[b] == s2[b]
        if hs == 0:
            assert abs(o1[b] - hv) <= 1e-6 * (1 + abs(hv))
            assert abs(o2[b] - hv) <= 1e-6 * (1 + abs(hv))
    # the refactored warm basis pays: fewer pivots than the slack basis
    assert i1[live].mean() < i2[live].mean()
