"""GPU: the batched QP relaxation solve (K5, MFMA KKT block) reaches the
same optimal objectives as the interior-point restatement (within 1e-6,
the north-star bar for relaxation objectives) with primal-feasible
solutions, on color_lab2_4x0 node boxes and on small random convex QPs.
On color_lab2, K5's own solutions are also certified optimal without the
restatement: each meets the LP-computed Wolfe dual bound at its x
(tests/test_qp_cpu.py dual_bound) within 1e-6."""
import os

import numpy as np
import pytest

import qp_ipm
from minotaur_amd import qp as qpm

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _check(P, LB, UB, st, ob, x, nref=None):
    B = LB.shape[0]
    assert np.all(st == 0)
    for b in range(B):
        assert np.max(np.abs(P.A @ x[b] - P.b), initial=0.0) <= 1e-7
        assert np.all(x[b] >= LB[b] - 1e-9) and np.all(x[b] <= UB[b] + 1e-9)
    for b in range(B if nref is None else nref):
        r = qp_ipm.solve_node(P.Q, P.c, P.A, P.b, LB[b], UB[b])
        assert r['status'] == 0
        assert abs(ob[b] - (r['obj'] + P.k)) <= 1e-6 * max(1.0, abs(r['obj']))


def test_color_lab2_batch(ctx):
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    ctx.load_qp(P)
    LB, UB = qpm.random_node_boxes(P, 24, 9)
    st, ob, it, x = ctx.qp_solve(LB, UB)
    _check(P, LB, UB, st, ob, x)              # every box against the restatement
    assert it.max() < 80 and ctx.last_kernel_ms('qp') > 0
    # and against the multiplier-free certificate, independent of the restatement
    from test_qp_cpu import assert_convex, dual_bound
    assert_convex(P)
    for b in range(LB.shape[0]):
        f = 0.5 * x[b] @ P.Q @ x[b] + P.c @ x[b]
        assert abs(ob[b] - (f + P.k)) <= 1e-9 * max(1.0, abs(f))
        D = dual_bound(P, LB[b], UB[b], x[b])
        tol = 1e-6 * max(1.0, abs(f))
        assert -tol <= f - D <= tol, (b, f, D)


@pytest.mark.parametrize('seed', range(3))
def test_random_qps(ctx, seed):
    from test_qp_cpu import random_qp
    P = random_qp(seed, n=20 + 7 * seed, m=3 + seed)
    ctx.load_qp(P)
    rng = np.random.default_rng(seed)
    B = 33
    LB = np.tile(P.l, (B, 1))
    UB = np.tile(P.u, (B, 1))
    st, ob, it, x = ctx.qp_solve(LB, UB)
    _check(P, LB, UB, st, ob, x, nref=3)


HS021 = os.path.join(ROOT, 'tests', 'golden', 'nl', 'hs021.nl')


def test_hs021_reference_answer(ctx):
    """The reference's own QP pin (AMPLBqpdUT, src/testing/AMPLBqpdUT.cpp:29,
    59-64): BQPD on instances/hs021 -> ProvenLocalOptimal with objective
    -99.96 within 1e-7.  Here: the .nl reader's QP (ranged rows as slack
    columns, BQPD's general-constraint bounds), the box K1 makes finite from
    the rows (qp.presolve_box), K5 -> status optimal and the reference's
    objective; and the QP tree over the same model (no integer columns: the
    root is feasible and is the answer)."""
    P = qpm.from_nl(HS021)
    LB, UB = qpm.presolve_box(ctx, P)
    ctx.load_qp(P)
    st, ob, it, x = ctx.qp_solve(LB, UB)
    assert st[0] == 0
    assert abs(ob[0] + 99.96) < 1e-7
    assert abs(x[0, 0] - 2.0) < 1e-7 and abs(x[0, 1]) < 1e-7
    obj, xt, stt, _ = qpm.solve_tree(ctx, P, batch=4, capacity=64)
    assert stt.open == 0 and stt.ndec[3] == 1
    assert abs(obj + 99.96) < 1e-7
