"""CPU: the interior-point restatement of the QP relaxation solve
(oracle/qp_ipm.py) converges on color_lab2_4x0 node boxes with a KKT
certificate (primal/dual residuals, duality gap) and agrees with an
independent solver (scipy SLSQP) on small convex QPs.  BQPD itself is
absent, so iterates are unpinned; the optimal objective of a convex QP is
unique and is what the GPU tests compare.

dual_bound (also used by tests/test_qp_gpu.py on K5's own solutions) is an
optimality certificate that needs no solver's multipliers: for a primal
point x and ANY y, z = Qx + c - A'y splits into z_l, z_u >= 0 with exact
stationarity at x, so -x'Qx/2 + b'y + l'z_l - u'z_u is a lower bound on a
convex QP's optimum (Wolfe duality); the best y is an LP, solved by HiGHS
(scipy.optimize.linprog).  A feasible x whose objective meets that bound
is optimal, whatever produced it."""
import os

import numpy as np
import pytest

import qp_ipm
from minotaur_amd import qp as qpm

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def random_qp(seed, n=12, m=3):
    rng = np.random.default_rng(seed)
    G = rng.normal(size=(n, n))
    Q = G @ G.T / n + 1e-3 * np.eye(n)
    c = rng.normal(size=n)
    A = rng.normal(size=(m, n))
    x0 = rng.uniform(0.2, 0.8, size=n)
    return qpm.QpProblem(f'rqp{seed}', Q, c, 0.0, A, A @ x0, np.zeros(n), np.ones(n),
                         np.full(n, 4, dtype=np.int32))


def dual_bound(P, l, u, x):
    """max over y of the Wolfe dual value at x (see the module docstring):
    max b'y + sum_j min(l_j z_j, u_j z_j), z = Qx + c - A'y, as an LP."""
    from scipy.optimize import linprog
    n, m = P.n, P.m
    g = P.Q @ x + P.c
    AT = P.A.T
    rows = np.vstack([np.hstack([l[:, None] * AT, np.eye(n)]),
                      np.hstack([u[:, None] * AT, np.eye(n)])])
    res = linprog(-np.concatenate([P.b, np.ones(n)]), A_ub=rows,
                  b_ub=np.concatenate([l * g, u * g]), bounds=[(None, None)] * (m + n),
                  method='highs')
    assert res.status == 0, res.message
    return -0.5 * x @ P.Q @ x - res.fun


def assert_convex(P):
    ev = np.linalg.eigvalsh(P.Q)
    assert ev.min() >= -1e-9 * max(1.0, ev.max())   # the dual bound needs Q PSD


def test_color_lab2_nodes_certified():
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    assert (P.n, P.m) == (300, 61)
    LB, UB = qpm.random_node_boxes(P, 3, 5)
    for b in range(3):
        r = qp_ipm.solve_node(P.Q, P.c, P.A, P.b, LB[b], UB[b])
        assert r['status'] == 0
        cert = qp_ipm.kkt_certificate(P.Q, P.c, P.A, P.b, LB[b], UB[b], r['x'], r['y'],
                                      r['zl'], r['zu'])
        assert cert['rp'] <= 1e-8 and cert['rd'] <= 1e-8 and cert['box'] == 0.0
        assert abs(cert['gap']) <= 1e-6 and cert['zmin'] >= 0.0


def test_color_lab2_restatement_meets_the_dual_bound():
    """The restatement's color_lab2 node optima against the multiplier-free
    certificate (dual_bound), on boxes of another seed."""
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    assert_convex(P)
    LB, UB = qpm.random_node_boxes(P, 4, 9)
    for b in range(4):
        r = qp_ipm.solve_node(P.Q, P.c, P.A, P.b, LB[b], UB[b])
        x = r['x']
        f = 0.5 * x @ P.Q @ x + P.c @ x
        D = dual_bound(P, LB[b], UB[b], x)
        tol = 1e-6 * max(1.0, abs(f))
        assert -tol <= f - D <= tol, (b, f, D)


@pytest.mark.parametrize('seed', range(4))
def test_small_qp_matches_slsqp(seed):
    from scipy.optimize import minimize
    P = random_qp(seed)
    r = qp_ipm.solve_node(P.Q, P.c, P.A, P.b, P.l, P.u)
    assert r['status'] == 0
    f = lambda x: 0.5 * x @ P.Q @ x + P.c @ x
    s = minimize(f, np.full(P.n, 0.5), jac=lambda x: P.Q @ x + P.c, method='SLSQP',
                 bounds=list(zip(P.l, P.u)),
                 constraints=[{'type': 'eq', 'fun': lambda x: P.A @ x - P.b,
                               'jac': lambda x: P.A}],
                 options={'ftol': 1e-14, 'maxiter': 500})
    assert s.success
    assert abs(r['obj'] - s.fun) <= 1e-6 * max(1.0, abs(s.fun))


HS021 = os.path.join(os.path.dirname(__file__), 'golden', 'nl', 'hs021.nl')


def test_hs021_reference_answer_by_restatement():
    """The reference's own QP answer (AMPLBqpdUT, src/testing/AMPLBqpdUT.cpp:
    29, 59-64: BQPD on instances/hs021 -> ProvenLocalOptimal, objective
    -99.96 within 1e-7; tests/golden/nl/hs021.nl is that instance file):
    the .nl reader's QP (ranged rows -> slack columns, as BQPD's general
    constraint bounds), the box the rows' FBBT makes finite (C restatement of
    LinearHandler::presolveNode), then the interior-point restatement."""
    import oracle
    P = qpm.from_nl(HS021)
    assert (P.n, P.m) == (5, 3)                  # x0, x1 + a slack per ranged row
    f = oracle.linear_fbbt(qpm.rows_problem(P), P.l[None], P.u[None])
    assert f.infeas[0] == 0 and np.all(np.isfinite(f.lb)) and np.all(np.isfinite(f.ub))
    r = qp_ipm.solve_node(P.Q, P.c, P.A, P.b, f.lb[0], f.ub[0])
    assert r['status'] == 0
    assert abs(r['obj'] + P.k + 99.96) < 1e-7
    assert abs(r['x'][0] - 2.0) < 1e-7 and abs(r['x'][1]) < 1e-7
