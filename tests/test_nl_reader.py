"""The `.nl` reader (minotaur_amd/nl.py) against the
headers and contents of the reference's own test instances.

The reference reads these files through ASL (AMPLInterface::readInstance,
src/interfaces/AMPLInterface.cpp), which is absent; what the files declare
in their header lines is the pin:
  tls4.nl:2-9        105 vars, 64 rows (20 equalities), 588 Jacobian nnz,
                     4 nonlinear rows, 85 binaries, 4 nonlinear integers,
                     25 objective-gradient entries;
  nvs08.nl:2-8       3 vars, 3 rows (all nonlinear), 9 Jacobian nnz,
                     1 nonlinear objective, 2 nonlinear integers;
  color_lab2_4x0.nl  (binary "b" format) 300 vars, 61 rows, 360 nnz.
tls4.nl and nvs08.nl are committed as data under tests/golden/nl/;
color_lab2_4x0.nl (1.5 MB) is read from /root/reference when present.
"""
import math
import os

import numpy as np
import pytest

from minotaur_amd.nl import evaluate, objective_value, read_nl, row_value
from minotaur_amd.problem import LinProblem, from_nl_linear, nvs08_oa

HERE = os.path.dirname(os.path.abspath(__file__))
NL = os.path.join(HERE, 'golden', 'nl')
INST = os.path.join(HERE, '..', 'minotaur_amd', 'instances')
COLOR = '/root/reference/test_instances/color_lab2_4x0.nl'


def _nnz(m):
    return sum(len(r) for r in m.rows)


def test_tls4_header_and_structure():
    m = read_nl(os.path.join(NL, 'tls4.nl'))
    assert (m.n, m.m, _nnz(m)) == (105, 64, 588)
    assert np.nonzero(m.con_nonlinear)[0].tolist() == [0, 1, 2, 3]
    assert int(np.sum(m.con_lb == m.con_ub)) == 20
    assert int(np.sum(m.var_type == 0)) == 85
    assert np.nonzero(m.var_type == 1)[0].tolist() == [16, 17, 18, 19]
    assert int(np.sum(m.var_type == 4)) == 16
    assert len(m.obj_grad) == 25 and not m.obj_nonlinear and m.obj_sense == 0
    # the nonlinear rows are -sum_i sqrt(v_{16+i} * v_{4r+i}) (tls4.nl:194-259)
    rng = np.random.default_rng(0)
    for r in range(4):
        x = rng.uniform(1.0, 9.0, m.n)
        v, g = evaluate(m.con_expr[r], x)
        ref = -sum(math.sqrt(x[16 + i] * x[4 * r + i]) for i in range(4))
        assert abs(v - ref) <= 1e-12 * abs(ref)
        k = 4 * r + 1
        assert abs(g[k] + 0.5 * math.sqrt(x[17] / x[k])) <= 1e-12


def test_tls4_lin_instance_is_the_reader_output():
    """The committed config-2 instance is exactly the linear rows the reader
    returns (SURVEY §0.1 "tls4-lin": 60 rows, 412 nnz after |a| <= 1e-9
    terms are dropped)."""
    got = from_nl_linear(read_nl(os.path.join(NL, 'tls4.nl')), name='tls4-lin')
    ref = LinProblem.load(os.path.join(INST, 'tls4_lin.npz'))
    assert (got.n, got.m, got.nnz) == (105, 60, 412)
    for k in ('rowptr', 'colidx', 'val', 'rlo', 'rhi', 'vlb', 'vub', 'vtype', 'obj'):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k


def test_nvs08_header_and_expressions():
    m = read_nl(os.path.join(NL, 'nvs08.nl'))
    assert (m.n, m.m, _nnz(m)) == (3, 3, 9)
    assert m.con_nonlinear.all() and m.obj_nonlinear
    assert m.var_type.tolist() == [4, 1, 1]
    assert m.var_lb.tolist() == [1e-3, 0.0, 0.0] and m.var_ub.tolist() == [200.0] * 3
    assert m.con_lb.tolist() == [10.0, -3.0, -12.0] and np.all(np.isinf(m.con_ub))
    x = np.array([0.7, 3.0, 5.0])
    x0, x1, x2 = x
    want = [math.sqrt(x0) + x1 + 2 * x2,
            0.240038406144983 * x1 ** 2 + 0.255036980362153 * x0 - x2,
            x2 ** 2 - 1.0 / (x0 ** 3 * math.sqrt(x0)) - 4 * x1]
    for i in range(3):
        v, g = row_value(m, i, x)
        assert abs(v - want[i]) <= 1e-12 * max(1.0, abs(want[i]))
        # gradient against central differences
        for j in range(3):
            h = 1e-6
            e = np.zeros(3)
            e[j] = h
            fd = (row_value(m, i, x + e)[0] - row_value(m, i, x - e)[0]) / (2 * h)
            assert abs(g[j] - fd) <= 1e-5 * max(1.0, abs(fd))
    f, _ = objective_value(m, x)
    assert abs(f - ((x1 - 3) ** 2 + (x2 - 2) ** 2 + (x0 + 4) ** 2)) <= 1e-12


@pytest.mark.skipif(not os.path.exists(COLOR), reason='color_lab2_4x0.nl needs /root/reference')
def test_color_lab2_binary_format_header():
    m = read_nl(COLOR)
    assert (m.n, m.m, _nnz(m)) == (300, 61, 360)
    assert int(np.sum(m.var_type == 0)) == 300
    assert np.all(m.con_lb == m.con_ub) and not m.con_nonlinear.any()
    assert m.obj_nonlinear


def test_nvs08_oa_instance_and_validity():
    """Config 1: the committed OA-LP is the builder's output from the file,
    and every row over-estimates its nonlinear row body on the root box (so
    the LP is a relaxation of nvs08): at random points x of the box, the
    linearised row's activity >= the true body minus the row's tangent /
    secant error sign (checked as row_oa(x) >= body(x))."""
    m = read_nl(os.path.join(NL, 'nvs08.nl'))
    p = nvs08_oa(m)
    ref = LinProblem.load(os.path.join(INST, 'nvs08_oa.npz'))
    for k in ('rowptr', 'colidx', 'val', 'rlo', 'rhi', 'vlb', 'vub', 'vtype', 'obj'):
        assert np.array_equal(getattr(p, k), getattr(ref, k)), k
    A = p.dense()
    rng = np.random.default_rng(1)
    X = np.column_stack([np.exp(rng.uniform(math.log(1e-3), math.log(200), 4000)),
                         rng.integers(0, 201, 4000), rng.integers(0, 201, 4000)])
    # row r of the LP bounds row `src[r]` of nvs08 (or the objective, -1)
    src = [0] * 4 + [1] + [2] * 4 + [-1] * 8
    for r, i in enumerate(src):
        for x in X[:400]:
            if i >= 0:
                body = row_value(m, i, x)[0]
                # row: a.x >= rlo  <=>  a.x - rlo + lo_i over-estimates body
                est = float(A[r, :3] @ x) - p.rlo[r] + m.con_lb[i]
                assert est >= body - 1e-9 * max(1.0, abs(body))
            else:
                f = objective_value(m, x)[0]
                # eta >= rlo - a[:3].x is a tangent plane: below f
                assert p.rlo[r] - float(A[r, :3] @ x) <= f + 1e-9 * max(1.0, f)


def test_nvs08_oa_milp_bounds_the_minlp_optimum():
    import oracle
    p = LinProblem.load(os.path.join(INST, 'nvs08_oa.npz'))
    st, v = oracle.highs_milp(p)
    assert st == 0 and v <= 23.4497 + 1e-4      # MINLPLib nvs08 optimum 23.44972
    st, lp = oracle.highs(p)
    assert st == 0 and lp <= v + 1e-9
