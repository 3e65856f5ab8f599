"""CPU: the restatement of the batched spatial branch-and-bound (oracle/
glob_tree.py, the checker of mgpu_glob_round) on bilinear QCQPs.  The
reference's own glob solver cannot run here (it needs an NLP engine for
PCBProcessor's fixNodeErr and its cut loop), so its incumbents are checked
against the QCQP itself: integral, feasible for every original constraint,
objective equal to the relaxation value, and -- on trees that never had to
close a node without a branching candidate (decision 5, where the reference
would call its NLP engine) -- no worse than the best of a multistart local
search (SLSQP over every integer assignment)."""
import itertools
import math

import numpy as np
import pytest

from minotaur_amd.quad import random_qcqp

CASES = [(0, 5, 3), (1, 6, 4), (1, 8, 5), (3, 6, 4), (3, 8, 5), (4, 8, 5), (5, 6, 4)]


def _funcs(qp):
    out = []
    for c in range(qp.ncon + (1 if qp.has_obj else 0)):
        lin = [(int(qp.lvar[t]), float(qp.lval[t])) for t in range(qp.lptr[c], qp.lptr[c + 1])]
        quad = [(int(qp.qv1[t]), int(qp.qv2[t]), float(qp.qval[t]))
                for t in range(qp.qptr[c], qp.qptr[c + 1])]
        out.append((lin, quad))
    return out


def _ev(f, x):
    lin, quad = f
    return sum(a * x[j] for j, a in lin) + sum(a * x[i] * x[j] for i, j, a in quad)


def _local_best(qp, starts=3, seed=0):
    from scipy.optimize import minimize
    rng = np.random.default_rng(seed)
    n, fs = qp.nv0, _funcs(qp)
    lb, ub = qp.vlb[:n], qp.vub[:n]
    ints = [j for j in range(n) if qp.vtype[j] in (0, 1)]
    cons = []
    for c in range(qp.ncon):
        if np.isfinite(qp.cub[c]):
            cons.append({'type': 'ineq', 'fun': (lambda x, c=c: qp.cub[c] - _ev(fs[c], x))})
        if np.isfinite(qp.clb[c]):
            cons.append({'type': 'ineq', 'fun': (lambda x, c=c: _ev(fs[c], x) - qp.clb[c])})
    best = math.inf
    for assign in itertools.product(*[range(int(lb[j]), int(ub[j]) + 1) for j in ints]):
        lo, hi = lb.copy(), ub.copy()
        for j, v in zip(ints, assign):
            lo[j] = hi[j] = v
        for _ in range(starts):
            r = minimize(lambda x: _ev(fs[qp.ncon], x) + qp.obj_const, lo + (hi - lo) * rng.random(n),
                         bounds=list(zip(lo, hi)), constraints=cons, method='SLSQP',
                         options={'maxiter': 300, 'ftol': 1e-12})
            if r.success and all(
                    (not np.isfinite(qp.cub[c]) or _ev(fs[c], r.x) <= qp.cub[c] + 1e-6) and
                    (not np.isfinite(qp.clb[c]) or _ev(fs[c], r.x) >= qp.clb[c] - 1e-6)
                    for c in range(qp.ncon)):
                best = min(best, float(r.fun))
    return best


def _run(qp, batch, rounds=400):
    from glob_tree import CpuGlobContext
    ctx = CpuGlobContext(qp)
    ctx.glob_init(1 << 16)
    st = None
    for _ in range(rounds):
        st = ctx.glob_round(batch)
        if st.open == 0:
            break
    return ctx, st


@pytest.mark.parametrize('seed,nv0,ncon', CASES)
def test_cpu_glob_tree_incumbent(seed, nv0, ncon):
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    assert qp.nsq == 0
    ctx, st = _run(qp, 64)
    assert st.open == 0
    assert st.nodes == sum(st.ndec) and st.ndec[4] == 0
    inc, x = ctx.glob_best()
    assert math.isfinite(inc)
    fs = _funcs(qp)
    ints = np.isin(qp.vtype[:qp.nv0], (0, 1))
    assert np.all(np.abs(x[:qp.nv0][ints] - np.round(x[:qp.nv0][ints])) <= 1e-6)
    for c in range(qp.ncon):
        act = _ev(fs[c], x)
        assert act <= qp.cub[c] + 1e-5 * max(1.0, abs(qp.cub[c]))
        assert act >= qp.clb[c] - 1e-5 * max(1.0, abs(qp.clb[c]))
    true_obj = _ev(fs[qp.ncon], x) + qp.obj_const
    assert abs(true_obj - inc) <= 1e-5 * max(1.0, abs(inc))
    if st.ndec[5] == 0:
        best = _local_best(qp)
        assert inc <= best + 1e-4 * max(1.0, abs(best))


def test_cpu_glob_tree_batch_independent_optimum():
    """Batch 1 and batch 64 trees close on the same incumbent (different
    trees: the round shares its incumbent) when no node closes without a
    candidate."""
    qp = random_qcqp(3, nv0=8, ncon=5, squares=False)
    a, sa = _run(qp, 1, rounds=5000)
    b, sb = _run(qp, 64)
    assert sa.open == 0 and sb.open == 0 and sa.ndec[5] == sb.ndec[5] == 0
    assert abs(a.inc - b.inc) <= 1e-6 * max(1.0, abs(a.inc))
