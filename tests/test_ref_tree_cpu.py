"""CPU: the tree-level CPU baseline (bench.py tree_cpu_baseline) -- the
reference's own BranchAndBound + LinearHandler with CpuLPEngine, an LPEngine
over the C restatement of the dual simplex (oracle/ref/CpuLPEngine.cpp,
integ_bnb_tree_cpu) -- proves the HiGHS optimum on the reference-tree
instances with both branchers, and the bench's bounded run honours the
reference's time_limit.  Skipped where the integration library is absent."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from minotaur_amd.problem import LinProblem, knapsack_oa, random_mkp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
LIB = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')
P = ctypes.c_void_p


@pytest.fixture(scope='module')
def integ():
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    from minotaur_amd import runtime
    runtime.load_library()
    lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_bnb_tree_cpu.argtypes = [ctypes.c_int] * 4 + [P] * 9 + [ctypes.c_double] * 2 + \
        [P, P]
    return lib


def cpu_tree(lib, p, brancher=0, guided=1, time_limit=0.0):
    def _p(a):
        return a.ctypes.data_as(P)
    res = np.zeros(3)
    cnt = np.zeros(6, dtype=np.int64)
    lib.integ_bnb_tree_cpu(brancher, guided, p.n, p.m, _p(p.rowptr), _p(p.colidx), _p(p.val),
                           _p(p.rlo), _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub), _p(p.obj),
                           float(p.obj_const), float(time_limit), _p(res), _p(cnt))
    return {"ub": res[0], "seconds": res[2], "processed": int(cnt[0]), "created": int(cnt[1]),
            "lps": int(cnt[2]), "sb_lps": int(cnt[3])}


def _cases():
    return {
        'nvs08_oa': LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances',
                                                 'nvs08_oa.npz')),
        'knapsack_oa': knapsack_oa(),
        'mkp-12-2': random_mkp(1, 12, 2),
        'mkp-18-3': random_mkp(2, 18, 3),
        'mkp-24-4': random_mkp(3, 24, 4),
    }


@pytest.mark.parametrize('brancher', [0, 1])
@pytest.mark.parametrize('name', list(_cases()))
def test_cpu_reference_tree_proves_highs_optimum(integ, name, brancher):
    p = _cases()[name]
    r = cpu_tree(integ, p, brancher)
    hs, hobj = oracle.highs_milp(p)
    assert hs == 0 and abs(r["ub"] - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert r["processed"] >= 1 and r["lps"] >= 1   # (FBBT prunes some nodes before their LP)
    assert (r["sb_lps"] > 0) == (brancher == 1 and r["processed"] > 1)


def test_cpu_reference_tree_time_limit(integ):
    """The bench's bounded sample: a tree far larger than the limit stops
    at it (BabOptions time_limit, read in the BranchAndBound constructor)."""
    p = random_mkp(1, 60, 8)
    r = cpu_tree(integ, p, 0, 1, time_limit=0.5)
    # the limit is read between nodes; the upper bound only shows the tree
    # stopped (loose: a loaded host, e.g. pytest -n, stretches one node)
    assert 0.45 <= r["seconds"] <= 4.0 and r["processed"] > 100


def test_growth_caps_each_round():
    """mgpu_bnb_growth restated (oracle/bnb.py): with div 2 every round
    evaluates at most max(1, nodes so far // 2) nodes, and the tree still
    proves HiGHS' optimum."""
    from bnb import CpuBnbContext
    p = random_mkp(2, 18, 3)
    hs, hobj = oracle.highs_milp(p)
    c = CpuBnbContext(p)
    c.bnb_config(1, 1)
    c.bnb_brancher(1)
    c.bnb_growth(2)
    c.bnb_init(1 << 14)
    before = 0
    while True:
        st = c.bnb_round(4096)
        if st.open == 0 and st.last_batch == 0:
            break
        assert st.last_batch <= max(1, before // 2)
        before = st.nodes
        if st.open == 0:
            break
    assert abs(c.inc - hobj) <= 1e-6 * max(1.0, abs(hobj))
