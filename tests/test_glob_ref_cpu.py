"""CPU: the glob tree's CPU restatement (oracle/glob_tree.py, which the GPU
tree equals round for round, tests/test_glob_gpu.py) against the reference's
OWN glob tree (integ_glob_tree: Glob::createBab_'s BranchAndBound,
PCBProcessor, NodeIncRelaxer, MaxVioBrancher, IntVarHandler, LinearHandler,
QuadHandler compiled from /root/reference, on CpuLPEngine, the C
restatement of the dual simplex).  Same instances and bar as
tests/test_glob_ref_gpu.py: the same optimum, no node left to an NLP call."""
import ctypes
import math
import os

import numpy as np
import pytest

from minotaur_amd.quad import random_qcqp
from test_glob_ref_gpu import ALIGNED, CASES

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
LIB = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')
P = ctypes.c_void_p


@pytest.fixture(scope='module')
def integ():
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_glob_tree2.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     P, P]
    return lib


CPU_CASES = [(c, 1, False) for c in CASES] + [(c, b[-1], True) for c, b in ALIGNED]


@pytest.mark.parametrize('case,batch,aligned', CPU_CASES)
def test_glob_restatement_optimum_equals_reference_tree(integ, case, batch, aligned):
    from glob_tree import CpuGlobContext
    from test_glob_ref_gpu import ref_glob_tree
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    res, cnt = ref_glob_tree(integ, qp, aligned, device=-1)
    ub, proc, closed = res[0], int(cnt[0]), int(cnt[3])
    cpu = CpuGlobContext(qp)
    cpu.glob_init(1 << 16)
    for _ in range(100000):
        st = cpu.glob_round(batch)
        if st.open == 0:
            break
    obj, x = cpu.glob_best()
    assert st.open == 0 and closed == 0 and st.ndec[5] == 0
    assert math.isfinite(ub) and proc >= 5
    assert abs(obj - ub) <= 1e-6 * max(1.0, abs(ub)), (obj, ub)
