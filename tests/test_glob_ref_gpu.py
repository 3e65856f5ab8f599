"""GPU: the batched spatial branch-and-bound (mgpu_glob_*) against the
reference's OWN glob tree (first step).

Reference side (oracle/_ref/libminotaur_hip_integ.so, integ_glob_tree):
Glob::createBab_'s objects (src/solvers/Glob.cpp:134-220) compiled from
/root/reference -- BranchAndBound, PCBProcessor, NodeIncRelaxer (parent warm
starts), MaxVioBrancher, IntVarHandler, LinearHandler and QuadHandler
(McCormick rows, presolveNode, isFeasible, spatial candidates,
QuadHandler.cpp:473-614, 904-953) -- over the QCQP's auxiliary form, with
HipLPEngine for the LPs (Clp is absent).  Where the reference's
PCBProcessor meets NoCandToBranch it calls QuadHandler::fixNodeErr, which
needs an NLP engine (QuadHandler.cpp:356-420; none in the image): the driver
closes such a node without a solution, as the batched tree does, and counts
it.

Bar: both prove the same optimum, within the trees' 1e-6 relative pruning
tolerance (PCBProcessor.cpp:400-523; measured agreement ~1e-14), on the
instances where neither tree closes a node that way: seven with Glob's
defaults (trees of 7..49 nodes) and seven with the reference configured like
the batched round (node presolve at every node, no LinearHandler presolve
at the nodes; trees of 17..57 nodes).  tests/test_glob_ref_cpu.py pins the CPU restatement
(oracle/glob_tree.py) against the same reference trees on CpuLPEngine.
The node sequences are not compared: the batched tree has no parent warm
starts and no LinearHandler presolve in its round, so the LP
vertices and the branching differ at degenerate nodes.
"""
import ctypes
import math
import os

import numpy as np
import pytest

from minotaur_amd import glob as mglob
from minotaur_amd.quad import random_qcqp

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
LIB = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')
P = ctypes.c_void_p

# bilinear QCQPs (random_qcqp(seed, nv0, ncon, squares=False)) on which
# neither tree meets NoCandToBranch, with the reference's glob defaults
# (LinearHandler node presolve, pres_freq 5); its trees take 7..49 nodes
CASES = [(16, 5, 3), (17, 6, 4), (26, 6, 4), (29, 8, 5), (30, 5, 3), (31, 8, 5), (33, 8, 5)]
# the reference configured like the batched round: node presolve at every
# node (pres_freq 1), no linear FBBT at the nodes; its trees take 17..57
# nodes.  Batches at which the batched tree meets no NoCandToBranch.
ALIGNED = [((3, 8, 5), (1, 64)), ((4, 8, 5), (64,)), ((6, 8, 5), (1, 64)),
           ((8, 6, 4), (64,)), ((8, 8, 5), (1, 64)), ((12, 6, 4), (1, 64)),
           ((12, 8, 5), (1, 64))]


@pytest.fixture(scope='module')
def integ():
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    from minotaur_amd import runtime
    runtime.load_library()
    lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_glob_tree2.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     P, P]
    return lib


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def ref_glob_tree(integ, qp, aligned=False, device=0):
    """integ_glob_tree2 (best-first): Glob's defaults, or aligned with the
    batched round (pres_freq 1, LinearHandler without node presolve)."""
    import oracle
    spec = oracle.qspec(qp)
    res = np.zeros(3)
    cnt = np.zeros(4, dtype=np.int64)
    flags, freq = (2, 1) if aligned else (0, 5)
    assert integ.integ_glob_tree2(device, ctypes.byref(spec), 1, flags, freq,
                                  res.ctypes.data_as(P), cnt.ctypes.data_as(P)) == 0
    return res, cnt


def _check(integ, ctx, seed, nv0, ncon, batch, aligned):
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    (ub, lb, secs), (proc, created, lps, closed) = ref_glob_tree(integ, qp, aligned)
    obj, x, st, _ = mglob.solve(ctx, qp, batch=batch, capacity=1 << 16)
    print(f"seed {seed} nv0 {nv0} ncon {ncon} aligned {int(aligned)}: reference {ub:.17g} "
          f"nodes {proc} lps {lps} ({secs * 1e3:.1f} ms); batched {obj:.17g} nodes {st.nodes}")
    assert st.open == 0
    assert closed == 0 and st.ndec[5] == 0      # no node left to an NLP call
    assert math.isfinite(ub) and proc >= 5
    assert abs(obj - ub) <= 1e-6 * max(1.0, abs(ub)), (seed, obj, ub)
    assert x is not None


@pytest.mark.parametrize('batch', [1, 64])
def test_glob_tree_optimum_equals_reference_tree(integ, ctx, batch):
    for seed, nv0, ncon in CASES:
        _check(integ, ctx, seed, nv0, ncon, batch, False)


def test_glob_tree_optimum_equals_aligned_reference_tree(integ, ctx):
    for (seed, nv0, ncon), batches in ALIGNED:
        for batch in batches:
            _check(integ, ctx, seed, nv0, ncon, batch, True)
