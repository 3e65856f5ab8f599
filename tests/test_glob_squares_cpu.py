"""CPU: squares in the batched glob tree -- the separation loop of
QuadHandler::separate (QuadHandler.cpp:1658-1689: findLinPt_ :238-285,
addCut_ / addTangent_ :805-840; PCBProcessor.cpp:267-280 re-solves the node
after a cut) restated in oracle/glob_tree.py (VERDICT r05 "next" #5).

On QCQPs with squares y = x^2 (random_qcqp(..., squares=True)), the CPU
restatement of the batched tree with tangent slots proves the optimum of the
reference's OWN glob tree (integ_glob_tree3: Glob::createBab_'s objects
compiled from /root/reference, CpuLPEngine), on the instances where neither
tree closes a node at NoCandToBranch (no NLP engine, QuadHandler.cpp:
356-420); the separation does act (cuts, re-solves).  The GPU tree equals
this restatement round for round (tests/test_glob_squares_gpu.py)."""
import math
import os

import pytest

from minotaur_amd.quad import random_qcqp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
LIB = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')

# (seed, nv0, ncon), squares=True: no NoCandToBranch closure in the
# reference's tree (Glob's defaults) nor in the batched one at batch 1..256
SQ_CASES = [(3, 5, 3), (12, 5, 3), (14, 5, 3), (33, 5, 3), (21, 6, 4), (29, 6, 4), (32, 6, 4),
            (33, 6, 4)]
SLOTS = 8


@pytest.fixture(scope='module')
def integ():
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    from test_simplex_cuts_cpu import load_integ
    return load_integ()


def run_cpu_tree(qp, batch, slots=SLOTS):
    from glob_tree import CpuGlobContext
    cpu = CpuGlobContext(qp, tan_slots=slots)
    cpu.glob_init(1 << 16)
    st = None
    for _ in range(100000):
        st = cpu.glob_round(batch)
        if st.open == 0:
            break
    obj, x = cpu.glob_best()
    return obj, x, st


@pytest.mark.parametrize('case', SQ_CASES)
def test_squares_restatement_proves_the_reference_optimum(integ, case):
    from test_simplex_cuts_cpu import glob_tree3
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True)
    assert qp.nsq > 0
    ub, cnt, _ = glob_tree3(integ, qp, 1, -1)
    assert cnt[3] == 0 and math.isfinite(ub)
    for batch in (1, 64):
        obj, x, st = run_cpu_tree(qp, batch)
        assert st.open == 0 and st.ndec[5] == 0
        assert abs(obj - ub) <= 1e-6 * max(1.0, abs(ub)), (batch, obj, ub)


def test_separation_acts():
    cuts = resolves = 0
    for seed, nv0, ncon in SQ_CASES:
        _, _, st = run_cpu_tree(random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True), 16)
        cuts += st.cuts
        resolves += st.resolves
    assert cuts >= 50 and resolves >= 30, (cuts, resolves)


def test_without_slots_squares_close_nodes():
    """Without the separation loop a point below y = x^2 has no branching
    candidate (QuadHandler branches only above the curve): such trees close
    nodes at NoCandToBranch, which the tangent slots remove."""
    closed = 0
    for seed, nv0, ncon in SQ_CASES:
        qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True)
        _, _, st = run_cpu_tree(qp, 16, slots=0)
        closed += st.ndec[5]
    assert closed > 0
