"""GPU: squares in the batched glob tree (VERDICT r05 "next" #5): the
separation loop of QuadHandler::separate (QuadHandler.cpp:1658-1689) on the
device -- glob_separate (findLinPt_'s golden-section search and addCut_'s
test per node and square, the tangent into the square's next free slot of
the node's record), the flagged nodes re-solved by K3R + K3 with their new
rows, merged and decided again until no node adds a cut -- equals the CPU
restatement (oracle/glob_tree.py) round for round: nodes, decisions,
branchings, LP solves and pivots (re-solves included), tangent cuts,
re-solves, open nodes, incumbent bits and point; and its optimum equals the
reference's own glob tree on HipLPEngine (integ_glob_tree3)."""
import math

import numpy as np
import pytest

from minotaur_amd import glob as mglob
from minotaur_amd.quad import random_qcqp
from test_glob_squares_cpu import SLOTS, SQ_CASES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize('batch', [1, 16, 256])
@pytest.mark.parametrize('case', SQ_CASES)
def test_glob_squares_match_cpu_restatement(ctx, case, batch):
    from glob_tree import CpuGlobContext
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True)
    mglob.setup(ctx, qp, SLOTS)
    cpu = CpuGlobContext(qp, tan_slots=SLOTS)
    ctx.glob_init(1 << 15)
    cpu.glob_init(1 << 15)
    for _ in range(200):
        sg, sc = ctx.glob_round(batch), cpu.glob_round(batch)
        assert (sg.rounds, sg.nodes, list(sg.ndec), sg.br_int, sg.br_cont, sg.lps, sg.pivots,
                sg.cuts, sg.resolves, sg.open) == \
            (sc.rounds, sc.nodes, list(sc.ndec), sc.br_int, sc.br_cont, sc.lps, sc.pivots,
             sc.cuts, sc.resolves, sc.open)
        assert sg.incumbent == sc.incumbent or (math.isinf(sg.incumbent) and
                                                math.isinf(sc.incumbent))
        if sg.open == 0:
            break
    assert sg.open == 0
    og, xg = ctx.glob_best()
    oc, xc = cpu.glob_best()
    assert og == oc and np.array_equal(xg, xc)


def test_glob_squares_optimum_equals_reference_tree(ctx):
    import os
    from test_simplex_cuts_cpu import LIB, glob_tree3, load_integ
    if not os.path.exists(LIB):
        pytest.skip("integration library not built")
    from minotaur_amd import runtime
    runtime.load_library()
    integ = load_integ()
    cuts = 0
    for seed, nv0, ncon in SQ_CASES:
        qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True)
        ub, cnt, _ = glob_tree3(integ, qp, 1, 0)      # the reference's tree, HipLPEngine
        obj, x, st, _ = mglob.solve(ctx, qp, batch=64, capacity=1 << 15, tan_slots=SLOTS)
        print(f"seed {seed}: reference {ub:.17g} ({cnt[0]} nodes, {cnt[7]} separation rows); "
              f"batched {obj:.17g} ({st.nodes} nodes, {st.cuts} cuts, {st.resolves} re-solves)")
        assert cnt[3] == 0 and st.open == 0 and st.ndec[5] == 0
        assert abs(obj - ub) <= 1e-6 * max(1.0, abs(ub)), (seed, obj, ub)
        cuts += st.cuts
    assert cuts > 0
