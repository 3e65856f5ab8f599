"""GPU: Glob's default brancher relstronger (mgpu_glob_brancher 1,
StrongBrancher with reliabilitySetup(20, 50, 5)) in a glob tree WITH squares:
the separation loop (QuadHandler::separate's tangents, re-solves) between a
node's LP and its strong branching, with the linear node presolve and root
OBBT as Glob runs them.  The device path equals the CPU restatement
(oracle/glob_tree.py _process_rs) round for round -- nodes, decisions,
branchings, LPs and pivots, strong-branching and OBBT LPs, tangent cuts,
re-solves, open nodes, incumbent bits -- and solve for solve (every
main-engine LP's status and pivots, its value to 1e-9), on the squares
cases of tests/test_glob_squares_cpu.py.  (With squares the reference's
own tree keeps every cut in one relaxation while the batched tree keeps
them per node path, DESIGN §8, so the node-for-node pin against the
reference stays the bilinear one, tests/test_glob_pin_gpu.py.)"""
import math

import numpy as np
import pytest

from minotaur_amd.quad import random_qcqp
from test_glob_squares_cpu import SLOTS, SQ_CASES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize('obbt', [0, 1])
@pytest.mark.parametrize('case', SQ_CASES)
def test_relstronger_with_squares_matches_cpu_restatement(ctx, case, obbt):
    from glob_tree import CpuGlobContext
    from minotaur_amd import glob as mglob
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=True)
    mglob.setup(ctx, qp, SLOTS)
    ctx.glob_config(2, 1, 0, 1, obbt)
    ctx.glob_brancher(1)
    cpu = CpuGlobContext(qp, tan_slots=SLOTS)
    cpu.glob_config(2, 1, 0, 1, obbt)
    cpu.glob_brancher(1)
    ctx.glob_init(1 << 15)
    cpu.glob_init(1 << 15)
    key = lambda s: (s.rounds, s.nodes, list(s.ndec), s.br_int, s.br_cont, s.lps, s.pivots,
                     s.sb_lps, s.obbt_lps, s.cuts, s.resolves, s.open)
    for _ in range(5000):
        sg, sc = ctx.glob_round(1), cpu.glob_round(1)
        assert key(sg) == key(sc)
        assert sg.incumbent == sc.incumbent or (math.isinf(sg.incumbent) and
                                                math.isinf(sc.incumbent))
        if sg.open == 0:
            break
    assert sg.open == 0
    og, xg = ctx.glob_best()
    oc, xc = cpu.glob_best()
    assert og == oc or (math.isinf(og) and math.isinf(oc))
    if math.isfinite(og):
        assert np.array_equal(xg, xc)
    gs, gv, gi = ctx.glob_lp_log()
    assert [int(v) for v in gs] == [r[0] for r in cpu.lplog]
    assert [int(v) for v in gi] == [r[2] for r in cpu.lplog]
    cv = np.array([r[1] for r in cpu.lplog])
    fin = np.isfinite(cv)
    assert np.array_equal(fin, np.isfinite(gv))
    assert np.allclose(gv[fin], cv[fin], rtol=0, atol=1e-9 * max(1.0, np.abs(cv[fin]).max(initial=0)))
