"""CPU: the glob tree restatement (oracle/glob_tree.py, CpuGlobContext) at
batch 1 with the reference's order IS the reference's own glob tree, node for
node -- the pin behind tests/test_glob_pin_gpu.py (VERDICT r05 "next" #6).

Reference side (oracle/_ref/libminotaur_hip_integ.so, integ_glob_tree3 on
CpuLPEngine, device -1): Glob::createBab_'s objects compiled from
/root/reference -- BranchAndBound with tree_search bfs, PCBProcessor,
NodeIncRelaxer (parent-basis warm starts; the problem's and relaxation's mods
replayed, SimpleTransformer's flags), MaxVioBrancher, IntVarHandler /
LinearHandler / QuadHandler.

Restatement side: glob_config(order 2, warm 1, qt 0, lin, obbt), batch 1.
lin 0 pairs with the reference's LinearHandler without node presolve; lin 1
with its real LinearHandler, whose presolveNode (simplePresolve on the node's
relaxation rows) runs at every node as Glob sets pres_freq 1 (Glob.cpp:404).
obbt 1 turns on the reference's root OBBT (the OBBT option, on in Glob;
QuadHandler::postSolveRootNode with CpuLPEngine as bte_) and the
restatement's (obbt_chained, the rows rewritten, the root re-solved when its
point leaves the tightened relaxation); the bound LPs are counted on both
sides.  brancher 1 is Glob's default brancher relstronger (StrongBrancher::
reliabilitySetup(20, 50, 5), Glob.cpp:171-181) on both sides: strong-
branching children with getBrMod's rows and every handler's node presolve,
LPs chained through the engine with 50 pivots at most, verdicts, pseudocosts
and updateAfterSolve; there every main-engine solve's pivots are compared.
Seeds are every seed of a fixed range (no selection).  Bar: nodes processed
and created, LP solves, closures, the incumbent's bits, the branching sequence (variable
and its LP value, 1e-9) and each node LP's pivot count and value (1e-9)."""
import ctypes
import math
import os

import numpy as np
import pytest

from minotaur_amd.quad import random_qcqp

PIN_CASES = [(s, 6, 4) for s in range(0, 16)] + [(s, 8, 5) for s in range(0, 12)] + \
    [(s, 10, 6) for s in range(0, 4)]


@pytest.fixture(scope='module')
def integ():
    from test_simplex_cuts_cpu import LIB, load_integ
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    lib = load_integ()
    P = ctypes.c_void_p
    lib.integ_last_branch_log.argtypes = [ctypes.c_int, P, P]
    lib.integ_last_solve_log.argtypes = [ctypes.c_int, P, P, P]
    return lib


def _logs(integ):
    k = integ.integ_last_branch_log(0, None, None)
    bv, bx = np.zeros(k, np.int32), np.zeros(k)
    integ.integ_last_branch_log(k, bv.ctypes.data, bx.ctypes.data)
    n = integ.integ_last_solve_log(0, None, None, None)
    ls, lv, li = np.zeros(n, np.int32), np.zeros(n), np.zeros(n, np.int32)
    integ.integ_last_solve_log(n, ls.ctypes.data, lv.ctypes.data, li.ctypes.data)
    return (bv, bx), (ls, lv, li)


# (lin, obbt, brancher): brancher 0 MaxVio, 1 Glob's relstronger; Glob's
# configuration is (1, 1, 1)
CONFIGS = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (1, 0, 1), (1, 1, 1)]


def ref_opts(lin, obbt, brancher=0):
    """integ_glob_tree3 bits: bfs (1), LinearHandler without node presolve
    (2) unless lin, root OBBT (8) with obbt, StrongBrancher with
    reliabilitySetup(20, 50, 5) (16) with brancher 1."""
    return 1 | (0 if lin else 2) | (8 if obbt else 0) | (16 if brancher else 0)


@pytest.mark.parametrize('config', CONFIGS)
@pytest.mark.parametrize('case', PIN_CASES)
def test_restated_glob_tree_is_the_reference_tree(integ, case, config):
    lin, obbt, brancher = config
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
    from glob_tree import CpuGlobContext
    from test_simplex_cuts_cpu import glob_tree3
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    ub, cnt, _ = glob_tree3(integ, qp, ref_opts(lin, obbt, brancher), -1, 1)   # pres_freq 1
    (bv, bx), (ls, lv, li) = _logs(integ)
    c = CpuGlobContext(qp)
    c.glob_config(2, 1, 0, lin, obbt)
    c.glob_brancher(brancher)
    c.glob_init(1 << 16)
    for _ in range(20000):
        st = c.glob_round(1)
        if st.open == 0:
            break
    obj, _ = c.glob_best()
    assert st.open == 0
    assert (st.nodes, 1 + 2 * int(st.ndec[0]), st.lps, int(st.ndec[5]), st.obbt_lps) == \
        (int(cnt[0]), int(cnt[1]), int(cnt[2]), int(cnt[3]), int(cnt[5]))
    assert obj == ub or (math.isinf(obj) and math.isinf(ub))
    if brancher:
        # the StrongBrancher's LPs are main-engine solves too: compare the
        # whole solve sequence (no branch log from the reference's brancher)
        assert [r[2] for r in c.lplog] == li.tolist()
        return
    mb = np.array([v for v, _ in c.brlog], np.int32)
    mx = np.array([x for _, x in c.brlog])
    assert np.array_equal(mb, bv)
    assert np.allclose(mx, bx, rtol=0, atol=1e-9 * max(1.0, np.abs(bx).max(initial=0.0)))
    assert len(c.lplog) == len(li)
    assert [r[2] for r in c.lplog] == li.tolist()
    fin = np.isfinite(lv) & (np.abs(lv) < 1e20)
    mv = np.array([r[1] for r in c.lplog])
    assert np.allclose(mv[fin], lv[fin], rtol=0, atol=1e-9 * max(1.0, np.abs(lv[fin]).max(initial=0.0)))
