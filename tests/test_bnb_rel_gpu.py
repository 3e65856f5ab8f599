"""GPU: batched reliability branching in the batched tree (mgpu_bnb_brancher
1; ReliabilityBrancher.cpp, the reference's default brancher): strong
branching from each node's optimal basis (K3 batch, iteration limit 25),
pseudocosts, pruning and one-sided bound changes by the brancher.

Bar: the GPU tree equals the CPU restatement (oracle/bnb.py, brancher 1)
round for round: rounds, nodes, decision counts, strong-branching LP counts,
nodes pruned / modified by the brancher; the optimum is HiGHS' MILP optimum
(1e-6) and the same bit for bit as the restatement's.  The strong-branching
chains run in one K3 launch per round (mgpu_set_sb_chain 1, the default) or
one launch per chain position (0): both equal the restatement."""
import math

import pytest

import oracle
from minotaur_amd import bnb
from minotaur_amd.problem import knapsack_oa, random_mkp, random_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _cases():
    return [knapsack_oa(), random_mkp(1, 12, 2), random_mkp(2, 20, 3), random_mkp(3, 24, 4),
            random_problem(2)]


def _sig(st):
    return (st.rounds, st.nodes, list(st.ndec), st.sb_lps, st.sb_pruned, st.sb_modified)


@pytest.mark.parametrize('warm', [0, 1])
@pytest.mark.parametrize('order', [0, 1])
@pytest.mark.parametrize('batch', [1, 8, 64])
@pytest.mark.parametrize('k', range(5))
def test_rel_tree_matches_cpu_and_highs(ctx, k, batch, order, warm):
    from bnb import CpuBnbContext
    p = _cases()[k]
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    og, xg, sg, _ = bnb.solve(ctx, batch=batch, capacity=1 << 15, order=order, warm=warm,
                              brancher=1)
    oc, xc, sc, _ = bnb.solve(CpuBnbContext(p), batch=batch, capacity=1 << 15, order=order,
                              warm=warm, brancher=1)
    assert sg.open == sc.open == 0
    assert _sig(sg) == _sig(sc)
    assert sg.sb_pivots == sc.sb_pivots
    assert og == oc
    if hs == 2:
        assert og == math.inf
    else:
        assert abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))


def test_rel_tree_smaller_than_maxvio(ctx):
    """Reliability branching is the reference default because it searches
    smaller trees: on mkp n=24 m=4 it evaluates far fewer nodes."""
    p = random_mkp(3, 24, 4)
    ctx.load(p)
    _, _, s0, _ = bnb.solve(ctx, batch=16, capacity=1 << 15, brancher=0)
    _, _, s1, _ = bnb.solve(ctx, batch=16, capacity=1 << 15, brancher=1)
    assert s1.nodes < 0.8 * s0.nodes and s1.sb_lps > 0


def test_rel_tls4_lin_tree(ctx):
    """The config-2 instance: reliability branching proves the HiGHS optimum."""
    import os
    from minotaur_amd.problem import LinProblem
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = LinProblem.load(os.path.join(root, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    og, _, sg, _ = bnb.solve(ctx, batch=4096, capacity=1 << 18, order=1, brancher=1)
    assert sg.open == 0 and hs == 0
    assert abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))


@pytest.mark.parametrize('chain', [1, 0])
@pytest.mark.parametrize('warm', [0, 1])
def test_rel_tree_growth_tls4_oa(ctx, warm, chain):
    """with a fixed batch the round's nodes share one
    pseudocost state and config 2's reliability tree grows to 4.9x the
    reference's.  mgpu_bnb_growth 2 (a round evaluates at most half the
    nodes evaluated so far) keeps it near the reference's own tree: the GPU
    tree equals the CPU restatement round for round, proves HiGHS' optimum,
    and with parent warm starts stays within 1.5x the reference
    BranchAndBound's processed nodes (integ_bnb_tree_cpu, one core)."""
    import os
    from bnb import CpuBnbContext
    from minotaur_amd.problem import LinProblem
    root = os.path.join(os.path.dirname(__file__), '..')
    p = LinProblem.load(os.path.join(root, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    ctx.set_sb_chain(chain)
    try:
        og, _, sg, _ = bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=warm,
                                 brancher=1, growth=2)
    finally:
        ctx.set_sb_chain(1)
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p), batch=131072, capacity=1 << 20, order=1,
                             warm=warm, brancher=1, growth=2)
    assert sg.open == sc.open == 0
    assert _sig(sg) == _sig(sc) and sg.sb_pivots == sc.sb_pivots
    assert og == oc and abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))
    if warm == 1:
        from test_ref_tree_cpu import LIB, cpu_tree
        if os.path.exists(LIB):
            import ctypes
            lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
            lib.integ_bnb_tree_cpu.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 9 + \
                [ctypes.c_double] * 2 + [ctypes.c_void_p] * 2
            ref = cpu_tree(lib, p, 1)
            assert abs(ref["ub"] - hobj) <= 1e-6 * max(1.0, abs(hobj))
            assert sg.nodes <= 1.5 * ref["processed"], (sg.nodes, ref["processed"])
