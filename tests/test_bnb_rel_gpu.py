"""GPU: batched reliability branching in the batched tree (mgpu_bnb_brancher
1; ReliabilityBrancher.cpp, the reference's default brancher): strong
branching from each node's optimal basis (K3 batch, iteration limit 25),
pseudocosts, pruning and one-sided bound changes by the brancher.

Bar: the GPU tree equals the CPU restatement (oracle/bnb.py, brancher 1)
round for round: rounds, nodes, decision counts, strong-branching LP counts,
nodes pruned / modified by the brancher; the optimum is HiGHS' MILP optimum
(1e-6) and the same bit for bit as the restatement's."""
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
