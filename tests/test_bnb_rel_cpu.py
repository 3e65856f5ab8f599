"""CPU: the restatement of batched reliability branching (oracle/bnb.py,
brancher 1) proves the HiGHS MILP optimum; batch 1 is the reference's
sequential ReliabilityBrancher."""
import math

import pytest

import oracle
from bnb import CpuBnbContext
from minotaur_amd import bnb
from minotaur_amd.problem import knapsack_oa, random_mkp, random_problem


@pytest.mark.parametrize('batch', [1, 8])
@pytest.mark.parametrize('p', [knapsack_oa(), random_mkp(1, 12, 2), random_mkp(2, 20, 3),
                               random_problem(2)], ids=lambda p: p.name)
def test_rel_restatement_matches_highs(p, batch):
    hs, hobj = oracle.highs_milp(p)
    o, x, st, _ = bnb.solve(CpuBnbContext(p), batch=batch, capacity=1 << 15, brancher=1)
    assert st.open == 0
    if hs == 2:
        assert o == math.inf
    else:
        assert abs(o - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert st.nodes == sum(st.ndec)
    assert st.sb_lps > 0
