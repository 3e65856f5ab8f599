"""GPU: the batched tree against the reference's OWN BranchAndBound, node for
node.

Reference side (oracle/_ref/libminotaur_hip_integ.so, integ_bnb_tree): the
unchanged BranchAndBound + TreeManager ("bfs" NodeHeap) + PCBProcessor
(pres_freq 1: LinearHandler::presolveNode at every node) + NodeIncRelaxer
(each node from its parent's warm start) + MaxVioBrancher or
ReliabilityBrancher + IntVarHandler
(guided dive on: the reference default), with the reference's own
LinearHandler for FBBT and HipLPEngine for the LPs (Clp is absent).

Batched side (libmgpu): mgpu_bnb_* at batch 1 with order 2 (the reference's
NodeHeap order, lazy pruning, TreeManager's node ids), warm 1 (parent bases,
root LP from the slack basis after its presolve), MaxVio or the batched
reliability brancher.

Bar: the same number of nodes processed and created, the same number of LP
solves, the same optimum bit for bit.  Larger batches run the same rounds
several nodes at a time and still prove the optimum.
"""
import ctypes
import math
import os

import numpy as np
import pytest

import oracle
from minotaur_amd import bnb
from minotaur_amd.problem import LinProblem, knapsack_oa, random_mkp

pytestmark = pytest.mark.gpu
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
    lib.integ_bnb_tree.argtypes = [ctypes.c_int] * 6 + [P] * 9 + [ctypes.c_double, P, P]
    return lib


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _p(a):
    return a.ctypes.data_as(P)


def reference_tree(integ, p, brancher=0, guided=1, hip_fbbt=0):
    res = np.zeros(3)
    cnt = np.zeros(6, dtype=np.int64)
    integ.integ_bnb_tree(0, hip_fbbt, brancher, guided, p.n, p.m, _p(p.rowptr), _p(p.colidx),
                         _p(p.val), _p(p.rlo), _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub),
                         _p(p.obj), float(p.obj_const), _p(res), _p(cnt))
    return {"ub": res[0], "lb": res[1], "seconds": res[2], "processed": int(cnt[0]),
            "created": int(cnt[1]), "lps": int(cnt[2]), "sb_lps": int(cnt[3])}


def batched_tree(ctx, p, batch=1, guided=1, warm=1, brancher=0):
    """A node the brancher modified is solved again inside the same process()
    call in the reference: it is not a processed or created node there."""
    ctx.load(p)
    ctx.bnb_guided_dive(guided)
    try:
        obj, x, st, secs = bnb.solve(ctx, batch=batch, capacity=1 << 18, order=2, warm=warm,
                                     brancher=brancher)
    finally:
        ctx.bnb_guided_dive(1)
    mod = st.sb_modified
    return {"ub": obj, "processed": st.nodes - mod, "created": 1 + 2 * (st.ndec[0] - mod),
            "lps": st.lps + st.sb_lps, "sb_lps": st.sb_lps, "open": st.open, "x": x,
            "seconds": secs, "sb_modified": mod, "sb_pruned": st.sb_pruned}


def _cases():
    return {
        'nvs08_oa': LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances',
                                                 'nvs08_oa.npz')),
        'knapsack_oa': knapsack_oa(),
        'mkp-12-2': random_mkp(1, 12, 2),
        'mkp-18-3': random_mkp(2, 18, 3),
        'mkp-22-3': random_mkp(5, 22, 3),
        'mkp-24-4': random_mkp(3, 24, 4),
    }


@pytest.mark.parametrize('brancher', [0, 1])
@pytest.mark.parametrize('guided', [1, 0])
@pytest.mark.parametrize('name', list(_cases()))
def test_batch1_tree_is_the_reference_tree(integ, ctx, name, guided, brancher):
    """brancher 0 MaxVioBrancher; 1 ReliabilityBrancher (strong-branching LPs
    chained through the engine, stopping at the first verdict; a modified
    node solved again from the last strong-branching basis): the reference's
    lps count every LPEngine::solve call, strong branching included."""
    p = _cases()[name]
    ref = reference_tree(integ, p, guided=guided, brancher=brancher)
    gpu = batched_tree(ctx, p, guided=guided, brancher=brancher)
    assert gpu["open"] == 0
    assert (gpu["processed"], gpu["created"], gpu["lps"], gpu["sb_lps"]) == \
        (ref["processed"], ref["created"], ref["lps"], ref["sb_lps"]), (gpu, ref)
    assert gpu["ub"] == ref["ub"]
    hs, hobj = oracle.highs_milp(p)
    assert hs == 0 and abs(gpu["ub"] - hobj) <= 1e-6 * max(1.0, abs(hobj))


@pytest.mark.parametrize('batch', [4, 64])
def test_reference_order_in_batches_proves_optimum(integ, ctx, batch):
    """Several nodes per round in the reference heap order: same optimum."""
    p = _cases()['mkp-24-4']
    ref = reference_tree(integ, p)
    gpu = batched_tree(ctx, p, batch=batch)
    assert gpu["open"] == 0 and gpu["ub"] == ref["ub"]


def test_gpu_fbbt_handler_same_reference_tree(integ):
    """The reference tree with HipLinearHandler (K1 at B = 1 inside the
    reference) is the same tree as with the reference's own LinearHandler."""
    p = _cases()['mkp-18-3']
    a = reference_tree(integ, p, hip_fbbt=0)
    b = reference_tree(integ, p, hip_fbbt=1)
    assert (a["processed"], a["created"], a["lps"], a["ub"]) == \
        (b["processed"], b["created"], b["lps"], b["ub"])


@pytest.mark.parametrize('brancher', [0, 1])
@pytest.mark.parametrize('name', ['nvs08_oa', 'knapsack_oa', 'mkp-18-3', 'mkp-24-4'])
def test_cpu_baseline_tree_is_the_gpu_engine_tree(integ, name, brancher):
    """bench.py's tree-level CPU baseline runs the same tree as the reference
    with HipLPEngine: CpuLPEngine (the C restatement) and K3 agree LP for LP,
    so BranchAndBound processes and creates the same nodes, solves the same
    LPs (strong branching included) and returns the same incumbent."""
    from test_ref_tree_cpu import cpu_tree
    integ.integ_bnb_tree_cpu.argtypes = [ctypes.c_int] * 4 + [P] * 9 + \
        [ctypes.c_double] * 2 + [P, P]
    p = _cases()[name]
    a = reference_tree(integ, p, brancher=brancher)
    b = cpu_tree(integ, p, brancher)
    assert (a["processed"], a["created"], a["lps"], a["sb_lps"]) == \
        (b["processed"], b["created"], b["lps"], b["sb_lps"]), (a, b)
    assert a["ub"] == b["ub"]
