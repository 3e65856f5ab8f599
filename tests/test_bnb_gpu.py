"""GPU: the batched branch-and-bound driver (mgpu_bnb_*, the caller of the
hot path) proves the same MILP optimum as scipy HiGHS (within 1e-6), for any
batch size, returns an integral feasible incumbent, and shards the open
nodes exactly (mgpu_bnb_shard)."""
import math

import numpy as np
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


def _check_solution(p, x, obj):
    assert np.all(x >= p.vlb - 1e-6) and np.all(x <= p.vub + 1e-6)
    ints = np.isin(p.vtype, (0, 1))
    assert np.all(np.abs(x[ints] - np.round(x[ints])) <= 1e-6)
    act = np.zeros(p.m)
    for i in range(p.m):
        s = slice(p.rowptr[i], p.rowptr[i + 1])
        act[i] = np.dot(p.val[s], x[p.colidx[s]])
    tol = 1e-6 * (1 + np.abs(act))
    assert np.all(act >= p.rlo - tol) and np.all(act <= p.rhi + tol)
    assert abs(float(np.dot(p.obj, x)) + p.obj_const - obj) <= 1e-6 * max(1.0, abs(obj))


def _cases():
    return [knapsack_oa(), random_mkp(1, 12, 2), random_mkp(2, 20, 3), random_mkp(3, 24, 4),
            random_problem(2), random_problem(3)]


@pytest.mark.parametrize('batch', [1, 7, 256])
@pytest.mark.parametrize('k', range(6))
def test_bnb_matches_highs_milp(ctx, k, batch):
    p = _cases()[k]
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    obj, x, st, secs = bnb.solve(ctx, batch=batch, capacity=1 << 16, max_rounds=200000)
    assert st.open == 0, 'tree not finished'
    if hs == 2:
        assert obj == math.inf
        return
    assert hs == 0
    assert abs(obj - hobj) <= 1e-6 * max(1.0, abs(hobj))
    _check_solution(p, x, obj)
    assert st.nodes == sum(st.ndec)
    assert st.ndec[4] == 0


def test_bnb_shard_partitions_pool(ctx):
    p = random_mkp(4, 24, 4)
    ctx.load(p)
    counts = []
    for r in range(3):
        ctx.bnb_init(1 << 14)
        st = None
        for _ in range(6):
            st = ctx.bnb_round(8)
        before = st.open
        counts.append(ctx.bnb_shard(r, 3))
    assert sum(counts) == before and max(counts) - min(counts) <= 1


@pytest.mark.parametrize('warm,brancher', [(0, 0), (1, 0), (2, 0), (0, 1), (1, 1)])
def test_bnb_depth_first_shard_matches_cpu(ctx, warm, brancher):
    """Depth-first shard (mgpu_bnb_shard packs the kept nodes): every
    per-slot array moves with its node — parent bases (warm 1), paths
    (warm 2), parent branching data (reliability) — so each rank's search
    after the shard is the CPU restatement's (which shards node objects),
    round for round, and together they prove the HiGHS optimum."""
    from bnb import CpuBnbContext
    from minotaur_amd.runtime import Context
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    other = Context(0)
    try:
        gpu = [ctx, other]
        cpu = [CpuBnbContext(p, ctx.oracle_pfi() if warm != 1 and not brancher else 0)
               for _ in range(2)]
        for c in gpu + cpu:
            if c in gpu:
                c.load(p)
            c.bnb_config(0, warm)
            c.bnb_brancher(brancher)
            c.bnb_init(1 << 15)
        for _ in range(3):
            sg = [c.bnb_round(16) for c in gpu]
            sc = [c.bnb_round(16) for c in cpu]
        for r in range(2):
            assert gpu[r].bnb_shard(r, 2) == cpu[r].bnb_shard(r, 2)
        inc = min(s.incumbent for s in sg)
        while True:
            sg = [c.bnb_round(16, inc) for c in gpu]
            sc = [c.bnb_round(16, inc) for c in cpu]
            for a, b in zip(sg, sc):
                assert (a.rounds, a.nodes, list(a.ndec), a.lps, a.pivots, a.sb_lps) == \
                    (b.rounds, b.nodes, list(b.ndec), b.lps, b.pivots, b.sb_lps)
            inc = min(s.incumbent for s in sg)
            if max(s.open for s in sg) == 0:
                break
        assert abs(inc - hobj) <= 1e-6 * max(1.0, abs(hobj))
    finally:
        other.close()


def test_bnb_two_shards_interleaved(ctx):
    """Two ranks simulated in one process (two contexts, incumbent MIN after
    every round): the sharded search proves the HiGHS optimum."""
    from minotaur_amd.runtime import Context
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    ctxs = [ctx, Context(0)]
    try:
        for c in ctxs:
            c.load(p)
            c.bnb_init(1 << 15)
        inc, sharded, open_ = math.inf, False, [1, 1]
        while True:
            sts = [c.bnb_round(16, inc) for c in ctxs]
            open_ = [s.open for s in sts]
            if not sharded and open_[0] >= 8:
                open_ = [c.bnb_shard(r, 2) for r, c in enumerate(ctxs)]
                sharded = True
            inc = min(s.incumbent for s in sts)
            if max(open_) == 0:
                break
        assert abs(inc - hobj) <= 1e-6 * max(1.0, abs(hobj))
    finally:
        ctxs[1].close()


@pytest.mark.parametrize('batch', [4, 64])
def test_bnb_tree_matches_cpu_restatement(ctx, batch):
    """Same rounds, same decisions: the GPU tree and the CPU restatement of
    the tree step (oracle/bnb.py over the C oracles) evaluate the same number
    of nodes with the same decision counts and find the same incumbent."""
    from bnb import CpuBnbContext
    for p in (knapsack_oa(), random_mkp(6, 16, 3)):
        ctx.load(p)
        og, xg, sg, _ = bnb.solve(ctx, batch=batch, capacity=1 << 15)
        oc, xc, sc, _ = bnb.solve(CpuBnbContext(p, ctx.oracle_pfi()), batch=batch, capacity=1 << 15)
        assert sg.open == sc.open == 0
        assert abs(og - oc) <= 1e-9 * max(1.0, abs(oc))
        assert (sg.rounds, sg.nodes, list(sg.ndec)) == (sc.rounds, sc.nodes, list(sc.ndec))


def test_bnb_k3l_tree_matches_cpu_and_highs(ctx):
    """More rows than a wave has lanes: the batched tree on the knapsack OA
    LP with f = 17 terms, N = 64 (m = 69 -> K3L node LPs) evaluates the same
    tree as the CPU restatement (rounds, nodes, decisions), ends on the same
    incumbent bit for bit (K3L sums like the oracle) and proves the HiGHS
    MILP optimum."""
    from bnb import CpuBnbContext
    p = knapsack_oa(f=17, N=64)
    assert p.m > 64
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    ctx.set_lp_variant(2)   # K3L (auto picks the product-form K3PW for this batch)
    try:
        og, xg, sg, _ = bnb.solve(ctx, batch=512, capacity=1 << 17)
        assert ctx.oracle_pfi() == 0
    finally:
        ctx.set_lp_variant(0)
    oc, xc, sc, _ = bnb.solve(CpuBnbContext(p, 0), batch=512, capacity=1 << 17)
    assert sg.open == sc.open == 0
    assert (sg.rounds, sg.nodes, list(sg.ndec)) == (sc.rounds, sc.nodes, list(sc.ndec))
    assert og == oc
    assert hs == 0 and abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))
    _check_solution(p, xg, og)


@pytest.mark.parametrize('order,warm', [(1, 0), (0, 1), (1, 1), (0, 2), (1, 2)])
@pytest.mark.parametrize('k', range(4))
def test_bnb_search_modes_match_cpu_and_highs(ctx, k, order, warm):
    """Best-first selection (TreeManager bfs: lowest bound first, open nodes
    pruned by the incumbent before evaluation) and parent warm starts
    (NodeIncRelaxer.cpp:146-150: each node LP from its parent's optimal
    basis, K3 / K3L per-node warm starts; warm 2: the same basis kept as its
    pivot path from the root, K3P): the GPU tree is the CPU
    restatement's tree (rounds, nodes, decisions, pruned-open counts) and
    proves the HiGHS MILP optimum."""
    import os
    from bnb import CpuBnbContext
    from minotaur_amd.problem import LinProblem
    cases = [knapsack_oa(), random_mkp(6, 16, 3), random_mkp(1, 30, 4),
             LinProblem.load(os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd',
                                          'instances', 'nvs08_oa.npz'))]
    p = cases[k]
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    og, xg, sg, _ = bnb.solve(ctx, batch=64, capacity=1 << 15, order=order, warm=warm)
    oc, xc, sc, _ = bnb.solve(CpuBnbContext(p, ctx.oracle_pfi()), batch=64, capacity=1 << 15,
                              order=order, warm=warm)
    assert sg.open == sc.open == 0
    assert (sg.rounds, sg.nodes, list(sg.ndec), sg.pruned, sg.lps, sg.pivots) == \
        (sc.rounds, sc.nodes, list(sc.ndec), sc.pruned, sc.lps, sc.pivots)
    assert abs(og - oc) <= 1e-9 * max(1.0, abs(oc))
    assert hs == 0 and abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))
    _check_solution(p, xg, og)


def test_bnb_best_first_k3l_parent_warm(ctx):
    """m > 64 (knapsack OA f = 17, K3L node LPs) with parent warm starts and
    best-first selection: same tree as the CPU restatement, HiGHS optimum."""
    from bnb import CpuBnbContext
    p = knapsack_oa(f=17, N=64)
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    og, xg, sg, _ = bnb.solve(ctx, batch=256, capacity=1 << 16, order=1, warm=1)
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p, ctx.oracle_pfi()), batch=256, capacity=1 << 16,
                             order=1, warm=1)
    assert (sg.rounds, sg.nodes, list(sg.ndec), sg.pruned) == \
        (sc.rounds, sc.nodes, list(sc.ndec), sc.pruned)
    assert og == oc
    assert hs == 0 and abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))


def test_bnb_tls4_lin_tree(ctx):
    """Config 2's own tree: tls4-lin's MILP optimum is 0 (HiGHS proves it at
    its root node); the LP optimum is degenerate and our dual simplex's
    root vertex is fractional, so the batched tree branches (a few hundred to
    a few thousand nodes by search mode) and proves 0, evaluating the same
    tree as the CPU restatement in every mode."""
    import os
    from bnb import CpuBnbContext
    from minotaur_amd.problem import LinProblem
    p = LinProblem.load(os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd',
                                     'instances', 'tls4_lin.npz'))
    hs, hobj = oracle.highs_milp(p)
    assert hs == 0 and hobj == 0.0
    ctx.load(p)
    for order, warm in ((0, 0), (1, 0), (1, 1)):
        og, xg, sg, _ = bnb.solve(ctx, batch=1024, capacity=1 << 14, order=order, warm=warm)
        oc, _, sc, _ = bnb.solve(CpuBnbContext(p, ctx.oracle_pfi()), batch=1024,
                                 capacity=1 << 14, order=order, warm=warm)
        assert sg.open == 0 and abs(og - hobj) <= 1e-9
        assert (sg.rounds, sg.nodes, list(sg.ndec), sg.pruned) == \
            (sc.rounds, sc.nodes, list(sc.ndec), sc.pruned)
        _check_solution(p, xg, og)


@pytest.mark.parametrize('order,warm', [(0, 0), (1, 0), (1, 1), (0, 2), (1, 2)])
def test_bnb_export_import_between_contexts(ctx, order, warm):
    """Node migration (mgpu_bnb_export / mgpu_bnb_import, the node send /
    receive of MpiBranchAndBound::LoadBalance_) between two engine contexts
    in one process: half of context A's open nodes move to context B after
    a few rounds; both trees then run to the end with the incumbent MIN
    exchanged each round and together prove the HiGHS optimum."""
    from minotaur_amd.runtime import Context
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    other = Context(0)
    try:
        ctx.load(p)
        other.load(p)
        for c in (ctx, other):
            c.bnb_config(order, warm)
        ctx.bnb_init(1 << 15)
        other.bnb_init(1 << 15)
        other.bnb_export(1 << 15)           # B starts with an empty pool
        st = None
        for _ in range(4):
            st = ctx.bnb_round(16)
        lb, ub, nlb, dep = ctx.bnb_export(st.open // 2)
        assert len(nlb) == st.open // 2 > 0
        other.bnb_import(lb, ub, nlb, dep)
        inc, open_ = st.incumbent, [1, 1]
        while max(open_) > 0:
            sts = [c.bnb_round(16, inc) for c in (ctx, other)]
            open_ = [s.open for s in sts]
            inc = min(s.incumbent for s in sts)
        assert abs(inc - hobj) <= 1e-6 * max(1.0, abs(hobj))
        assert sts[1].nodes > 0
    finally:
        other.close()


@pytest.mark.parametrize('order,warm', [(0, 0), (1, 0), (1, 1), (0, 2), (1, 2)])
def test_bnb_pick_rows_match_cpu_restatement(ctx, order, warm):
    """The bound-aware migration entry points (mgpu_bnb_pick / export_dev /
    import_dev, LoadBalance_'s pop, send and receive) equal the CPU
    restatement's: the same picked bounds, the same device rows, and after
    the rows went out and came back (into the lowest free slots / on top of
    the stack) the tree still runs round for round like the restatement's
    and proves the HiGHS optimum."""
    from bnb import CpuBnbContext
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    cpu = CpuBnbContext(p, ctx.oracle_pfi())
    for c in (ctx, cpu):
        c.bnb_config(order, warm)
        c.bnb_brancher(0)
        c.bnb_init(1 << 14)
    for _ in range(5):
        sg, sc = ctx.bnb_round(16), cpu.bnb_round(16)
    assert ctx.bnb_count() == cpu.bnb_count()
    lg, lc = ctx.bnb_pick(40), cpu.bnb_pick(40)
    assert len(lg) > 8 and np.array_equal(lg, lc)
    idx = [1, 4, 5, 7, 2]
    rg, rc = ctx.bnb_export_rows(idx), cpu.bnb_export_rows(idx)
    assert np.array_equal(rg.cpu().numpy(), rc.numpy())
    assert ctx.bnb_count() == cpu.bnb_count()
    ctx.bnb_import_rows(rg)
    cpu.bnb_import_rows(rc)
    assert ctx.bnb_count() == cpu.bnb_count()
    while True:
        sg, sc = ctx.bnb_round(16), cpu.bnb_round(16)
        assert (sg.rounds, sg.nodes, list(sg.ndec), sg.open) == \
            (sc.rounds, sc.nodes, list(sc.ndec), sc.open)
        if sg.open == 0:
            break
    assert abs(sg.incumbent - hobj) <= 1e-6 * max(1.0, abs(hobj))


def test_bnb_repeated_migration_near_capacity(ctx):
    """best-first imports reuse free slots below the high-water
    mark, so many export / import cycles on a nearly full pool never run out
    of slots, and the tree still proves the optimum afterwards."""
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    ctx.load(p)
    ctx.bnb_config(1, 0)
    ctx.bnb_brancher(0)
    cap = 2048        # 200 cycles x 64 rows would need 12 800 slots if imports grew the pool
    ctx.bnb_init(cap)
    st = None
    for _ in range(6):
        st = ctx.bnb_round(16)
    for cycle in range(200):
        lbs = ctx.bnb_pick(64)              # (prunes by the incumbent first)
        n_open, spare = ctx.bnb_count()
        k = len(lbs)
        rows = ctx.bnb_export_rows(list(range(k)))
        ctx.bnb_import_rows(rows)
        assert ctx.bnb_count() == (n_open, spare)
    while st.open:
        st = ctx.bnb_round(16)
    assert abs(st.incumbent - hobj) <= 1e-6 * max(1.0, abs(hobj))
