"""CPU, world_size 2 over gloo: the multi-GPU semantics of bench.py /
minotaur_amd.dist — disjoint per-rank node shards, incumbent all-reduce MIN,
stop-flag OR, statistics SUM — with the node processing done by the CPU
oracles as stand-ins for the GPU kernels (this test exercises the
collectives, not the kernels)."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import oracle
    from minotaur_amd import dist as mdist
    from minotaur_amd.problem import LinProblem, random_boxes
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'knapsack9.npz'))
    r, w, _ = mdist.env_ranks()
    assert (r, w) == (rank, world)
    LB, UB = random_boxes(p, 64, mdist.shard_seed(7, rank))
    f = oracle.linear_fbbt(p, LB, UB)
    keep = f.infeas == 0
    _, _, _, _, _, ws = oracle.dual_simplex_root(p)
    st, obj, it, x = oracle.dual_simplex(p, f.lb[keep], f.ub[keep], ws, want_x=True)
    frac = np.abs(x - np.floor(x + 0.5))[:, :9].max(axis=1) > 1e-6
    cand = np.where((st == 0) & ~frac, obj, math.inf)
    local_best = float(cand.min()) if cand.size else math.inf
    best = mdist.allreduce_incumbent(torch.tensor([local_best], dtype=torch.float64))
    stop = mdist.allreduce_stop(torch.tensor([1 if rank == 1 else 0], dtype=torch.int32))
    cnt = mdist.allreduce_sum(torch.tensor([float(keep.sum()), 64.0], dtype=torch.float64))
    allb = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allb, torch.tensor([local_best], dtype=torch.float64))
    out[rank] = (float(best.item()), int(stop.item()), cnt.tolist(),
                 [float(t.item()) for t in allb], LB[:4].tobytes())
    dist.destroy_process_group()


def test_two_rank_incumbent_and_stats():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    b0, s0, c0, allb0, lb0 = out[0]
    b1, s1, c1, allb1, lb1 = out[1]
    assert b0 == b1 == min(allb0)           # MIN over ranks, identical everywhere
    assert s0 == s1 == 1                    # OR of stop flags
    assert c0 == c1 and c0[1] == 128.0      # SUM of counters
    assert lb0 != lb1                       # disjoint shards (different seeds)


def test_round_robin_deal_covers_all():
    from minotaur_amd.dist import deal_round_robin
    items = sorted(sum((deal_round_robin(10, r, 4) for r in range(4)), []))
    assert items == list(range(10))


def _bnb_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from bnb import CpuBnbContext
    from minotaur_amd import bnb
    from minotaur_amd import dist as mdist
    from minotaur_amd.problem import random_mkp
    p = random_mkp(2, 16, 3)
    ctx = CpuBnbContext(p)

    def amin(v):
        return float(mdist.allreduce_incumbent(torch.tensor([v], dtype=torch.float64)).item())

    def amax(v):
        return float(mdist.allreduce_max(torch.tensor([v], dtype=torch.float64)).item())

    inc, x, st, rounds, mine = bnb.solve_distributed(ctx, 8, rank, world, amin, amax,
                                                     capacity=1 << 14)
    out[rank] = (inc, rounds, mine['nodes'], st.nodes)
    dist.destroy_process_group()


def test_two_rank_sharded_tree_search():
    """bnb.solve_distributed over gloo with the CPU restatement of the tree
    step: both ranks prove the HiGHS optimum, stop in the same round, and
    split the work."""
    import oracle
    from minotaur_amd.problem import random_mkp
    hs, hobj = oracle.highs_milp(random_mkp(2, 16, 3))
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bnb_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (i0, r0, m0, n0), (i1, r1, m1, n1) = out[0], out[1]
    assert i0 == i1 and abs(i0 - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert r0 == r1
    assert m0 > 0 and m1 > 0


def test_cpu_tree_step_matches_highs():
    import oracle
    from bnb import CpuBnbContext
    from minotaur_amd import bnb
    from minotaur_amd.problem import knapsack_oa, random_mkp
    for p in (knapsack_oa(), random_mkp(3, 14, 2)):
        hs, hobj = oracle.highs_milp(p)
        obj, x, st, _ = bnb.solve(CpuBnbContext(p), batch=16, capacity=1 << 14)
        assert st.open == 0 and abs(obj - hobj) <= 1e-6 * max(1.0, abs(hobj))


def _lb_worker(rank, world, port, out, order):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from bnb import CpuBnbContext
    from minotaur_amd import bnb
    from minotaur_amd.dist import Comm
    from minotaur_amd.problem import random_mkp

    class Skewed(CpuBnbContext):
        """An intentionally imbalanced split: rank 0 keeps every open node."""

        def bnb_shard(self, r, w):
            if r != 0:
                self.pool = [] if self.order == 0 else [None] * len(self.pool)
            self.tot.open = sum(nd is not None for nd in self.pool)
            return self.tot.open

    p = random_mkp(2, 18, 3)
    ctx = Skewed(p)
    inc, x, st, rounds, mine = bnb.solve_distributed(ctx, 8, rank, world, capacity=1 << 14,
                                                     order=order, comm=Comm(rank, world),
                                                     lb_every=3)
    out[rank] = (inc, rounds, mine['nodes'], mine['moved'], mine['lb_log'])
    dist.destroy_process_group()


def _expected_receipts(picks, world):
    """LoadBalance_'s deal restated in plain Python (MpiBranchAndBound.cpp:
    111-188): all picked bounds in (bound, owner, local) order, the i-th to
    rank i mod world; per rank the bounds it receives from other ranks, in
    deal order."""
    infos = sorted((lb, r, t) for r in range(world) for t, lb in enumerate(picks[r]))
    got = [[] for _ in range(world)]
    for i, (lb, r, t) in enumerate(infos):
        if lb == math.inf:
            break
        if i % world != r:
            got[i % world].append(lb)
    return got


@pytest.mark.parametrize('order', [0, 1])
def test_rebalanced_sharded_tree_search(order):
    """MpiBranchAndBound::LoadBalance_ semantics over gloo: the split after
    the shared rounds leaves rank 1 without nodes; the periodic bound-aware
    rebalance (pick, all-gather of bounds and pool room, common deal, one
    all-to-all of node rows, import in deal order) gives it work, both ranks
    evaluate nodes, and the run still proves the HiGHS optimum with one
    packed all-reduce per round.  Every rebalance moved exactly the nodes the
    reference's deal names: the bounds each rank received are those of the
    deal positions i with i mod 2 = rank owned by the other rank -- at the
    first one (rank 1 empty) the odd-positioned best bounds of rank 0."""
    import oracle
    from minotaur_amd.problem import random_mkp
    hs, hobj = oracle.highs_milp(random_mkp(2, 18, 3))
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_lb_worker, args=(world, _free_port(), out, order), nprocs=world, join=True)
    (i0, r0, m0, mv0, log0), (i1, r1, m1, mv1, log1) = out[0], out[1]
    assert i0 == i1 and abs(i0 - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert r0 == r1
    assert mv0 == mv1 > 0            # the plan is global: same count on every rank
    assert m0 > 0 and m1 > 0         # rank 1 got work only through migration
    assert len(log0) == len(log1) > 0
    assert len(log1[0][0]) == 0 and len(log1[0][1]) > 0
    assert log1[0][1] == sorted(log0[0][0])[1::2]
    for (p0, g0), (p1, g1) in zip(log0, log1):
        e0, e1 = _expected_receipts([p0, p1], world)
        assert g0 == e0 and g1 == e1


def test_lb_deal():
    """lb_deal on a hand-made gather: stable (bound, owner, local) order,
    round-robin receivers, +inf padding dropped."""
    from minotaur_amd.dist import lb_deal
    inf = math.inf
    g = torch.tensor([3.0, 1.0, inf,      # rank 0 picks
                      1.0, 2.0, 0.5])     # rank 1 picks
    owner, local, recv = lb_deal(g, 2, 3)
    assert owner.tolist() == [1, 0, 1, 1, 0]
    assert local.tolist() == [2, 1, 0, 1, 0]
    assert recv.tolist() == [0, 1, 0, 1, 0]


def test_cpu_pick_export_import_roundtrip():
    """The CPU restatement's pick / export_rows / import_rows: best-first
    picks ascend by bound, exported rows leave the pool and come back into
    the lowest free slots (imports reuse holes before growing the
    high-water mark); depth-first keeps the order of the nodes left."""
    import oracle
    from bnb import CpuBnbContext
    from minotaur_amd.problem import random_mkp
    p = random_mkp(2, 18, 3)
    hs, hobj = oracle.highs_milp(p)
    for order in (0, 1):
        ctx = CpuBnbContext(p)
        ctx.bnb_config(order, 0)
        ctx.bnb_brancher(0)
        ctx.bnb_init(1 << 12)
        for _ in range(4):
            st = ctx.bnb_round(8)
        n_open, spare = ctx.bnb_count()
        assert n_open == st.open and spare == (1 << 12) - n_open
        hw = len(ctx.pool)
        lbs = ctx.bnb_pick(6)
        if order == 1:
            assert list(lbs) == sorted(lbs)
        before = [nd for nd in ctx.pool if nd is not None]
        rows = ctx.bnb_export_rows([1, 3, 4])
        assert rows.shape == (3, 2 * p.n + 2)
        assert [float(v) for v in rows[:, 2 * p.n]] == [lbs[1], lbs[3], lbs[4]]
        assert ctx.bnb_count()[0] == n_open - 3
        gone = {id(before_nd) for before_nd in before} - {id(nd) for nd in ctx.pool}
        assert len(gone) == 3
        if order == 0:   # the others keep their order
            assert [id(nd) for nd in ctx.pool] == [id(nd) for nd in before if id(nd) not in gone]
        ctx.bnb_import_rows(rows)
        assert ctx.bnb_count()[0] == n_open
        assert len(ctx.pool) == hw          # best-first: the holes were reused
        while st.open:                      # the tree still proves the optimum
            st = ctx.bnb_round(8)
        assert abs(ctx.inc - hobj) <= 1e-6 * max(1.0, abs(hobj))


@pytest.mark.parametrize("world,S", [(1, 5), (2, 3), (3, 50), (8, 400)])
def test_engine_lb_deal_equals_restatement(world, S):
    """mgpu_lb_deal (the deal inside mgpu_bnb_rebalance, host code of
    libmgpu: no device needed) equals dist.lb_deal -- the restatement of
    LoadBalance_'s deal the gloo tests check -- on gathers with ties,
    -0.0 / +0.0, -inf and +inf padding."""
    from minotaur_amd import runtime
    from minotaur_amd.dist import lb_deal
    rng = np.random.default_rng(world * 1000 + S)
    g = rng.integers(-3, 6, size=(world, S)).astype(np.float64)   # many ties
    g[rng.random((world, S)) < 0.1] = -0.0
    g[rng.random((world, S)) < 0.05] = -math.inf
    for r in range(world):                     # each rank's picks, then padding
        k = int(rng.integers(0, S + 1))
        g[r, k:] = math.inf
    o1, l1, r1 = runtime.lb_deal(world, S, g.reshape(-1))
    o2, l2, r2 = lb_deal(torch.from_numpy(g.reshape(-1)), world, S)
    assert o1.tolist() == o2.tolist()
    assert l1.tolist() == l2.tolist()
    assert r1.tolist() == r2.tolist()


def test_bench_pool_rows_decode_equals_restatement():
    """bench.py's CPU baseline decodes the headline pool's warm-mode-2 rows
    (the parent basis each node carries) vectorised; the result equals the
    restatement's own per-row import (CpuBnbContext.bnb_import_rows)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
    import bench
    from bnb import CpuBnbContext
    from minotaur_amd.problem import random_mkp
    p = random_mkp(2, 18, 3)
    ctx = CpuBnbContext(p, 32)          # product form, 32 etas (K3P's)
    ctx.bnb_config(0, 2)
    ctx.bnb_brancher(0)
    ctx.bnb_init(1 << 12)
    for _ in range(5):
        ctx.bnb_round(8)
    lbs = ctx.bnb_pick(12)
    picked = [ctx.pool[ctx.pick[i]] for i in range(len(lbs))]
    rows = ctx.bnb_export_rows(list(range(len(lbs)))).numpy()
    lb, ub, k_in, path, st = bench.pool_rows_decode(p, rows)
    assert any(int(k) > 0 for k in k_in)
    for t, nd in enumerate(picked):
        assert np.array_equal(lb[t], nd.lb) and np.array_equal(ub[t], nd.ub)
        if nd.path is None or int(nd.path[0]) == 0:
            assert k_in[t] == 0
            continue
        k, pv, sv = nd.path
        assert k_in[t] == k
        assert np.array_equal(path[t, :k], np.asarray(pv, dtype=np.uint32)[:k])
        assert np.array_equal(st[t], np.asarray(sv, dtype=np.int8) & 3)
