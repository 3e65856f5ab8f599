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
    out[rank] = (inc, rounds, mine['nodes'], mine['moved'])
    dist.destroy_process_group()


@pytest.mark.parametrize('order', [0, 1])
def test_rebalanced_sharded_tree_search(order):
    """MpiBranchAndBound::LoadBalance_ semantics over gloo: the split after
    the shared rounds leaves rank 1 without nodes; the periodic rebalance
    (all-gather of open counts, common plan, nodes exported, sent, imported)
    gives it work, both ranks evaluate nodes, and the run still proves the
    HiGHS optimum with one packed all-reduce per round."""
    import oracle
    from minotaur_amd.problem import random_mkp
    hs, hobj = oracle.highs_milp(random_mkp(2, 18, 3))
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_lb_worker, args=(world, _free_port(), out, order), nprocs=world, join=True)
    (i0, r0, m0, mv0), (i1, r1, m1, mv1) = out[0], out[1]
    assert i0 == i1 and abs(i0 - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert r0 == r1
    assert mv0 == mv1 > 0            # the plan is global: same count on every rank
    assert m0 > 0 and m1 > 0         # rank 1 got work only through migration


def test_balance_plan():
    from minotaur_amd.dist import balance_plan
    assert balance_plan([10, 0], 2) == [(0, 1, 5)]
    plan = balance_plan([7, 0, 3, 10], 4)
    after = [7, 0, 3, 10]
    for s, d, k in plan:
        after[s] -= k
        after[d] += k
    assert sorted(after) == [5, 5, 5, 5] and sum(k for _, _, k in plan) == 7
    assert balance_plan([4, 4, 4], 3) == []
