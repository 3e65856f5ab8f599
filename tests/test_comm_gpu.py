"""GPU: the engine's round collectives (include/mgpu.h mgpu_comm_*, the
MpiBranchAndBound exchange a C++ host calls through the C ABI).

* world 1 over RCCL (a one-GPU box): every collective is driven through a real
  RCCL communicator -- incumbent MIN, the packed round reduce, all-gather,
  the device-row all-to-all -- and mgpu_bnb_rebalance runs inside a tree
  without changing it;
* world 2 on one GPU over the host transport (RCCL refuses two ranks on one
  device; the engine calls back into gloo): mgpu_bnb_rebalance moves the
  nodes LoadBalance_'s deal assigns (checked against the plain restatement
  of the deal) in warm modes 0 and 2, and the sharded tree proves the HiGHS
  optimum.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch

import oracle
from minotaur_amd import bnb
from minotaur_amd.problem import random_mkp

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context, comm_unique_id
    c = Context(0)
    c.comm_init(0, 1, comm_unique_id())
    yield c
    c.close()


def test_world1_rccl_collectives(ctx):
    from minotaur_amd.runtime import OP_MAX, OP_MIN, OP_SUM
    assert ctx.comm_info() == (0, 1)
    v = [3.5, -math.inf, 7.0, 0.25]
    for op in (OP_SUM, OP_MIN, OP_MAX):
        assert ctx.allreduce(v, op).tolist() == v
    assert ctx.round_reduce(2.5, 17, 0) == (2.5, 17.0, 17.0, 0.0)
    assert ctx.round_reduce(math.inf, 0, 1) == (math.inf, 0.0, 0.0, 1.0)
    g = ctx.allgather(np.arange(5.0))
    assert g.shape == (1, 5) and g[0].tolist() == [0.0, 1.0, 2.0, 3.0, 4.0]
    rows = torch.arange(24, dtype=torch.float64, device='cuda').view(4, 6)
    out = ctx.alltoall_rows(rows, [4], [4])
    torch.cuda.synchronize()
    assert torch.equal(out, rows)


@pytest.mark.parametrize('order,warm', [(0, 0), (1, 0), (0, 2), (1, 2)])
def test_world1_rebalance_keeps_the_tree(ctx, order, warm):
    """At world 1 the deal gives every picked node back to its owner: the
    rebalance reports the picked bounds, moves nothing, and the tree runs on
    round for round like an untouched one."""
    from minotaur_amd.runtime import Context
    p = random_mkp(5, 22, 3)
    hs, hobj = oracle.highs_milp(p)
    ref = Context(0)
    try:
        for c in (ctx, ref):
            c.load(p)
            c.bnb_config(order, warm)
            c.bnb_brancher(0)
            c.bnb_init(1 << 14)
        for _ in range(5):
            sa, sb = ctx.bnb_round(16), ref.bnb_round(16)
        n_open = ctx.bnb_count()[0]
        S = 50
        after, moved, picked, got = ctx.bnb_rebalance(S)
        assert moved == 0 and got.size == 0 and after == ctx.bnb_count()[0]
        assert np.array_equal(picked, ref.bnb_pick(S))
        if order == 0:
            assert after == n_open
        while True:
            sa, sb = ctx.bnb_round(16), ref.bnb_round(16)
            assert (sa.nodes, list(sa.ndec), sa.open, sa.lps, sa.pivots) == \
                (sb.nodes, list(sb.ndec), sb.open, sb.lps, sb.pivots)
            if sa.open == 0:
                break
        assert abs(sa.incumbent - hobj) <= 1e-6 * max(1.0, abs(hobj))
    finally:
        ref.close()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_worker(rank, world, port, out, order, warm):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from minotaur_amd import dist as mdist
    from minotaur_amd.runtime import Context
    try:
        p = random_mkp(6, 26, 3)
        ctx = Context(0)
        comm = mdist.NativeComm(ctx, rank, world, 'host')
        assert ctx.comm_info() == (rank, world)
        r = ctx.round_reduce(10.0 + rank, 5 * rank, rank)
        g = ctx.allgather([float(rank), 2.0 * rank])
        ctx.load(p)
        inc, x, st, rounds, mine = bnb.solve_distributed(
            ctx, 8, rank, world, capacity=1 << 14, order=order, warm=warm, comm=comm,
            lb_every=3)
        tot = ctx.allreduce([float(mine['nodes'])], 0)
        out[rank] = (r, g.tolist(), inc, mine['moved'], mine['lb_log'], float(tot[0]))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('order,warm', [(0, 0), (1, 0), (1, 2)])
def test_world2_host_transport_rebalance(order, warm):
    """Two ranks on device 0, the engine's collectives over its host
    transport (gloo underneath): round reduce and all-gather values, every
    mgpu_bnb_rebalance delivers exactly the nodes LoadBalance_'s deal assigns
    to each rank (the restatement of test_dist_cpu), nodes actually move, and
    the sharded tree proves the HiGHS optimum."""
    import torch.multiprocessing as mp
    from test_dist_cpu import _expected_receipts
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_host_worker, args=(world, _free_port(), out, order, warm), nprocs=world,
             join=True)
    hs, hobj = oracle.highs_milp(random_mkp(6, 26, 3))
    r0, g0, inc0, mv0, log0, tot0 = out[0]
    r1, g1, inc1, mv1, log1, tot1 = out[1]
    assert r0 == r1 == (10.0, 5.0, 0.0, 1.0)
    assert g0 == g1 == [[0.0, 0.0], [1.0, 2.0]]
    assert inc0 == inc1 and abs(inc0 - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert tot0 == tot1 > 0
    assert len(log0) == len(log1) > 0 and mv0 == mv1 > 0
    for (p0, gt0), (p1, gt1) in zip(log0, log1):
        e0, e1 = _expected_receipts([p0, p1], world)
        assert gt0 == e0 and gt1 == e1


def _alloc_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from minotaur_amd import dist as mdist
    from minotaur_amd.runtime import Context, alloc_stats
    try:
        p = random_mkp(6, 26, 3)
        ctx = Context(0)
        mdist.NativeComm(ctx, rank, world, 'host')
        ctx.load(p)
        ctx.bnb_config(1, 2)
        ctx.bnb_brancher(0)
        ctx.bnb_init(1 << 14)
        if rank > 0:
            ctx.bnb_export(1)          # the root belongs to rank 0
        for _ in range(6):
            ctx.bnb_round(8)
        S = 100
        ctx.bnb_rebalance(S)           # sizes the exchange for S
        a1 = alloc_stats()
        moved = [ctx.bnb_rebalance(S)[1] for _ in range(2)]
        a2 = alloc_stats()
        # a warm export / import round trip of equal size allocates nothing
        trips = []
        for _ in range(2):
            got = len(ctx.bnb_pick(S))
            k = min(4, got)
            rows = ctx.bnb_export_rows(np.arange(k))
            ctx.bnb_import_rows(rows)
            torch.cuda.synchronize()
            trips.append(alloc_stats())
        out[rank] = (a1, a2, moved, trips)
        ctx.close()
    finally:
        dist.destroy_process_group()


def test_world2_warm_rebalance_allocates_nothing():
    """after the first mgpu_bnb_rebalance at a pick size S (which
    reserves the exchange's worst case for S: rows sent / received, the
    gather staging, the pool's pack and move workspaces), further rebalances
    at S and equal-size export / import round trips make no device (or
    pinned host) allocation -- what lets bench.py assert a timed multi-GPU
    headline allocation-free."""
    import torch.multiprocessing as mp
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_alloc_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        a1, a2, moved, trips = out[r]
        assert a2 == a1, (r, a1, a2)
        assert trips[1] == trips[0], (r, trips)
