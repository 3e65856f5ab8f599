"""Multi-GPU semantics of the batched B&B path (one process per GPU).

Mirrors the collectives of MpiBranchAndBound (src/base/MpiBranchAndBound.cpp)
that touch the hot path, on torch.distributed (RCCL over xGMI on MI355X,
gloo on CPU for the tests):

* incumbent: ``MPI_Allreduce(MIN)`` of the upper bound (:387-389) plus the
  eager point-to-point pushes of new incumbents (:197-208, :36-50), folded
  here into ONE all-reduce MIN of a single f64 per batch round;
* stop flags: ``MPI_Allreduce(LOR)`` (:85) -> all-reduce MAX on an int;
* statistics: ``MPI_Gather`` of counters (:417, :442) -> all-reduce SUM.

Node batches are sharded: every rank owns its own open nodes (rank 0 solves
the root and first-level children are dealt round-robin, :142-188); the data
path itself has no collective.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_ranks():
    return (int(os.environ.get('RANK', '0')), int(os.environ.get('WORLD_SIZE', '1')),
            int(os.environ.get('LOCAL_RANK', '0')))


def active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def shard_seed(base: int, rank: int) -> int:
    """Per-rank seed of the synthetic node batch (weak scaling)."""
    return int(base) + int(rank)


def deal_round_robin(n_items: int, rank: int, world: int):
    """Indices of items owned by `rank` when dealt round-robin (the root's
    children distribution of MpiBranchAndBound::LoadBalance_)."""
    return list(range(rank, n_items, world))


def allreduce_incumbent(best: torch.Tensor) -> torch.Tensor:
    """In-place MIN of a 1-element f64 tensor across ranks."""
    if active():
        dist.all_reduce(best, op=dist.ReduceOp.MIN)
    return best


def allreduce_stop(flag: torch.Tensor) -> torch.Tensor:
    """Logical OR of per-rank stop flags (int tensor) across ranks."""
    if active():
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    return flag


def allreduce_sum(t: torch.Tensor) -> torch.Tensor:
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_max(t: torch.Tensor) -> torch.Tensor:
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def balance_plan(counts, world):
    """MpiBranchAndBound::LoadBalance_ (:78-195) made deterministic: from the
    all-gathered open-node counts, the (src, dst, k) transfers that leave
    every rank with floor(T/P) or ceil(T/P) nodes (the first T mod P ranks get
    the extra one), donors and receivers matched in rank order.  Every rank
    computes the same list."""
    total = int(sum(counts))
    target = [total // world + (1 if r < total % world else 0) for r in range(world)]
    give = [(r, int(counts[r]) - target[r]) for r in range(world) if counts[r] > target[r]]
    need = [(r, target[r] - int(counts[r])) for r in range(world) if counts[r] < target[r]]
    plan, i, j = [], 0, 0
    while i < len(give) and j < len(need):
        src, g = give[i]
        dst, d = need[j]
        k = min(g, d)
        plan.append((src, dst, k))
        give[i] = (src, g - k)
        need[j] = (dst, d - k)
        if give[i][1] == 0:
            i += 1
        if need[j][1] == 0:
            j += 1
    return plan


class Comm:
    """The per-round exchange of the node-sharded tree on torch.distributed
    (RCCL over xGMI with device tensors, gloo with CPU tensors):

    * ``round_reduce(inc, open)``: ONE all-reduce MIN of the packed triple
      [incumbent, -open, open] -> (global incumbent, max and min open count
      over ranks): the incumbent MIN of :387-389 / :197-208, the stop test of
      :85 and the idle-rank test of the load balancer in one collective per
      round;
    * ``allgather_counts``: the open-node counts of every rank (the
      Allgather of :107, node counts instead of 50·P lower bounds);
    * ``send_nodes`` / ``recv_nodes``: node boxes, bounds and depths packed
      in one f64 tensor per transfer (Serializer.cpp:26-112 content)."""

    def __init__(self, rank, world, device=None):
        self.rank, self.world = rank, world
        self.device = device if device is not None else torch.device('cpu')

    def round_reduce(self, inc, n_open):
        t = torch.tensor([float(inc), -float(n_open), float(n_open)], dtype=torch.float64,
                         device=self.device)
        if active():
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        v = t.tolist()
        return v[0], -v[1], v[2]

    def allgather_counts(self, n_open):
        t = torch.tensor([float(n_open)], dtype=torch.float64, device=self.device)
        if not active():
            return [int(n_open)]
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [int(o.item()) for o in out]

    def send_nodes(self, dst, lb, ub, nlb, depth):
        k, n = lb.shape
        buf = torch.empty(k * (2 * n + 2), dtype=torch.float64)
        v = buf.view(k, 2 * n + 2)
        v[:, :n] = torch.from_numpy(lb)
        v[:, n:2 * n] = torch.from_numpy(ub)
        v[:, 2 * n] = torch.from_numpy(nlb)
        v[:, 2 * n + 1] = torch.from_numpy(depth.astype('float64'))
        dist.send(buf.to(self.device), dst)

    def recv_nodes(self, src, k, n):
        buf = torch.empty(k * (2 * n + 2), dtype=torch.float64, device=self.device)
        dist.recv(buf, src)
        v = buf.cpu().view(k, 2 * n + 2).numpy()
        return (v[:, :n].copy(), v[:, n:2 * n].copy(), v[:, 2 * n].copy(),
                v[:, 2 * n + 1].astype('int32'))


def rebalance(ctx, comm, n_open, n):
    """One load-balancing step on the tree pool of ``ctx``: all-gather the
    counts, run the common plan, export / send, receive / import.  Returns
    (this rank's open count afterwards, nodes moved globally)."""
    counts = comm.allgather_counts(n_open)
    plan = balance_plan(counts, comm.world)
    for src, dst, k in plan:
        if comm.rank == src:
            lb, ub, nlb, dep = ctx.bnb_export(k)
            assert len(nlb) == k
            comm.send_nodes(dst, lb, ub, nlb, dep)
            n_open -= k
        elif comm.rank == dst:
            lb, ub, nlb, dep = comm.recv_nodes(src, k, n)
            ctx.bnb_import(lb, ub, nlb, dep)
            n_open += k
    return n_open, sum(k for _, _, k in plan)
