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
