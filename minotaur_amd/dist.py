"""Multi-GPU semantics of the batched B&B path (one process per GPU).

Mirrors the collectives of MpiBranchAndBound (src/base/MpiBranchAndBound.cpp)
that touch the hot path.  Two carriers with one interface:

* ``NativeComm``: a ctypes client of the engine's own collectives
  (mgpu_comm_* / mgpu_round_reduce / mgpu_bnb_rebalance in libmgpu, RCCL over
  xGMI, or a host transport) -- what a C++ host shaped like MpiBranchAndBound
  calls; the bench and the trees on GPUs use it;
* ``Comm``: torch.distributed (gloo on CPU), for the CPU restatement's
  multi-process tests (oracle contexts have no engine).

The collectives:

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

import numpy as np
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


MIN_NODES_PER_RANK = 50   # MpiBranchAndBound.cpp:80


def lb_deal(world_lbs, world, per_rank):
    """MpiBranchAndBound::LoadBalance_'s deal (:111-188) on a tensor of the
    all-gathered bounds [world * per_rank] (rank-major, +inf padding): the
    picked nodes in ascending (bound, owner, local index) order -- a stable
    sort of the rank-major vector; the reference's std::sort leaves ties
    unordered -- the i-th one dealt to rank i mod world, stopping at the
    first +inf (:137-148).  Returns (owner, local, receiver) tensors in that
    order (on world_lbs' device)."""
    import math as _m
    order = torch.sort(world_lbs, stable=True).indices
    nfin = int((world_lbs != _m.inf).sum().item())
    order = order[:nfin]
    i = torch.arange(nfin, device=world_lbs.device)
    return order // per_rank, order % per_rank, i % world


class Comm:
    """The per-round exchange of the node-sharded tree on torch.distributed
    (RCCL over xGMI with device tensors, gloo with CPU tensors):

    * ``round_reduce(inc, open, err)``: ONE all-reduce MIN of the packed
      [incumbent, -open, open, -err] -> (global incumbent, max and min open
      count over ranks, any rank failed): the incumbent MIN of :387-389 /
      :197-208, the stop test of :85 and the idle-rank test of the load
      balancer in one collective per round; a rank whose round failed makes
      every rank stop together instead of leaving its peers blocked;
    * ``allgather_vec``: one f64 vector per rank (the Allgather of :107);
    * ``all_to_all_rows``: node rows between all ranks in one collective
      (the per-node MPI_Send / MPI_Recv of :159-185)."""

    def __init__(self, rank, world, device=None):
        self.rank, self.world = rank, world
        self.device = device if device is not None else torch.device('cpu')
        # gloo moves host tensors only (the N>1 rehearsal on one GPU box):
        # device tensors are staged through the host there; RCCL takes them
        # as they are
        if active() and dist.get_backend() == 'gloo':
            self.device = torch.device('cpu')

    def allreduce(self, vals, op):
        """SUM / MIN / MAX (runtime.OP_*) of a small f64 vector -> numpy."""
        t = torch.as_tensor(np.array(vals, dtype=np.float64).reshape(-1)).to(self.device)
        if active():
            dist.all_reduce(t, op=(dist.ReduceOp.SUM, dist.ReduceOp.MIN, dist.ReduceOp.MAX)[op])
        return t.cpu().numpy()

    def barrier(self):
        if active():
            dist.barrier()

    def round_reduce(self, inc, n_open, err=0):
        if not active():   # one rank: nothing to reduce (no device round trip per round)
            return float(inc), float(n_open), float(n_open), float(err)
        t = torch.tensor([float(inc), -float(n_open), float(n_open), -float(err)],
                         dtype=torch.float64, device=self.device)
        if active():
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        v = t.tolist()
        return v[0], -v[1], v[2], -v[3]

    def allgather_vec(self, vec):
        t = torch.as_tensor(vec, dtype=torch.float64).to(self.device)
        if not active():
            return t.view(1, -1)
        out = torch.empty((self.world, t.numel()), dtype=torch.float64, device=self.device)
        if self.device.type == 'cpu':   # gloo
            dist.all_gather(list(out.unbind(0)), t)
        else:
            dist.all_gather_into_tensor(out, t)
        return out

    def all_to_all_rows(self, rows, send_counts, recv_counts, width):
        inp = rows.to(self.device).contiguous()
        out = torch.empty((int(sum(recv_counts)), width), dtype=torch.float64,
                          device=self.device)
        if active():
            dist.all_to_all_single(out, inp, [int(c) for c in recv_counts],
                                   [int(c) for c in send_counts])
        else:
            out.copy_(inp)
        return out


class NativeComm:
    """The round collectives inside the engine (include/mgpu.h mgpu_comm_*):
    ``transport`` 'rccl' -- an RCCL communicator over the ranks' GPUs (rank 0
    makes the unique id, the bootstrap process group hands it to the others;
    torch.distributed is only the launcher's rendezvous here) -- or 'host' --
    the engine calls back into torch.distributed (gloo) on host buffers (the
    one-GPU rehearsal of N ranks, where RCCL refuses a shared device).  A
    world of one needs no communicator: every collective is the identity.
    Load balancing is ONE engine call (mgpu_bnb_rebalance)."""

    def __init__(self, ctx, rank, world, transport='rccl'):
        self.ctx, self.rank, self.world, self.transport = ctx, rank, world, transport
        if world == 1:
            return
        if transport == 'rccl':
            from .runtime import comm_unique_id
            obj = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.comm_init(rank, world, obj[0])
        elif transport == 'host':
            ops = (dist.ReduceOp.SUM, dist.ReduceOp.MIN, dist.ReduceOp.MAX)

            def ar(v, op):
                t = torch.from_numpy(v)          # shares the engine's buffer
                dist.all_reduce(t, op=ops[op])

            def ag(send, recv):
                out = torch.from_numpy(recv)
                dist.all_gather(list(out.unbind(0)), torch.from_numpy(send.copy()))

            def a2a(send, sc, recv, rc):
                out = torch.from_numpy(recv) if recv.size else torch.empty((0, recv.shape[1]),
                                                                           dtype=torch.float64)
                dist.all_to_all_single(out, torch.from_numpy(send.copy()),
                                       [int(c) for c in rc], [int(c) for c in sc])
            ctx.comm_init_host(rank, world, ar, ag, a2a)
        else:
            raise ValueError(f"NativeComm: unknown transport {transport!r}")

    def allreduce(self, vals, op):
        return self.ctx.allreduce(vals, op)

    def barrier(self):
        self.ctx.allreduce([0.0], 0)

    def round_reduce(self, inc, n_open, err=0):
        return self.ctx.round_reduce(inc, n_open, err)

    def allgather_vec(self, vec):
        return torch.from_numpy(self.ctx.allgather(vec))

    def all_to_all_rows(self, rows, send_counts, recv_counts, width):
        return self.ctx.alltoall_rows(rows, send_counts, recv_counts)


def make_comm(ctx, rank, world, device=None):
    """The carrier of the round collectives for a GPU run: the engine's own
    (NativeComm; MGPU_COMM=rccl (default) or host) or torch.distributed's
    (MGPU_COMM=torch, Comm).  The one-GPU rehearsal (MGPU_BENCH_REHEARSAL=1)
    uses the host transport: RCCL refuses ranks that share a device."""
    mode = os.environ.get('MGPU_COMM', 'host' if os.environ.get('MGPU_BENCH_REHEARSAL') == '1'
                          else 'rccl')
    if mode == 'torch':
        return Comm(rank, world, device)
    return NativeComm(ctx, rank, world, mode)


def rebalance(ctx, comm, batch=0):
    """One bound-aware load-balancing step (MpiBranchAndBound::LoadBalance_,
    :78-195) on the tree pool of ``ctx``:

    1. every rank picks its next S candidates (mgpu_bnb_pick) -- the
       reference pops 50 P per rank; a round of the batched tree takes
       ``batch`` nodes, so S = max(50 P, batch): the globally best P x batch
       nodes are what the ranks evaluate next;
    2. one all-gather of the S bounds (+inf padded) and the pool room of
       every rank;
    3. every rank computes the same deal (lb_deal): the i-th best goes to
       rank i mod P; nodes whose owner is their receiver stay in place;
    4. a plan that would overflow some receiver's pool fails on EVERY rank
       (same data, same check), so no rank is left blocked in a collective;
    5. the moving nodes leave as device rows (mgpu_bnb_export_dev; in warm
       mode 2 each row carries its node's basis), cross in
       ONE all-to-all (RCCL over xGMI on MI355X) and are imported in deal
       order (mgpu_bnb_import_dev).

    Returns (this rank's open count afterwards, nodes moved globally, the
    bounds this rank picked, the bounds of the nodes it received in deal
    order)."""
    P, r = comm.world, comm.rank
    S = max(MIN_NODES_PER_RANK * P, int(batch))
    if isinstance(comm, NativeComm):      # the whole step inside the engine
        return ctx.bnb_rebalance(S)
    lbs = ctx.bnb_pick(S)
    n_open, spare = ctx.bnb_count()
    vec = torch.full((S + 1,), float('inf'), dtype=torch.float64)
    vec[:len(lbs)] = torch.from_numpy(lbs)
    vec[S] = float(spare)
    g = comm.allgather_vec(vec)
    owner, local, recv = lb_deal(g[:, :S].reshape(-1), P, S)
    moved = owner != recv
    gain = (torch.bincount(recv[moved], minlength=P) -
            torch.bincount(owner[moved], minlength=P)).to(torch.float64)
    if bool((gain > g[:, S]).any().item()):
        raise RuntimeError('rebalance: the deal would overflow a node pool '
                           f'(gain {gain.tolist()}, room {g[:, S].tolist()})')
    send = moved & (owner == r)
    dst = recv[send]
    perm = torch.sort(dst, stable=True).indices            # grouped by receiver, deal order
    idx = local[send][perm].to(torch.int32).cpu().numpy()
    send_counts = torch.bincount(dst, minlength=P).tolist()
    got = moved & (recv == r)
    src = owner[got]
    recv_counts = torch.bincount(src, minlength=P).tolist()
    rows = ctx.bnb_export_rows(idx)
    width = ctx.bnb_row_width()
    out = comm.all_to_all_rows(rows, send_counts, recv_counts, width)
    # the all-to-all delivers rows grouped by sender; import them in deal order
    a2a = torch.sort(src, stable=True).indices               # a2a row -> deal position
    inv = torch.empty_like(a2a)
    inv[a2a] = torch.arange(a2a.numel(), device=a2a.device)
    ordered = out[inv.to(out.device)] if out.shape[0] else out
    ctx.bnb_import_rows(ordered)
    n_open = n_open - len(idx) + int(ordered.shape[0])
    nb = 2 * ctx.problem.n   # the node bound's column
    got_lbs = ordered[:, nb].cpu().numpy() if ordered.shape[0] else np.empty(0)
    return n_open, int(moved.sum().item()), lbs, got_lbs
