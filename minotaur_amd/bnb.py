"""Batched branch-and-bound drivers over the engine's tree step
(mgpu_bnb_*, minotaur_amd/csrc/bnb.cpp).

``solve`` runs one tree to completion on one GPU.  ``solve_distributed``
is the node-sharded multi-GPU form (MpiBranchAndBound analogue):
every rank runs the same deterministic first rounds, the open nodes are
then dealt round-robin (rank r keeps nodes r, r + P, ...;
MpiBranchAndBound.cpp:142-188), each rank searches its share depth-first,
and the incumbent is all-reduced (MIN, RCCL) after every round; the run
ends when every rank's pool is empty (all-reduce MAX of the open counts).
"""
from __future__ import annotations

import math
import time


def solve(ctx, batch=4096, capacity=None, max_rounds=10**9, incumbent=math.inf,
          root_lb=None, root_ub=None, order=0, warm=0, brancher=0, growth=0):
    """Tree search on the loaded LinProblem: returns (obj, x, stats, seconds).
    order 0 depth-first / 1 best-first; warm 0 root basis / 1 parent basis
    (mgpu_bnb_config); brancher 0 MaxVio / 1 reliability (mgpu_bnb_brancher);
    growth > 0: rounds of at most nodes-so-far // growth (mgpu_bnb_growth)."""
    cap = capacity or 64 * batch
    t0 = time.perf_counter()
    ctx.bnb_config(order, warm)
    ctx.bnb_brancher(brancher)
    ctx.bnb_growth(growth)
    ctx.bnb_init(cap, root_lb, root_ub, incumbent)
    st = None
    for _ in range(max_rounds):
        st = ctx.bnb_round(batch)
        if st.open == 0:
            break
    obj, x = ctx.bnb_best()
    return obj, x, st, time.perf_counter() - t0


def checkpoint(ctx, root_lb=None, root_ub=None) -> bytes:
    """The open pool as Minotaur Serializer records (Serializer::writeNode,
    src/base/Serializer.cpp:26-112; runtime.serialize_nodes): every open node
    exported (mgpu_bnb_export), written with id = its position and lb = its
    bound against the root box (default: the loaded problem's bounds), then
    put back (mgpu_bnb_import; re-imported nodes warm-start from the root
    basis, as any import).  The incumbent is not part of the format (the
    reference sends it separately too): take it from ctx.bnb_best()."""
    from minotaur_amd import runtime
    p = ctx.problem
    rl = p.vlb if root_lb is None else root_lb
    ru = p.vub if root_ub is None else root_ub
    k, _ = ctx.bnb_count()
    lb, ub, nlb, depth = ctx.bnb_export(k)
    data = runtime.serialize_nodes(rl, ru, lb, ub, nlb)
    if len(nlb):
        ctx.bnb_import(lb, ub, nlb, depth)
    return data


def restore(ctx, data, capacity, root_lb=None, root_ub=None, incumbent=math.inf):
    """A tree from checkpoint() bytes, or any stream of the reference's
    Serializer::writeNode records (DeSerializer::readNode, :130-191): the
    pool initialised on the root box, the root replaced by the records' nodes
    (their depth is not in the format: 0).  The caller has set the search
    order, warm mode and brancher (bnb_config / bnb_brancher) as for bnb_init;
    bnb_round continues the search."""
    import numpy as np
    from minotaur_amd import runtime
    p = ctx.problem
    rl = p.vlb if root_lb is None else root_lb
    ru = p.vub if root_ub is None else root_ub
    _, nlb, lb, ub = runtime.deserialize_nodes(data, rl, ru)
    ctx.bnb_init(capacity, rl, ru, incumbent)
    k, _ = ctx.bnb_count()
    ctx.bnb_export(k)                        # the fresh root
    if len(nlb):
        ctx.bnb_import(lb, ub, nlb, np.zeros(len(nlb), dtype=np.int32))


def solve_distributed(ctx, batch, rank, world, allreduce_min=None, allreduce_max=None,
                      capacity=None, max_rounds=10**9, shard_at=None, order=0, warm=0,
                      comm=None, lb_every=0, brancher=0, trace=None, growth=0):
    """Node-sharded tree search.  Every rank runs the same deterministic
    rounds until the pool holds at least ``shard_at`` (default 4 * world)
    open nodes, then keeps nodes i = rank (mod world) (mgpu_bnb_shard) and
    searches its share.  After every round ONE collective carries the
    incumbent (MIN) and the largest open count (the stop test): ``comm``
    (minotaur_amd.dist.Comm over RCCL / gloo) packs both into one all-reduce;
    without it the two callables allreduce_min / allreduce_max(float) ->
    float are used.  With ``comm`` and lb_every > 0, every lb_every rounds
    (and whenever some rank ran out of nodes while others hold more than a
    batch) the open nodes are rebalanced across ranks by their bounds
    (dist.rebalance: MpiBranchAndBound::LoadBalance_).  A rank whose round
    fails makes every rank raise in the same round (the error rides the
    round's all-reduce).  Returns (incumbent, x or None, stats, rounds, mine)
    where mine = {nodes, lps, pivots, pruned, sb_lps, sb_pivots, moved,
    lb_log: per rebalance the bounds picked and received} evaluated
    by this rank, the shared first rounds counted on rank 0 only (so sums
    over ranks are exact).  ``trace`` (a list) receives (perf_counter time,
    all-reduced incumbent) after every round."""
    from . import dist as mdist
    cap = capacity or 64 * batch
    shard_at = shard_at or 4 * world
    ctx.bnb_config(order, warm)
    ctx.bnb_brancher(brancher)
    ctx.bnb_growth(growth)
    ctx.bnb_init(cap, None, None, math.inf)
    inc = math.inf
    sharded = world == 1
    st = None
    rounds = 0
    moved = 0
    shared = (0, 0, 0, 0, 0, 0)
    lb_log = []
    while rounds < max_rounds:
        err, exc = 0, None
        try:
            st = ctx.bnb_round(batch, inc)
        except Exception as e:              # reported to every rank below
            if comm is None or world == 1:
                raise
            err, exc = 1, e
        rounds += 1
        open_now = st.open if not err else 0
        if not err and not sharded and (open_now >= shard_at or open_now == 0):
            shared = (st.nodes, st.lps, st.pivots, st.pruned, st.sb_lps,
                      st.sb_pivots)                           # identical on every rank
            open_now = ctx.bnb_shard(rank, world)
            sharded = True
        if comm is not None:
            inc_r = st.incumbent if st is not None and not err else math.inf
            inc, most, least, failed = comm.round_reduce(inc_r, open_now, err)
            if failed:
                raise exc if exc is not None else RuntimeError(
                    'solve_distributed: a peer rank failed in round %d' % rounds)
            if trace is not None:
                trace.append((time.perf_counter(), inc))
            if most == 0.0:
                break
            # the trigger uses only all-reduced values: every rank agrees
            if sharded and world > 1 and lb_every > 0 and (
                    rounds % lb_every == 0 or (least == 0 and most > batch)):
                open_now, k, picked, got = mdist.rebalance(ctx, comm, batch)
                moved += k
                lb_log.append((picked.tolist(), got.tolist()))
        else:
            inc = allreduce_min(st.incumbent)
            if trace is not None:
                trace.append((time.perf_counter(), inc))
            if allreduce_max(float(open_now)) == 0.0:
                break
    obj, x = ctx.bnb_best()
    sub = shared if rank != 0 else (0, 0, 0, 0, 0, 0)
    mine = {k: v - w for k, v, w in zip(('nodes', 'lps', 'pivots', 'pruned', 'sb_lps',
                                         'sb_pivots'),
                                        (st.nodes, st.lps, st.pivots, st.pruned, st.sb_lps,
                                         st.sb_pivots), sub)}
    mine['moved'] = moved
    mine['lb_log'] = lb_log
    return inc, (x if obj == inc else None), st, rounds, mine
