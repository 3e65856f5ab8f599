"""Batched spatial branch-and-bound over a QCQP's McCormick relaxation (the
glob path; mgpu_glob_*, minotaur_amd/csrc/glob_runtime.cpp).

The reference's glob solver (src/solvers/Glob.cpp:134-220) runs
BranchAndBound with NodeIncRelaxer, PCBProcessor, the handlers IntVarHandler
/ LinearHandler / QuadHandler of SimpleTransformer and (option
brancher=maxvio) MaxVioBrancher.  Here one round evaluates the top ``batch``
nodes of an HBM stack at once: optionally LinearHandler::presolveNode on the
node's relaxation rows (glob_linear), K2 (QuadHandler::presolveNode, rows
rewritten from the parent's), K3R + K3 (each node's LP with its own rows), the decision,
the squares' separation loop (tangent cuts, re-solve), MaxVio branching,
children pushed.
"""
from __future__ import annotations

import math
import time

from .quad import relaxation_lp


TAN_SLOTS = 8   # tangent-cut rows per square (QuadHandler::separate's cuts)


def setup(ctx, qp, tan_slots=None):
    """Load a QuadProblem for the glob tree: the quadratic problem, the LP
    relaxation at the root box (QuadHandler::relax_'s rows) and the map of
    the per-node rewritten entries; with squares, ``tan_slots`` tangent-cut
    rows per square for the separation loop (default TAN_SLOTS; 0: none).
    Returns (LinProblem, NodeRows)."""
    ctx.load_quad(qp)
    rows0 = ctx.quad_rows()
    S = (TAN_SLOTS if tan_slots is None else int(tan_slots)) if qp.nsq > 0 else 0
    p, nr = relaxation_lp(qp, rows0, S)
    ctx.load(p)
    ctx.set_node_rows(nr)
    return p, nr


def solve(ctx, qp, batch=1024, capacity=None, max_rounds=10**9, incumbent=math.inf,
          loaded=False, tan_slots=None, order=0, warm=0, qt=1, lin=0, obbt=0, brancher=0):
    """Runs the tree until the stack is empty (or max_rounds): returns
    (incumbent, x or None, stats, seconds).  order / warm / qt / lin / obbt:
    mgpu_glob_config (order 2, warm 1 at batch 1: the reference's own glob
    tree node for node; lin 1: LinearHandler's node presolve too; obbt 1:
    root OBBT).  brancher 1: Glob's relstronger (one node per round)."""
    if not loaded:
        setup(ctx, qp, tan_slots)
    cap = capacity or 64 * batch
    t0 = time.perf_counter()
    ctx.glob_config(order, warm, qt, lin, obbt)
    ctx.glob_brancher(brancher)
    ctx.glob_init(cap, incumbent)
    st = None
    for _ in range(max_rounds):
        st = ctx.glob_round(batch)
        if st.open == 0:
            break
    obj, x = ctx.glob_best()
    # a finite objective from an outside incumbent comes without our point
    ok = math.isfinite(obj) and x is not None and not any(math.isnan(v) for v in x)
    return obj, (x if ok else None), st, time.perf_counter() - t0
