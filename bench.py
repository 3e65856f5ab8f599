#!/usr/bin/env python
"""Headline benchmark: batched branch-and-bound tree rounds on MI355X.

BASELINE.json metric: "B&B nodes/sec + relaxations solved/sec at 1/2/4/8
MI355X", quoted on configs[1] ("tls4.nl glob solver, batched FBBT + LP
relaxation on 1 MI355X").  Config 2's instance is tls4.nl itself as a MINLP:
its outer-approximation LP (minotaur_amd/instances/tls4_oa.npz: the four
convex sqrt rows as tangent rows, the 60 linear rows).  One STEP is one round
of the batched tree per GPU, device resident (mgpu_bnb_round):

  select       pop the top B open nodes of the HBM node stack (TreeManager)
  K1 FBBT      LinearHandler::presolveNode      (LinearHandler.cpp:1592-1653)
  K3P LP       OsiLPEngine::solve, root basis   (OsiLPEngine.cpp:571-652)
  decision     PCBProcessor::shouldPrune_ + IntVarHandler::isFeasible +
               MaxVioBrancher's choice
  branch       IntVarHandler::getBranches: both children written to the stack
  incumbent    one packed all-reduce (MIN incumbent, open counts) over ranks
               (MpiBranchAndBound.cpp:387-389)

Nodes pruned by FBBT are not LP-solved (as in PCBProcessor::process), so
relaxations/s <= nodes/s.  The pool starts as the root plus B * N synthetic
boxes (seeded random branching from the root) dealt round-robin
over the N ranks (the root on rank 0; B per rank: weak scaling); later rounds
pop their descendants, and every --lb-every rounds the ranks rebalance their
open nodes by bound (dist.rebalance, inside the timed loop).
Supplementary objects: the round-1/2 fixed batch (tls4-lin), complete trees
from the root, configs 3/4/5, the glob batch.

Run: python bench.py [--gpus N --steps K --warmup W --batch B]
     N > 1: one process per GPU, either launched by torch.distributed.run or,
     without WORLD_SIZE in the environment, started by this script itself
     (launch_ranks); the round collectives are the engine's own (mgpu_comm_*
     over RCCL, minotaur_amd.dist.NativeComm).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PFI_DEFAULT = 32            # MGPU_LP_PFI_MAX: K3P's default eta-file cap
OP_SUM, OP_MIN, OP_MAX = 0, 1, 2   # MGPU_OP_* (include/mgpu.h)
# the carrier of every cross-rank reduction of this run (minotaur_amd.dist:
# the engine's own collectives, mgpu_comm_*, or torch.distributed); set by
# main() once the ranks are up
COMM = None
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 dense (vector = matrix rate), spec
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec


def fbbt_bytes(p, B):
    """shared CSR + row bounds once, per node box in/out,
    types and status."""
    shared = p.nnz * (8 + 4) + (p.m + 1) * 4 + p.m * 16
    return shared + B * (p.n * 16 + p.n * 1 + p.n * 16 + 8)


def lp_flops(p, pivots, solves):
    """Algorithmic flops of the explicit-inverse dual simplex: per pivot the
    rank-1 update of B^-1 (2m^2), the pivot row rho'A (2 nnz) and the column
    B^-1 a_q (2 m nnz/n); per solve the primal recompute (2m^2 + 2 nnz)."""
    per_pivot = 2.0 * p.m * p.m + 2.0 * p.nnz + 2.0 * p.m * p.nnz / p.n
    per_solve = 2.0 * p.m * p.m + 2.0 * p.nnz
    return pivots * per_pivot + solves * per_solve


def pmc_traffic(kernel, batch, eta_cap, tree=False):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py from rocprofv3
    FETCH_SIZE/WRITE_SIZE passes of this same bench at the same batch and
    eta cap; tree: summaries of the tree-round headline, marked "workload":
    "tree_rounds").  Returns (bytes, file, fresh): fresh is True when the
    summary's source digest equals this tree's engine sources, False when
    the counters were taken on other code (reported as stale), None when the
    summary predates the digest."""
    import glob
    from minotaur_amd.build import source_digest
    keys = {'fbbt': ('fbbt_linear_persist', 'fbbt_linear_kernel'), 'lp_dual': ('lp_dual_kernel',),
            'lp_pfi': ('lp_pfi_kernel',)}[kernel]
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*_pmc.json')), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("workload") == "tree_rounds") != tree:
            continue
        args = d.get("bench_args", "").split()
        b = int(args[args.index('--batch') + 1]) if '--batch' in args else 65536
        cap = int(args[args.index('--eta-cap') + 1]) if '--eta-cap' in args else PFI_DEFAULT
        if b != batch or cap != eta_cap:
            continue
        for key in keys:
            k = d.get("kernels", {}).get(key)
            if k and k.get("hbm_bytes_per_launch"):
                dig = d.get("source_digest")
                return (k["hbm_bytes_per_launch"], os.path.basename(f),
                        None if dig is None else dig == source_digest())
    return None, None, None


def host_cpu():
    """(model name, threads the all-cores leg uses): the OpenMP thread count
    the box allows (OMP_NUM_THREADS; 16 per GPU on the GPU pool) capped by the
    CPUs this process may run on."""
    model = "unknown"
    try:
        with open('/proc/cpuinfo') as fh:
            for ln in fh:
                if ln.startswith('model name'):
                    model = ln.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0))
    want = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or avail
    return model, max(1, min(want, avail))


def pool_rows_decode(p, rows):
    """Migration rows of warm mode 2 ([lb | ub | bound | depth | k | path |
    packed statuses], bnb_migrate.hip) -> (lb, ub, k_in, path_in, st_in) for
    oracle.dual_simplex_path (the decoding of CpuBnbContext.bnb_import_rows,
    vectorised)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    n, N = p.n, p.n + p.m
    w = 2 * n + 2
    k_in = rows[:, w].astype(np.int32)
    path = rows[:, w + 1:w + 1 + oracle.PATH_MAX].astype(np.uint64).astype(np.uint32)
    words = rows[:, w + 1 + oracle.PATH_MAX:w + 1 + oracle.PATH_MAX + (N + 15) // 16]
    words = words.astype(np.int64)
    j = np.arange(N)
    st = ((words[:, j // 16] >> (2 * (j % 16))) & 3).astype(np.int8)
    return (np.ascontiguousarray(rows[:, :n]), np.ascontiguousarray(rows[:, n:2 * n]), k_in,
            path, st)


def cpu_baseline(p, LB, UB, budget_s, what_inst="tls4-lin", pool=None):
    """Rank 0, N=1, the same node boxes on the host:

    * all-cores leg (the reported value): the C restatement of the FBBT
      (bit-identical to the reference's LinearHandler::presolveNode, pinned
      by tests/golden/fbbt_*.npz) and of the dual simplex warm-started from
      the root basis, OpenMP over nodes on every core the box grants;
    * one-core leg: FBBT by the reference's own LinearHandler::presolveNode
      (oracle/_ref, prebuilt) when present, then the same dual simplex.
    Clp is unavailable, so the LP is the restatement in both."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    use_ref = oracle.have_ref()
    try:
        if use_ref:
            oracle.ref_lib()
    except OSError:
        use_ref = False
    _, _, _, _, _, ws = oracle.dual_simplex_root(p)
    model, T = host_cpu()

    def run(lb, ub, threads, ref):
        t0 = time.perf_counter()
        if ref:
            f = oracle.ref_linear_fbbt(p, lb, ub, None)
        else:
            f = oracle.linear_fbbt(p, lb, ub, None, nthreads=threads)
        t1 = time.perf_counter()
        keep = f.infeas == 0
        oracle.dual_simplex(p, f.lb[keep], f.ub[keep], ws, nthreads=threads)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, int(keep.sum())

    def sample(S):
        if S <= LB.shape[0]:
            return LB[:S], UB[:S], f"first {S} of the rank-0 node boxes"
        # more work than the batch holds: the batch again, cyclically (the
        # host code keeps no state between boxes; generating millions of new
        # boxes in Python would take minutes)
        idx = np.arange(S) % LB.shape[0]
        return (LB[idx], UB[idx],
                f"{S} boxes: the {LB.shape[0]} rank-0 node boxes cycled")

    def leg(threads, ref, budget):
        probe = min(256 * threads, LB.shape[0])
        a, b, _ = run(LB[:probe], UB[:probe], threads, ref)
        per = (a + b) / probe
        S = int(min(64 * LB.shape[0], max(probe, budget / max(per, 1e-9))))
        progress(0, f"cpu baseline leg ({threads} threads, ref={ref}): probe {probe} nodes "
                    f"{a + b:.2f}s -> sample {S}")
        lb, ub, what = sample(S)
        tf, tl, solved = run(lb, ub, threads, ref)
        progress(0, f"cpu baseline leg done: {tf + tl:.2f}s")
        return S, tf, tl, solved, what

    def pool_leg(budget, parent):
        """The GPU's own next nodes after the timed rounds (the work its next
        rounds would do), every LP warm-started either from the node's parent
        basis as K3P starts it (basis difference from the root rebuilt by
        column replacement, product form with the same eta cap, dense
        continuation past it) or from the root basis."""
        rows, inc, cap = pool
        lb, ub, k_in, path, st = pool_rows_decode(p, rows)
        inc_ = inc if math.isfinite(inc) else None

        def run_pool(idx):
            t0 = time.perf_counter()
            f = oracle.linear_fbbt(p, lb[idx], ub[idx], inc_, nthreads=T)
            t1 = time.perf_counter()
            keep = f.infeas == 0
            ki = idx[keep]
            if parent:
                oracle.dual_simplex_path(p, f.lb[keep], f.ub[keep], ws, k_in[ki], path[ki],
                                         st[ki], cap, min(32, cap), nthreads=T, want_x=False)
            else:
                oracle.dual_simplex(p, f.lb[keep], f.ub[keep], ws, nthreads=T)
            return t1 - t0, time.perf_counter() - t1, int(keep.sum())
        probe = np.arange(min(256 * T, lb.shape[0]))
        a, b, _ = run_pool(probe)
        per = (a + b) / len(probe)
        S = int(min(64 * lb.shape[0], max(len(probe), budget / max(per, 1e-9))))
        progress(0, f"cpu baseline pool leg ({T} threads, parent={parent}): probe "
                    f"{len(probe)} nodes {a + b:.2f}s -> sample {S}")
        tf, tl, solved = run_pool(np.arange(S) % lb.shape[0])
        progress(0, f"cpu baseline pool leg done: {tf + tl:.2f}s")
        return S, tf, tl, solved, lb.shape[0]

    fb1 = ('the reference LinearHandler::presolveNode (oracle/_ref)' if use_ref
           else 'the C restatement')
    if pool is not None and pool[0] is not None and len(pool[0]):
        # the GPU's own next nodes, both warm starts; the value is the faster
        # (the host's best choice: the restatement's column-replacement
        # rebuild of a parent basis costs more on a CPU than the pivots it saves)
        legs = {}
        for parent in (True, False):
            Sp, tfp, tlp, solvedp, npool = pool_leg(0.3 * budget_s, parent)
            legs[parent] = {
                "value": Sp / (tfp + tlp), "unit": "nodes/s", "cores": T,
                "relaxations_per_s": solvedp / (tfp + tlp),
                "sample": (f"{Sp} nodes: the {npool} next open nodes of the GPU's own pool "
                           f"after the timed rounds (cycled), {T} threads (OpenMP over nodes): "
                           f"FBBT by the C restatement (bit-identical to the reference) "
                           f"{tfp:.2f}s, then {solvedp} LPs by the dual-simplex restatement "
                           f"(Clp absent) warm-started from "
                           + ("the parent basis each node carries, as K3P starts them "
                              "(column replacement from the root inverse, product form, the "
                              "same eta cap)" if parent else "the root basis")
                           + f" {tlp:.2f}s")}
        S1, tf1, tl1, solved1, what1 = leg(1, use_ref, 0.4 * budget_s)
        best = legs[True] if legs[True]["value"] >= legs[False]["value"] else legs[False]
        head = dict(best, kind="port", cpu_model=model,
                    parent_warm=legs[True], root_warm=legs[False])
    else:
        S, tf, tl, solved, what = leg(T, False, 0.5 * budget_s)
        S1, tf1, tl1, solved1, what1 = leg(1, use_ref, 0.5 * budget_s)
        head = {
            "value": S / (tf + tl), "unit": "nodes/s", "cores": T, "kind": "port",
            "cpu_model": model,
            "sample": (f"{what} ({what_inst}), {T} threads (OpenMP over nodes): FBBT by the C "
                       f"restatement (bit-identical to the reference) {tf:.2f}s, then {solved} "
                       f"root-warm-started LPs by the dual-simplex restatement (Clp absent) "
                       f"{tl:.2f}s"),
            "relaxations_per_s": solved / (tf + tl),
        }
    return {
        **head,
        "one_core": {
            "value": S1 / (tf1 + tl1), "unit": "nodes/s", "cores": 1,
            "kind": "reference" if use_ref else "port",
            "sample": (f"{what1} ({what_inst}), one core: FBBT by {fb1} {tf1:.2f}s, then "
                       f"{solved1} LPs by the dual-simplex restatement {tl1:.2f}s"),
            "relaxations_per_s": solved1 / (tf1 + tl1),
        },
    }


def tree_cpu_baseline(p, brancher, seconds):
    """The tree on the CPU at one core: the reference's
    own BranchAndBound (bfs NodeHeap, PCBProcessor, NodeIncRelaxer,
    LinearHandler node FBBT, MaxVio or ReliabilityBrancher, guided dive) with
    CpuLPEngine -- an LPEngine over the C restatement of the dual simplex
    (oracle/ref/CpuLPEngine.cpp; Clp is absent) -- from the prebuilt
    oracle/_ref/libminotaur_hip_integ.so, bounded by the reference's
    time_limit option.  None when that library is absent."""
    import ctypes
    path = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')
    if not os.path.exists(path):
        return None
    from minotaur_amd import runtime
    runtime.load_library()
    lib = ctypes.CDLL(path, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    P = ctypes.c_void_p
    lib.integ_bnb_tree_cpu.argtypes = [ctypes.c_int] * 4 + [P] * 9 + [ctypes.c_double] * 2 + \
        [P, P]

    def _p(a):
        return a.ctypes.data_as(P)
    res = np.zeros(3)
    cnt = np.zeros(6, dtype=np.int64)
    lib.integ_bnb_tree_cpu(int(brancher), 1, p.n, p.m, _p(p.rowptr), _p(p.colidx), _p(p.val),
                           _p(p.rlo), _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub), _p(p.obj),
                           float(p.obj_const), float(seconds), _p(res), _p(cnt))
    done = bool(res[2] < 0.98 * seconds)
    return {"value": float(cnt[0]) / max(res[2], 1e-9), "unit": "nodes/s", "cores": 1,
            "kind": "reference",
            "sample": (f"{p.name}: the reference BranchAndBound (bfs, LinearHandler FBBT, "
                       f"{'ReliabilityBrancher' if brancher else 'MaxVioBrancher'}) with the "
                       f"dual-simplex restatement as its LP engine (Clp absent), one core, "
                       + (f"solved in {res[2]:.3f}s" if done else
                          f"stopped by time_limit {seconds:g}s")),
            "nodes": int(cnt[0]), "lp_solves": int(cnt[2]), "seconds": float(res[2]),
            "solved": done, "ub": float(res[0])}


TIMED_ALLOCS = {}   # per tree: device allocations / bytes inside its timed solve (all ranks)


def run_tree(ctx, dev, rank, world, p, B, order, warm, cap, brancher=0, trace=None, growth=0,
             reps=1, times=None):
    """One complete tree with the batched driver (mgpu_bnb_*), node-sharded
    across ranks after the shared first rounds: one packed all-reduce per
    round (incumbent MIN + open counts), open nodes rebalanced every 8 rounds
    or when a rank runs dry (dist.rebalance).  Returns (incumbent, nodes, LP
    solves, pivots, pruned-open, rounds, seconds, nodes moved, strong-branching
    LPs, their pivots) — counts summed over ranks, seconds the max.  ``trace``
    (a list) receives (seconds since the start, incumbent) per round of the
    first timed run.  reps > 1 times that many complete solves (the same tree
    each time) and returns the median; ``times`` (a list) receives each."""
    import torch
    from minotaur_amd import bnb
    from minotaur_amd.runtime import alloc_stats
    comm = COMM
    ctx.load(p)
    # warm-up: the whole tree once, at the timed batch and pool capacity, so
    # every device buffer the timed solve needs (pool, per-round batch
    # buffers, warm-start slots, continuation slots) already exists: the timed
    # region makes no device allocation (checked below; round 4's best-first
    # dense-warm entry timed a 17 GB pool allocation).  (A tree
    # whose later widths differ between runs could still grow a buffer: the
    # check then fails loudly instead of timing it.)
    # Across ranks the rebalancing exchanges (rows sent / received per deal)
    # can size their buffers differently from run to run, so with N > 1 the
    # warm-up repeats (at most three times) until a run allocates nothing.
    for _ in range(3 if world > 1 else 1):
        w0 = alloc_stats()
        bnb.solve_distributed(ctx, B, rank, world, capacity=cap, order=order, warm=warm,
                              comm=comm, lb_every=8, brancher=brancher, growth=growth)
        torch.cuda.synchronize()
        grew = float(comm.allreduce([float(alloc_stats() != w0)], OP_MAX)[0])
        if not grew:
            break
    a0 = alloc_stats()
    els = []
    for rep in range(reps):
        comm.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr = []
        inc, x, st, rounds, mine = bnb.solve_distributed(ctx, B, rank, world, capacity=cap,
                                                         order=order, warm=warm, comm=comm,
                                                         lb_every=8, brancher=brancher, trace=tr,
                                                         growth=growth)
        torch.cuda.synchronize()
        if rep == 0 and trace is not None:
            trace.extend((t - t0, v) for t, v in tr)
        comm.barrier()
        els.append(float(comm.allreduce([time.perf_counter() - t0], OP_MAX)[0]))
    a1 = alloc_stats()
    # summed over the ranks (rank 0 writes the line)
    na = [int(v) for v in comm.allreduce([float(a1[0] - a0[0]), float(a1[1] - a0[1])], OP_SUM)]
    if na[0] != 0:
        msg = (f"run_tree {p.name}: {na[0]} device allocation(s) ({na[1]} bytes, all ranks) "
               f"inside the timed tree")
        if world == 1:
            raise RuntimeError(msg)
        # N > 1: reported (timed_device_allocations in the result), not fatal,
        # so that a multi-GPU run still measures
        progress(rank, msg)
    TIMED_ALLOCS[p.name] = na
    if times is not None:
        times.extend(els)
    el = sorted(els)[len(els) // 2]
    c = [float(v) for v in comm.allreduce([float(mine[k]) for k in (
        'nodes', 'lps', 'pivots', 'pruned', 'sb_lps', 'sb_pivots')], OP_SUM)]
    return inc, c[0], c[1], c[2], c[3], rounds, el, mine['moved'], c[4], c[5]


# Complete trees in the bench line: config 2's instance as a
# MINLP (tls4's OA-LP: 10^5-node MaxVio trees, OA-MILP optimum 3.2 = HiGHS),
# its linear rows alone (tls4-lin, trivial: LP bound = optimum 0), config 1's
# OA-LP, and a weak-bound MILP whose tree is large enough to time the
# driver's throughput (multi-dimensional knapsack n = 60, m = 8).
# (name, kind, order, warm, optimum, brancher, growth): brancher 1 = the
# reference's default ReliabilityBrancher (strong-branching LPs count as
# relaxations); growth 2 (mgpu_bnb_growth): rounds of at most half the nodes
# evaluated so far, so the reliability brancher's decisions rest on earlier
# rounds' pseudocosts (a fixed wide batch grew tls4-OA's tree to 4.9x the
# reference's)
TREES = [("tls4_oa", "instance", 0, 0, 3.2, 0, 0),
         ("tls4_oa", "instance", 0, 2, 3.2, 0, 0),
         ("tls4_oa", "instance", 1, 0, 3.2, 0, 0),
         ("tls4_oa", "instance", 1, 1, 3.2, 0, 0),
         ("tls4_oa", "instance", 1, 2, 3.2, 0, 0),
         ("tls4_oa", "instance", 1, 1, 3.2, 1, 2),
         ("tls4_lin", "instance", 1, 1, 0.0, 1, 2),
         ("nvs08_oa", "instance", 1, 0, None, 0, 0),
         ("mkp-1-n60-m8", "mkp", 0, 0, -1915.0, 0, 0),
         ("mkp-1-n60-m8", "mkp", 1, 0, -1915.0, 0, 0),
         ("mkp-1-n60-m8", "mkp", 1, 1, -1915.0, 0, 0),
         ("mkp-1-n60-m8", "mkp", 1, 1, -1915.0, 1, 2)]


def tree_search(ctx, dev, rank, world, B, args):
    """Supplementary: complete branch-and-bound trees (every node popped from
    the HBM pool, children pushed, incumbent pruning) with their proven
    optima checked against HiGHS' MILP value."""
    from minotaur_amd.problem import LinProblem, random_mkp
    out = []
    cpu_trees = {}
    for name, kind, order, warm, opt, br, grow in TREES:
        if kind == "mkp":
            p = random_mkp(1, 60, 8)
        else:
            p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', f'{name}.npz'))
        if opt is None:
            sys.path.insert(0, os.path.join(ROOT, 'oracle'))
            import oracle
            opt = oracle.highs_milp(p)[1]
        # pool capacity: parent warm starts keep a basis per slot (m*m*8 B:
        # 32 KB for tls4-oa), so those pools are sized to the tree
        cap = 1 << 19 if warm and p.m > 16 else 1 << 23
        inc, nodes, lps, piv, pruned, rounds, el, moved, sbl, sbp = run_tree(
            ctx, dev, rank, world, p, B, order, warm, cap, br, growth=grow)
        progress(rank, f"tree {p.name} order {order} warm {warm} brancher {br}: "
                       f"{nodes:.0f} nodes in {el:.2f}s")
        out.append({"instance": p.name, "vars": p.n, "rows": p.m,
                    "search": ("best-first" if order else "depth-first over batches") +
                              (", parent-basis warm starts as pivot paths" if warm == 2 else
                               ", parent-basis warm starts" if warm else
                               ", root-basis warm start") +
                              (", reliability branching (strong branching + pseudocosts)"
                               if br else ", MaxVio branching") +
                              (f", batch growth {grow}" if grow else ""),
                    "nodes": nodes, "lp_solves": lps, "pivots_per_lp": piv / max(lps, 1.0),
                    "strong_branching_lps": sbl,
                    "pruned_open": pruned, "rounds": rounds, "seconds": el,
                    "nodes_migrated": moved,
                    "nodes_per_s": nodes / el, "relaxations_per_s": (lps + sbl) / el,
                    "batch_per_gpu": B, "optimum": inc, "optimum_highs": opt,
                    "timed_device_allocations": TIMED_ALLOCS.get(p.name),
                    "optimum_matches_highs": bool(abs(inc - opt) <= 1e-6 * max(1.0, abs(opt)))})
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            key = (p.name, br)
            if key not in cpu_trees:
                cpu_trees[key] = tree_cpu_baseline(p, br, args.tree_cpu_seconds)
                progress(rank, f"cpu tree {p.name} brancher {br}: {cpu_trees[key]}")
            if cpu_trees[key] is not None:
                out[-1]["cpu_baseline"] = cpu_trees[key]
    return out


def tls4_oa_tree(ctx, dev, rank, world, args):
    """Config 2's complete tree: tls4-OA from the root to
    the proven OA-MILP optimum 3.2 (= HiGHS), depth-first over batches, MaxVio
    branching, parent-basis warm starts (warm 2), node-sharded across ranks.
    Reported next to the headline because the headline's pool is the root
    plus B synthetic boxes: this is the instance's own tree, its nodes/s and
    its time to the optimum.  CPU baseline: the reference's own
    BranchAndBound on one core (oracle/_ref, LP restatement behind
    CpuLPEngine), bounded by --tree-cpu-seconds."""
    from minotaur_amd.problem import LinProblem
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = args.oa_tree_batch
    tr = []
    # the tree is solved once untimed (a warm process: kernels loaded, pool
    # buffers in place, clocks up), then timed.  Its rounds are narrow
    # (~2 700 nodes): K3P's 48-eta build keeps the LPs that need 33-48 etas
    # out of the dense continuation (the headline's wide rounds keep 32)
    ctx.load(p)
    ctx.set_lp_pfi(args.oa_tree_eta_cap)
    try:
        inc, nodes, lps, piv, pruned, rounds, el, moved, _, _ = run_tree(
            ctx, dev, rank, world, p, B, 0, 2, 1 << 21, 0, trace=tr)
    finally:
        ctx.set_lp_pfi(PFI_DEFAULT)
    tol = 1e-6 * max(1.0, abs(inc))
    tto = next((t for t, v in tr if v <= inc + tol), el)
    out = {"instance": f"tls4-oa ({p.m} rows, {p.n} cols)", "batch_per_gpu": B,
           "search": "depth-first over batches, MaxVio, parent-basis warm starts",
           "timing": "second of two full solves (the first warms the process)",
           "nodes": nodes, "rounds": rounds, "seconds": el, "nodes_per_s": nodes / el,
           "relaxations_per_s": lps / el, "pivots_per_lp": piv / max(lps, 1.0),
           "time_to_optimum_s": tto, "optimum": inc, "optimum_highs": 3.2,
           "optimum_matches_highs": bool(abs(inc - 3.2) <= 1e-6 * 3.2),
           "timed_device_allocations": TIMED_ALLOCS.get(p.name)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c1 = tree_cpu_baseline(p, 0, 4 * args.tree_cpu_seconds)
        if c1 is not None:
            out["cpu_reference_one_core"] = {k: c1[k] for k in ("value", "unit", "cores", "kind",
                                                                 "nodes", "seconds", "solved",
                                                                 "ub")}
            out["vs_reference_one_core"] = out["nodes_per_s"] / max(c1["value"], 1e-9)
    return out


def tls4_oa_rel_tree(ctx, dev, rank, world, args):
    """Config 2's tree with the reference's DEFAULT brancher (VERDICT r04 item
    3): reliability branching (Environment.cpp:574-576 sets "rel"), best-
    first, parent-basis warm starts, batch growth 2 -- its node count and
    time to proof (the whole tree: the optimum proven) next to the
    reference's own BranchAndBound + ReliabilityBrancher on one core
    (oracle/_ref, LP restatement behind CpuLPEngine)."""
    from minotaur_amd.problem import LinProblem
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = args.tree_batch
    # the median of five complete solves (each ~25 ms; a single run moves by
    # about 1 ms from process to process)
    runs = []
    inc, nodes, lps, piv, pruned, rounds, el, moved, sbl, sbp = run_tree(
        ctx, dev, rank, world, p, B, 1, 1, 1 << 20, 1, growth=2, reps=5, times=runs)
    out = {"instance": f"tls4-oa ({p.m} rows, {p.n} cols)", "batch_cap_per_gpu": B,
           "search": "best-first, reliability branching (strong branching + pseudocosts), "
                     "parent-basis warm starts, batch growth 2",
           "nodes": nodes, "rounds": rounds, "lp_solves": lps, "strong_branching_lps": sbl,
           "time_to_proof_s": el, "time_to_proof_runs_s": [round(t, 5) for t in runs],
           "optimum": inc,
           "optimum_matches_highs": bool(abs(inc - 3.2) <= 1e-6 * 3.2),
           "timed_device_allocations": TIMED_ALLOCS.get(p.name)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c1 = tree_cpu_baseline(p, 1, 4 * args.tree_cpu_seconds)
        if c1 is not None:
            out["reference_one_core"] = {"nodes": c1["nodes"], "seconds": c1["seconds"],
                                         "solved": c1["solved"], "ub": c1["ub"]}
            out["nodes_vs_reference"] = nodes / max(c1["nodes"], 1)
            out["time_to_proof_speedup"] = c1["seconds"] / max(el, 1e-9)
    return out


def knapsack_nodes(ctx, dev, rank, world, args, reps=50):
    """Supplementary (config 3): 1000 synthetic knapsack-MINLP
    nodes (seeded boxes of [1, 64]^9, seed 7) of the examples/knapsack OA-LP
    (f = 9, N = 64, 4 tangents per term: m = 37), batched FBBT + LP relaxation
    from the root basis + decision, repeated `reps` times."""
    import torch
    from minotaur_amd import dist as mdist
    from minotaur_amd.problem import knapsack_oa, random_boxes
    from minotaur_amd.runtime import WarmStart
    p = knapsack_oa()
    ctx.load(p)
    root, ws_h = ctx.root_solve()
    ws = WarmStart(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (ws_h.head, ws_h.st, ws_h.d, ws_h.binv)))
    LB, UB = random_boxes(p, 1000, mdist.shard_seed(7, rank))
    B = LB.shape[0]
    lb0, ub0 = torch.from_numpy(LB).to(dev), torch.from_numpy(UB).to(dev)
    lb1, ub1 = torch.empty_like(lb0), torch.empty_like(ub0)
    z32 = lambda: torch.zeros(B, dtype=torch.int32, device=dev)   # noqa: E731
    inf, nm, st, it, dec = z32(), z32(), z32(), z32(), z32()
    ob = torch.zeros(B, dtype=torch.float64, device=dev)
    x = torch.zeros((B, p.n), dtype=torch.float64, device=dev)

    def step():
        ctx.fbbt_dev(lb0, ub0, lb1, ub1, inf, nm)
        ctx.lp_solve_dev(lb1, ub1, st, ob, it, ws=ws, skip=inf, x=x)
        ctx.node_decide_dev(st, ob, x, dec, fbbt_infeas=inf)

    step()
    torch.cuda.synchronize()
    fb, lp = [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
        fb.append(ctx.last_kernel_ms('fbbt'))
        lp.append(ctx.last_kernel_ms('lp'))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    solved = int((st != 12).sum().item())
    piv = int(it.sum().item())
    fbm, lpm = float(np.median(fb)), float(np.median(lp))
    lpf = lp_flops(p, piv, solved)
    out = {"instance": f"{p.name} ({p.m} rows, {p.n} cols)", "nodes": B, "reps": reps,
           "nodes_per_s": B * reps / el, "relaxations_per_s": solved * reps / el,
           "ms_per_batch": 1e3 * el / reps, "fbbt_ms": fbm, "lp_ms": lpm,
           "pivots_per_lp": piv / max(solved, 1),
           "roofline": {"kernel": "lp", "bound": "fp64", "unit": "TFLOP/s",
                        "achieved": lpf / (lpm * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                        "frac": lpf / (lpm * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                        "note": "1000 LPs are a fraction of one wave per SIMD: launch- and "
                                "latency-bound by construction"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(p, LB, UB, 4.0, "knapsack boxes")
    return out


# Config 5 ("64 synthetic convex separable MINLPs (knapsack
# family) until MINLPLib .nl files are provided", node-sharded): outer-
# approximation LPs of examples/knapsack (knapsack_oa: min sum a_i x_i^b_i,
# sum x <= N, x integer in [1, N], 4 tangents per term) with f terms,
# N = 3 f; m = 1 + 4 f rows, so f >= 16 crosses the K3 / K3L boundary
# (m > 64 -> K3L).  Optima: scipy HiGHS MILP on the same LPs (this
# container; tools/convex_batch_optima.py prints them).
CONVEX_BATCH = [(16, 48, 6.931342750371372), (20, 60, 7.812507818465321),
                (24, 72, 9.458626537799338), (28, 84, 13.920825697253907)]


def convex_batch(ctx, dev, rank, world, B, args):
    """Supplementary (config 5): complete trees over the convex batch, each
    node-sharded across ranks (mgpu_bnb_shard) with an incumbent all-reduce
    MIN per round; nodes/s and LP relaxations/s over the whole batch."""
    import torch
    from minotaur_amd import bnb
    from minotaur_amd.problem import knapsack_oa
    comm = COMM

    per, tot_nodes, tot_s, ok = [], 0.0, 0.0, True
    for f, N, opt in CONVEX_BATCH:
        p = knapsack_oa(f=f, N=N)
        ctx.load(p)
        bnb.solve_distributed(ctx, 64, rank, world, capacity=1 << 14, max_rounds=2,
                              comm=comm)                     # warm-up (kernel loads)
        comm.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        inc, x, st, rounds, mine = bnb.solve_distributed(ctx, B, rank, world, capacity=1 << 21,
                                                         comm=comm)
        torch.cuda.synchronize()
        comm.barrier()
        el = float(comm.allreduce([time.perf_counter() - t0], OP_MAX)[0])
        nodes = float(comm.allreduce([float(mine['nodes'])], OP_SUM)[0])
        good = abs(inc - opt) <= 1e-6 * max(1.0, abs(opt))
        ok &= good
        tot_nodes += nodes
        tot_s += el
        kern = (("K3P + K3 overflow" if p.m <= 64 else "K3PW + K3L overflow")
                if ctx.oracle_pfi() > 0 else ("K3" if p.m <= 64 else "K3L"))
        per.append({"f": f, "rows": p.m, "lp_kernel": kern,
                    "nodes": nodes, "seconds": el, "rounds": rounds, "optimum": inc,
                    "optimum_highs": opt})
    return {"instances": per, "nodes": tot_nodes, "seconds": tot_s,
            "nodes_per_s": tot_nodes / tot_s, "all_optima_match_highs": bool(ok),
            "batch_per_gpu": B,
            "search": "depth-first over batches, MaxVio branching, root-basis warm start, "
                      "node-sharded after the shared first rounds"}


def glob_batch(ctx, dev, rank, world, args, B=65536, reps=10):
    """Supplementary (the batched glob path): node boxes of
    a random QCQP (seeded; 14 original variables, 8 quadratic rows -> 31
    columns, 52 LP rows with 40 McCormick / secant rows rewritten per node)
    through K2 (QuadHandler::presolveNode: bounds + row rewrite), then every
    node's own LP (mgpu_lp_solve_rows: K3R refactors the root basis for the
    node's rows, K3 solves), device-resident, repeated `reps` times."""
    import torch
    from minotaur_amd import dist as mdist
    from minotaur_amd.quad import random_qcqp, random_quad_boxes, relaxation_lp
    from minotaur_amd.runtime import WarmStart
    qp = random_qcqp(7, nv0=14, ncon=8)
    ctx.load_quad(qp)
    rows0 = ctx.quad_rows()
    p, nr = relaxation_lp(qp, rows0)
    ctx.load(p)
    root, ws = ctx.root_solve()          # the device's own root LP and basis
    st0 = int(root.status[0])
    ctx.set_node_rows(nr)
    LB, UB = random_quad_boxes(qp, B, mdist.shard_seed(23, rank))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    lb, ub, rows = t(LB), t(UB), t(np.tile(rows0, (B, 1)))
    lb2, ub2, rows2 = torch.empty_like(lb), torch.empty_like(ub), torch.empty_like(rows)
    z32 = lambda: torch.zeros(B, dtype=torch.int32, device=dev)   # noqa: E731
    inf, nm, st, it = z32(), z32(), z32(), z32()
    ob = torch.zeros(B, dtype=torch.float64, device=dev)
    # the root inverse (column-major) lets K3R replace only the basic columns
    # a node's rows changed instead of refactoring from scratch
    wsd = WarmStart(t(ws.head.astype(np.int32)), t(ws.st.astype(np.int8)), None,
                    t(ws.binv))       # column-major, the ABI layout

    def step():
        ctx.quad_fbbt_dev(lb, ub, rows, lb2, ub2, rows2, inf, nm, qt=1)
        ctx.lp_solve_rows_dev(lb2, ub2, rows2, st, ob, it, ws=wsd, skip=inf)

    step()
    torch.cuda.synchronize()
    k2, rf, lp = [], [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
        k2.append(ctx.last_kernel_ms('quad'))
        rf.append(ctx.last_kernel_ms('refactor'))
        lp.append(ctx.last_kernel_ms('lp'))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    solved = int((st != 12).sum().item())
    out = {"instance": f"{qp.name} relaxation ({p.n} cols, {p.m} rows, "
                       f"{nr.row_idx.size} rows rewritten per node)",
           "nodes_per_gpu": B, "reps": reps, "nodes_per_s": B * reps * world / el,
           "relaxations_per_s": solved * reps * world / el,
           "k2_ms": float(np.median(k2)), "refactor_ms": float(np.median(rf)),
           "lp_ms": float(np.median(lp)), "pivots_per_lp": float(it.sum().item()) / max(solved, 1),
           "root_lp_status": int(st0)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import oracle
        S = 2048
        t0 = time.perf_counter()
        o = oracle.quad_fbbt(qp, LB[:S], UB[:S], None, 1, rows0)
        oracle.dual_simplex_rows(p, o.lb, o.ub, nr, o.rows, ws=WarmStart(ws.head, ws.st, None,
                                                                          None))
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": S / dt, "unit": "nodes/s", "cores": 1, "kind": "port",
                               "sample": f"first {S} node boxes: K2 by the C restatement "
                                         "(bit-identical to the reference QuadHandler), node "
                                         f"LPs by the dual-simplex restatement, {dt:.2f}s"}
    return out


def glob_tree(ctx, dev, rank, world, args, B=8192, max_rounds=400):
    """Supplementary (the glob path's own tree): the
    batched spatial branch-and-bound (mgpu_glob_*) on seeded bilinear QCQPs
    -- every round pops B nodes, runs K2 from the parents' rows, K3R + K3 on
    each node's own rows, the glob decision with MaxVio branching over the
    IntVarHandler and QuadHandler candidates and pushes the children -- to
    completion (or max_rounds).  Rank r runs seed s + r (weak scaling).  The
    last instance's relaxation has 90 rows: its node LPs run on K3L with the
    rows in HBM and the root basis refactored inside the kernel.
    A one-core CPU baseline runs the restatement (oracle/glob_tree.py) on
    the same instance for a bounded time."""
    import torch
    from minotaur_amd import glob as mglob
    from minotaur_amd.quad import random_qcqp
    out = []
    # bilinear QCQPs, and one with squares (y >= x^2 by the separation loop's
    # tangent cuts, S slots per square: round 6)
    for seed, nv0, ncon, sq in ((17, 10, 6, False), (9, 12, 7, False), (19, 12, 7, False),
                                (2, 16, 10, False), (2, 16, 10, True)):
        qp = random_qcqp(seed + rank, nv0=nv0, ncon=ncon, squares=sq)
        p, nr = mglob.setup(ctx, qp)
        mglob.solve(ctx, qp, batch=64, capacity=1 << 14, max_rounds=2, loaded=True)  # warm-up
        torch.cuda.synchronize()
        obj, x, st, secs = mglob.solve(ctx, qp, batch=B, capacity=64 * B,
                                       max_rounds=max_rounds, loaded=True)
        torch.cuda.synchronize()
        kind = (f"QCQP with {qp.nsq} squares and {qp.nbil} products" if sq else
                f"bilinear QCQP ({qp.nbil} products")
        e = {"instance": f"{qp.name} {kind}, {qp.nv0} vars, "
                         f"{qp.ncon} rows -> LP {p.n} cols x {p.m} rows)",
             "batch_per_gpu": B, "rounds": int(st.rounds), "nodes": int(st.nodes),
             "open": int(st.open), "solved": st.open == 0,
             "decisions": {"branched": int(st.ndec[0]), "infeasible": int(st.ndec[1]),
                           "pruned_by_bound": int(st.ndec[2]), "feasible": int(st.ndec[3]),
                           "no_candidate": int(st.ndec[5])},
             "branchings_int": int(st.br_int), "branchings_spatial": int(st.br_cont),
             "lp_solves": int(st.lps), "pivots_per_lp": st.pivots / max(st.lps, 1),
             "tangent_cuts": int(st.cuts), "resolves": int(st.resolves),
             "incumbent": obj, "seconds": secs, "nodes_per_s": st.nodes / secs,
             "relaxations_per_s": st.lps / secs}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, 'oracle'))
            from glob_tree import CpuGlobContext
            c = CpuGlobContext(qp, tan_slots=mglob.TAN_SLOTS if sq else 0)
            c.glob_init(1 << 22)
            t0 = time.perf_counter()
            cs = None
            while time.perf_counter() - t0 < args.tree_cpu_seconds:
                cs = c.glob_round(64)
                if cs.open == 0:
                    break
            dt = time.perf_counter() - t0
            e["cpu_baseline"] = {"value": cs.nodes / dt, "unit": "nodes/s", "cores": 1,
                                 "kind": "port",
                                 "sample": f"the same tree by the CPU restatement (C K2 + "
                                           f"dual-simplex restatement + Python decision), "
                                           f"rounds of 64, {cs.nodes} nodes in {dt:.2f}s"}
        out.append(e)
    return out


def qp_relaxation(ctx, dev, rank, world, args, B=1024, reps=3):
    """Supplementary (config 4): QP relaxations of color_lab2_4x0 node boxes
    (300 vars relaxed to [0,1] with random fixings, 61 equality rows, dense
    Q) solved in one batch per rank by K5 — interior point with the KKT
    block factored on MFMA f64 — with its MFMA roofline and a one-core CPU
    baseline of the same algorithm (oracle/qp_ipm.py, numpy/LAPACK)."""
    import torch
    from minotaur_amd import dist as mdist
    from minotaur_amd import qp as qpm
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    ctx.load_qp(P)
    LB, UB = qpm.random_node_boxes(P, B, mdist.shard_seed(17, rank))
    lb = torch.from_numpy(LB).to(dev)
    ub = torch.from_numpy(UB).to(dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    ob = torch.zeros(B, dtype=torch.float64, device=dev)
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    ctx.qp_solve_dev(lb[:64], ub[:64], st, ob, it)        # warm-up
    torch.cuda.synchronize()
    ms, iters, ok = [], 0, 0
    for _ in range(reps):
        ctx.qp_solve_dev(lb, ub, st, ob, it)
        torch.cuda.synchronize()
        ms.append(ctx.last_kernel_ms('qp'))
        iters = int(it.sum().item())
        ok = int((st == 0).sum().item())
    k = float(np.median(ms))
    np_, mp = 304, 64                                    # padded KKT sizes
    flops = iters * (np_ ** 3 / 3 + np_ ** 2 * mp + np_ * mp ** 2)
    # one more solve with per-kernel events (outside the timed reps): the
    # factor kernel's and the W / Schur kernel's own rooflines
    ctx.set_qp_ktime(True)
    ctx.qp_solve_dev(lb, ub, st, ob, it)
    torch.cuda.synchronize()
    ctx.set_qp_ktime(False)
    kms = {name: ctx.last_kernel_ms(name) for name in ('qp_potrf', 'qp_trsm', 'qp_step')}
    kit = int(it.sum().item())
    f_potrf = kit * np_ ** 3 / 3
    f_trsm = kit * (np_ ** 2 * mp + np_ * mp ** 2)

    def kroof(f, ms_):
        a = f / (ms_ * 1e-3) / 1e12 if ms_ > 0 else 0.0
        return {"achieved": a, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": a / FP64_PEAK_TFLOPS, "ms": ms_}
    tot = float(COMM.allreduce([B / (k * 1e-3)], OP_SUM)[0])
    out = {"instance": "color_lab2_4x0 (n=300, m=61, dense Q)", "batch_per_gpu": B,
           "qp_per_s": tot, "ms_per_batch": k, "converged": ok,
           "ipm_iters_per_qp": iters / B,
           # the dominant MFMA kernel (the KKT factor) over its own time, as
           # the headline's roofline is; the whole-solve figure beside it
           "roofline": dict(kroof(f_potrf, kms['qp_potrf']), bound="mfma",
                            kernel="qp_potrf_ll (KKT block Cholesky, n^3/3 per node-iteration)",
                            note="per-kernel hipEvents over one extra solve; MFMA-busy "
                                 "fraction by counter in profiles/r05r_k5_counters.json"),
           "kernels": {"qp_potrf_ll": kroof(f_potrf, kms['qp_potrf']),
                       "qp_trsm_syrk_lds": kroof(f_trsm, kms['qp_trsm']),
                       "qp_step_ms": kms['qp_step']},
           "whole_solve_roofline": {"bound": "mfma", "achieved": flops / (k * 1e-3) / 1e12,
                                    "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                    "frac": flops / (k * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                                    "note": "algorithmic f64 flops of the KKT factorizations "
                                            "(n^3/3 + n^2 m + n m^2 per IPM iteration, padded "
                                            "n=304, m=64) over the whole solve time"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import qp_ipm
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1):             # one core, as "cores" says
            t0 = time.perf_counter()
            S = 0
            while S < 8 and time.perf_counter() - t0 < 10.0:
                qp_ipm.solve_node(P.Q, P.c, P.A, P.b, LB[S], UB[S])
                S += 1
            dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": S / dt, "unit": "QP/s", "cores": 1, "kind": "port",
                               "sample": f"first {S} node QPs, the same interior point in "
                                         f"numpy/LAPACK (oracle/qp_ipm.py), {dt:.2f}s "
                                         "(BQPD is binary-only and absent)"}
    return out


def qp_tree(ctx, dev, rank, world, args, B=256, max_rounds=200):
    """Supplementary (config 4 as a path): branch-and-bound over
    QP relaxations of color_lab2_4x0 -- every round pops B nodes, K1 FBBT on
    the equality rows, K5 (MFMA KKT) on the node QPs, decision + MaxVio
    branching, children pushed -- for a bounded number of rounds.  200
    depth-first rounds reach leaves: the run finds incumbents and prunes by
    bound (12 rounds, round 4's bound, branched every node and found none;
    tools/qp_tree_probe.py)."""
    import torch
    from minotaur_amd import qp as qpm
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    qpm.solve_tree(ctx, P, batch=16, capacity=1 << 12, max_rounds=1)     # warm-up
    torch.cuda.synchronize()
    obj, x, st, secs = qpm.solve_tree(ctx, P, batch=B, capacity=1 << 18, max_rounds=max_rounds)
    torch.cuda.synchronize()
    return {"instance": "color_lab2_4x0 (300 binaries, 61 rows, dense Q)", "batch_per_gpu": B,
            "rounds": int(st.rounds), "nodes": int(st.nodes), "qp_solves": int(st.lps),
            "ipm_iters_per_qp": st.pivots / max(st.lps, 1), "open": int(st.open),
            "incumbent": obj, "seconds": secs, "nodes_per_s": st.nodes / secs,
            "decisions": {"branched": int(st.ndec[0]), "infeasible": int(st.ndec[1]),
                          "pruned_by_bound": int(st.ndec[2]), "feasible": int(st.ndec[3])}}


def lp_flops_tableau(p, pivots):
    """SURVEY 8(d)'s LP flop count: the tableau rank-1 update, 2 m (n + m)
    per pivot (tls4: 19.8 kflop per pivot)."""
    return pivots * 2.0 * p.m * (p.n + p.m)


def kernel_entries(p, nb, fbbt_ms, lp_main_ms, lp_ms, lp_tail_ms, lps, lp_pivots, pfi_pivots):
    """Per-launch roofline entries of K1 and K3P (algorithmic bytes / flops of
    one launch over its HIP-event time).  K3P's work: the pivots it ran itself
    (an LP that overflows its eta file runs its first pfi_cap pivots in K3P,
    the rest in the dense continuation, timed apart as overflow_resolve_ms)."""
    fb = fbbt_bytes(p, nb)
    tab = lp_flops_tableau(p, pfi_pivots)
    rev = lp_flops(p, pfi_pivots, lps)
    k = {
        "fbbt": {"ms": fbbt_ms, "bound": "hbm", "achieved": fb / (fbbt_ms * 1e-3) / 1e9,
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "bytes_per_launch": fb,
                 "nodes_per_launch": nb},
        "lp_pfi": {"ms": lp_main_ms, "bound": "fp64", "unit": "TFLOP/s",
                   "achieved": tab / (lp_main_ms * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                   "flops_per_launch": tab,
                   "flop_count": "SURVEY 8(d): 2 m (n + m) per pivot",
                   "revised_flops_per_launch": rev,
                   "revised_achieved": rev / (lp_main_ms * 1e-3) / 1e12,
                   "revised_flop_count": "per pivot 2m^2 + 2 nnz + 2 m nnz / n, per solve "
                                         "2m^2 + 2 nnz (explicit-inverse revised simplex)",
                   "solves_per_launch": lps, "pivots_in_launch": pfi_pivots,
                   "pivots_per_solve": lp_pivots / max(lps, 1),
                   "lp_call_ms": lp_ms, "overflow_resolve_ms": lp_tail_ms},
    }
    for e in k.values():
        e["frac"] = e["achieved"] / e["peak"]
    k["lp_pfi"]["revised_frac"] = k["lp_pfi"]["revised_achieved"] / FP64_PEAK_TFLOPS
    return k


def tree_rounds(ctx, dev, rank, world, p, LB, UB, args):
    """The headline: rounds of the batched tree (mgpu_bnb_round) over an HBM
    node stack that starts as the root plus the B seeded boxes; every step is
    ONE round (pop B nodes, K1, K3P, decide + MaxVio choice, children pushed)
    and one packed all-reduce of the incumbent and open counts.  Returns the
    aggregate counts (summed over ranks), the max elapsed time and rank 0's
    per-launch kernel entries."""
    import torch
    from minotaur_amd import dist as mdist
    B = LB.shape[0]
    ctx.load(p)
    cap = B * (max(1, args.warmup) + args.steps + 2) + 2
    ctx.set_lp_pfi(args.eta_cap)
    ctx.bnb_config(0, args.warm)
    ctx.bnb_brancher(0)
    ctx.bnb_init(cap)
    if rank > 0:
        ctx.bnb_export(1)        # the root belongs to rank 0 (MpiBranchAndBound.cpp:246-279)
    ctx.bnb_import(LB, UB, np.full(B, -math.inf), np.zeros(B, dtype=np.int32))
    comm = COMM
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    state = {"inc": math.inf, "prev": None}
    keys = ("nodes", "lps", "pivots", "pfi_pivots")

    def step(acc):
        st = ctx.bnb_round(B, state["inc"])
        ev[0].record()
        inc, most, _, _ = comm.round_reduce(st.incumbent, st.open)
        ev[1].record()
        ev[1].synchronize()
        state["inc"] = min(state["inc"], inc)
        cur = {k: getattr(st, k) for k in keys}
        if acc is not None:
            prev = state["prev"]
            for k in keys:
                acc[k] += cur[k] - prev[k]
            acc["fbbt_ms"].append(ctx.last_kernel_ms('fbbt'))
            acc["lp_ms"].append(ctx.last_kernel_ms('lp'))
            acc["lp_main_ms"].append(ctx.last_kernel_ms('lp_main'))
            acc["lp_tail_ms"].append(ctx.last_kernel_ms('lp_tail'))
            acc["batch"].append(st.last_batch)
            acc["rccl_ms"].append(ev[0].elapsed_time(ev[1]))
            acc["open"] = st.open
        state["prev"] = cur
        return most

    lb_pick = B if args.lb_pick == 'batch' else 0
    for _ in range(max(1, args.warmup)):
        step(None)
    if world > 1 and args.lb_every > 0:
        # one rebalance at the timed pick size: the exchange's workspaces are
        # sized here (mgpu_bnb_rebalance reserves its worst case for that
        # size), so the timed loop's rebalances allocate nothing
        mdist.rebalance(ctx, comm, lb_pick)
    acc = {k: 0 for k in keys}
    acc.update({"fbbt_ms": [], "lp_ms": [], "lp_main_ms": [], "lp_tail_ms": [], "batch": [],
                "rccl_ms": [], "open": 0})
    comm.barrier()
    torch.cuda.synchronize()
    from minotaur_amd.runtime import alloc_stats
    a0 = alloc_stats()
    t0 = time.perf_counter()
    moved = 0
    for k in range(args.steps):
        step(acc)
        if world > 1 and args.lb_every > 0 and (k + 1) % args.lb_every == 0:
            # one pool across the ranks: bound-aware rebalancing inside the
            # timed loop (MpiBranchAndBound::LoadBalance_, dist.rebalance);
            # --lb-pick reference: each rank offers the reference's 50 P next
            # candidates (:80-105); batch: max(50 P, B), the globally best
            # P * B nodes dealt (~(P-1)/P of a batch crosses xGMI)
            _, mv, _, _ = mdist.rebalance(ctx, comm, lb_pick)
            moved += mv
    torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    a1 = alloc_stats()
    tot = float(comm.allreduce([elapsed], OP_MAX)[0])
    nodes, lps, pivots, pfi_pivots = (float(v) for v in comm.allreduce(
        [float(acc[k]) for k in keys], OP_SUM))
    S = args.steps
    nb = float(np.mean(acc["batch"]))
    kernels = kernel_entries(p, nb, float(np.mean(acc["fbbt_ms"])),
                             float(np.mean(acc["lp_main_ms"])), float(np.mean(acc["lp_ms"])),
                             float(np.mean(acc["lp_tail_ms"])), acc["lps"] / S,
                             acc["pivots"] / S, acc["pfi_pivots"] / S)
    summary = {"nodes": nodes, "lp_solves": lps, "pivots_per_lp": pivots / max(lps, 1.0),
               "nodes_per_round_per_gpu": nb, "open_after_rank0": acc["open"],
               "search": "depth-first over batches (HBM stack), MaxVio branching, " +
                         ("parent-basis warm starts kept as pivot paths from the root basis "
                          "(K3P)" if args.warm == 2 else "root-basis warm start (K3P)"),
               "incumbent": state["inc"]}
    summary["nodes_migrated"] = moved
    # device allocations inside the timed loop, summed over the ranks: none
    # at any N (the warm-up sized every buffer, the rebalance's included)
    na = comm.allreduce([float(a1[0] - a0[0]), float(a1[1] - a0[1])], OP_SUM)
    summary["device_allocs_timed"] = int(na[0])
    if na[0] != 0:
        raise RuntimeError(f"headline: {int(na[0])} device allocation(s) ({int(na[1])} bytes, "
                           f"all ranks) inside the timed rounds")
    # after the timed rounds: the next nodes of this pool, with the parent
    # bases they carry, for the CPU baseline (exported and imported back)
    pool_sample = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.warm == 2:
        lbs = ctx.bnb_pick(args.cpu_pool_nodes)
        if len(lbs):
            rows = ctx.bnb_export_rows(np.arange(len(lbs)))
            pool_sample = rows.cpu().numpy()
            ctx.bnb_import_rows(rows)
    return {"elapsed": tot, "nodes": nodes, "lps": lps, "kernels": kernels,
            "summary": summary, "incumbent": state["inc"],
            "rccl_ms": float(np.sum(acc["rccl_ms"])), "pool_sample": pool_sample}


def fixed_batch(ctx, dev, rank, world, args, reps=10):
    """Supplementary (round 1-2 headline, kept for continuity): one FIXED
    batch of tls4-lin node boxes re-evaluated every step — K1 FBBT -> K3P LP
    from the root basis -> prune/integrality decision — with no branching,
    no selection and no child writes (the kernel-only throughput of the node
    pipeline)."""
    import torch
    from minotaur_amd import dist as mdist
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import WarmStart
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    B = args.batch
    LB, UB = random_boxes(p, B, mdist.shard_seed(20261015, rank))
    ctx.load(p)
    root, ws_h = ctx.root_solve()
    assert root.status[0] == 0, "root LP not optimal"
    ws = WarmStart(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (ws_h.head, ws_h.st, ws_h.d, ws_h.binv)))
    lb0, ub0 = torch.from_numpy(LB).to(dev), torch.from_numpy(UB).to(dev)
    lb1, ub1 = torch.empty_like(lb0), torch.empty_like(ub0)
    z32 = lambda: torch.zeros(B, dtype=torch.int32, device=dev)   # noqa: E731
    infeas, nmods, status, iters, decision = z32(), z32(), z32(), z32(), z32()
    obj = torch.zeros(B, dtype=torch.float64, device=dev)
    cand = torch.zeros(B, dtype=torch.float64, device=dev)
    x = torch.zeros((B, p.n), dtype=torch.float64, device=dev)
    # root-warm-started batches make few pivots (5.9 on average, 99.9 % <= 24):
    # the 16-eta file runs four waves per SIMD instead of three;
    # the path-warm-started headline keeps the 32-eta file
    ctx.set_lp_pfi(16)
    cap = ctx.oracle_pfi()

    def step():
        ctx.fbbt_dev(lb0, ub0, lb1, ub1, infeas, nmods)
        ctx.lp_solve_dev(lb1, ub1, status, obj, iters, ws=ws, skip=infeas, x=x)
        ctx.node_decide_dev(status, obj, x, decision, fbbt_infeas=infeas, cand_obj=cand)

    step()
    torch.cuda.synchronize()
    fb, lp, lpm, lpt = [], [], [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
        fb.append(ctx.last_kernel_ms('fbbt'))
        lp.append(ctx.last_kernel_ms('lp'))
        lpm.append(ctx.last_kernel_ms('lp_main'))
        lpt.append(ctx.last_kernel_ms('lp_tail'))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    solved = float((status != 12).sum().item())
    piv = float(iters.sum().item())
    pfi_piv = float(torch.where(status != 12, torch.clamp(iters, max=cap), 0).sum().item())
    k = kernel_entries(p, B, float(np.mean(fb)), float(np.mean(lpm)), float(np.mean(lp)),
                       float(np.mean(lpt)), solved, piv, pfi_piv)
    ctx.set_lp_pfi(32)
    return {"instance": f"tls4-lin ({p.m} rows, {p.n} cols, {p.nnz} nnz)",
            "nodes_per_gpu": B, "reps": reps, "nodes_per_s": B * reps * world / el,
            "relaxations_per_s": solved * reps * world / el, "ms_per_batch": 1e3 * el / reps,
            "kernels": k}


def _r(v, k=4):
    """Round floats for the compact line (significant digits kept)."""
    if isinstance(v, float) and math.isfinite(v) and v != 0.0:
        return float(f"{v:.{k}g}")
    return v


LINE_MAX = 6000   # the driver keeps the tail of stdout: the line must stay short


def compact_line(args, world, B, p, h, elapsed, nodes, lps, roofline, kernels, cpu, oa_tree,
                 supp, supp_path, rel_tree=None):
    """The ONE stdout JSON line (< 6 KB so the driver's
    stdout tail holds it whole): the metric, the roofline of the dominant
    kernel, the CPU baselines, config 2's complete tree and one number per
    supplementary object; the objects themselves go to ``supp_path``."""
    kf, kl = kernels["fbbt"], kernels["lp_pfi"]
    ks = {"fbbt": {"ms": _r(kf["ms"]), "achieved_gbs": _r(kf["achieved"]),
                   "frac": _r(kf["frac"]), "bytes_per_launch": _r(kf["bytes_per_launch"])},
          "lp_pfi": {"ms": _r(kl["ms"]), "achieved_tflops": _r(kl["achieved"]),
                     "frac": _r(kl["frac"]), "revised_frac": _r(kl["revised_frac"]),
                     "pivots_per_solve": _r(kl["pivots_per_solve"]),
                     "overflow_resolve_ms": _r(kl["overflow_resolve_ms"])}}
    rf = {k: _r(v) for k, v in roofline.items()}
    cb = None
    if cpu is not None:
        cb = {"value": _r(cpu["value"]), "unit": cpu["unit"], "cores": cpu["cores"],
              "kind": cpu["kind"], "cpu_model": cpu["cpu_model"],
              "sample": cpu["sample"][:300],
              "relaxations_per_s": _r(cpu["relaxations_per_s"]),
              "one_core": {k: (_r(v) if k != "sample" else v[:200])
                           for k, v in cpu["one_core"].items()}}
        for key in ("parent_warm", "root_warm"):
            if key in cpu:
                cb[key] = _r(cpu[key]["value"])
        rt = cpu.get("reference_tree_one_core")
        if rt:
            cb["reference_tree_one_core"] = {"value": _r(rt["value"]), "nodes": rt["nodes"],
                                             "seconds": _r(rt["seconds"]),
                                             "solved": rt["solved"]}
    oa = {k: _r(v) if isinstance(v, float) else v for k, v in oa_tree.items()
          if not isinstance(v, dict)}
    if "cpu_reference_one_core" in oa_tree:
        c1 = oa_tree["cpu_reference_one_core"]
        oa["cpu_reference_one_core"] = {"value": _r(c1["value"]), "solved": c1["solved"],
                                        "seconds": _r(c1["seconds"])}

    def rate(key, field="nodes_per_s"):
        v = supp.get(key)
        if v is None:
            return None
        if isinstance(v, list):
            return [_r(e.get(field)) for e in v]
        return _r(v.get(field))
    ts = supp.get("tree_search") or []
    line = {
        "metric": "B&B nodes/sec + relaxations solved/sec at 1/2/4/8 MI355X",
        "value": nodes / elapsed,
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": ("config 2 (tls4.nl as a MINLP: its OA-LP) branch-and-bound tree rounds: "
                         "per step and GPU one mgpu_bnb_round = pop the top B open nodes of the "
                         "HBM stack, K1 FBBT, K3P dual simplex from the parent's optimal basis, "
                         "decision + MaxVio, children pushed; then one packed all-reduce "
                         "(incumbent MIN, open counts). Pool = root + B seeded boxes (SURVEY 8d)"
                         if args.warm == 2 else
                         "config 2 tree rounds, root-basis warm starts (K3P), MaxVio"),
            "instance": f"tls4-oa ({p.m} rows, {p.n} cols, {p.nnz} nnz)",
            "nodes_per_gpu": B,
            "global_batch": B * world,
            "parallelism": f"node-sharded x{world}",
        },
        "relaxations_per_s": lps / elapsed,
        "fbbt_node_passes_per_s": float(B) * world / (kf["ms"] * 1e-3),
        "tree_rounds": {k: _r(v) if isinstance(v, float) else v
                        for k, v in h["summary"].items() if k != "search"},
        "rccl_ms_total": _r(h["rccl_ms"]),
        "roofline": rf,
        "kernels": ks,
        "cpu_baseline": cb,
        "tls4_oa_tree": oa,
        "tls4_oa_rel_tree": ({k: (_r(v) if isinstance(v, float) else v)
                              for k, v in rel_tree.items() if k not in ("instance", "search")}
                             if rel_tree else None),
        "supplementary": {
            "file": supp_path,
            "fixed_batch_nodes_per_s": rate("fixed_batch"),
            "tree_search_nodes_per_s": [_r(e["nodes_per_s"]) for e in ts] or None,
            "tree_search_all_optima_match_highs": (all(e["optimum_matches_highs"] for e in ts)
                                                   if ts else None),
            "convex_batch_nodes_per_s": rate("convex_batch"),
            "qp_per_s": rate("qp_relaxation", "qp_per_s"),
            "qp_potrf_roofline_frac": (_r(supp["qp_relaxation"]["roofline"]["frac"])
                                       if isinstance(supp.get("qp_relaxation"), dict)
                                       and "roofline" in supp["qp_relaxation"] else None),
            "qp_tree_nodes_per_s": rate("qp_tree"),
            "knapsack_nodes_per_s": rate("knapsack_nodes"),
            "glob_batch_nodes_per_s": rate("glob_batch"),
            "glob_tree_nodes_per_s": rate("glob_tree"),
        },
    }
    # keep the line under the driver's limit whatever the supplementary holds
    for drop in ("supplementary", "tree_rounds", "tls4_oa_rel_tree", "tls4_oa_tree"):
        if len(json.dumps(line)) <= LINE_MAX:
            break
        line[drop] = "see " + str(supp_path)
    return line


def progress(rank, msg):
    """One line per phase on stderr (the JSON line stays alone on stdout)."""
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def launch_ranks(n):
    """Run this bench as N rank processes through torch.distributed.run on
    127.0.0.1 (the driver's own multi-GPU launch) and return its exit code.
    A child process, not an exec: the ranks' stdout is this process's
    stdout, so rank 0's JSON line is the one line printed."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={n}', '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    progress(0, f"launching {n} ranks: {' '.join(cmd[2:])}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=524288,
                    help='open nodes per GPU per step (524288: K1 persistent waves refill '
                         'their lanes; 131072 = one node per resident lane)')
    ap.add_argument('--tree-batch', type=int, default=131072,
                    help='open nodes per GPU per round of the complete trees (tree_search, '
                         'convex_batch)')
    ap.add_argument('--oa-tree-batch', type=int, default=16384,
                    help="open nodes per GPU per round of config 2's complete tree "
                         "(tls4_oa_tree in the line)")
    ap.add_argument('--supp-out', default=os.path.join('gpurun_out', 'bench_supplementary.json'),
                    help='where the supplementary objects (trees, configs 3/4/5, glob) are '
                         'written; the stdout line carries their headline numbers only')
    ap.add_argument('--oa-tree-eta-cap', type=int, default=48,
                    help="K3P eta-file cap of config 2's complete tree (32 / 48 builds)")
    ap.add_argument('--lb-pick', choices=('reference', 'batch'), default='reference',
                    help="N > 1 headline: candidates each rank offers per rebalance: the "
                         "reference's 50 P (default) or max(50 P, batch)")
    ap.add_argument('--warm', type=int, default=2,
                    help='headline tree warm starts: 2 parent basis as a pivot path (default; '
                         'NodeIncRelaxer semantics), 0 the root basis')
    ap.add_argument('--lb-every', type=int, default=8,
                    help='N > 1: rebalance the open nodes across the ranks every this many '
                         'headline rounds (dist.rebalance; 0 = never)')
    ap.add_argument('--cpu-seconds', type=float, default=16.0)
    ap.add_argument('--cpu-pool-nodes', type=int, default=65536,
                    help="open nodes (with their parent bases) exported after the headline's "
                         "timed rounds for the all-cores CPU baseline")
    ap.add_argument('--tree-cpu-seconds', type=float, default=3.0,
                    help="time_limit of each tree_search entry's one-core reference tree")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-bnb', action='store_true',
                    help='skip the supplementary full tree search (mkp MILP)')
    ap.add_argument('--no-convex', action='store_true',
                    help='skip the supplementary convex batch (config 5, knapsack OA trees)')
    ap.add_argument('--no-qp', action='store_true',
                    help='skip the supplementary QP relaxation batch (color_lab2, MFMA KKT)')
    ap.add_argument('--no-glob', action='store_true',
                    help='skip the supplementary glob batch (QCQP: K2 -> per-node rows LP)')
    ap.add_argument('--no-fixed', action='store_true',
                    help='skip the supplementary fixed batch (K1 + K3P on tls4-lin boxes)')
    ap.add_argument('--no-oa-tree', action='store_true',
                    help="skip config 2's complete tree (tls4_oa_tree; profiling runs)")
    ap.add_argument('--eta-cap', type=int, default=PFI_DEFAULT,
                    help="K3P's eta-file cap for the headline rounds (32; 33-48 select "
                         'the 48-eta build)')
    ap.add_argument('--no-knapsack', action='store_true',
                    help='skip the supplementary config-3 batch (1000 knapsack nodes)')
    args = ap.parse_args()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # `python bench.py --gpus N`: this process only launches; N fresh rank
        # processes (one per GPU) run the bench and rank 0 prints the line.
        # Nothing here touches the GPU (no torch import), so the ranks start
        # from a clean device state.
        sys.exit(launch_ranks(args.gpus))
    global COMM

    import torch
    import torch.distributed as dist
    from minotaur_amd import dist as mdist
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context

    rank, world, local = mdist.env_ranks()
    if args.gpus != world:
        progress(rank, f"--gpus {args.gpus} but WORLD_SIZE {world}: running {world} ranks")
    # MGPU_BENCH_REHEARSAL=1 (test hook): every rank on device 0, to rehearse
    # the N>1 path on a one-GPU box (RCCL refuses a shared device: the
    # engine's collectives run over its host transport, gloo underneath)
    rehearse = os.environ.get('MGPU_BENCH_REHEARSAL') == '1'
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    comm_mode = os.environ.get('MGPU_COMM', 'host' if rehearse else 'rccl')
    if world > 1:
        if comm_mode == 'torch':
            dist.init_process_group('nccl', device_id=dev)
        else:
            # the rendezvous of torch.distributed.run (and the host transport's
            # gloo); the round collectives themselves are the engine's
            dist.init_process_group('gloo')

    ctx = Context(local)
    # one dedicated stream for the engine AND the torch glue (the legacy null
    # stream would not order against the engine's non-blocking stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    COMM = mdist.make_comm(ctx, rank, world, dev)
    progress(rank, f"{world} rank(s), round collectives: "
                   f"{type(COMM).__name__}/{getattr(COMM, 'transport', 'torch')}")

    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = args.batch
    # ONE pool: the root (rank 0) plus B * world seeded boxes, dealt
    # round-robin (MpiBranchAndBound.cpp:142-188); B per rank (weak scaling)
    LB, UB = random_boxes(p, B * world, 20261017)
    LB, UB = LB[rank::world].copy(), UB[rank::world].copy()
    h = tree_rounds(ctx, dev, rank, world, p, LB, UB, args)
    ctx.set_lp_pfi(PFI_DEFAULT)
    elapsed, nodes, lps = h["elapsed"], h["nodes"], h["lps"]
    progress(rank, f"headline done: {1e3 * elapsed / args.steps:.2f} ms/step, "
                   f"{nodes / elapsed / 1e6:.2f} M nodes/s")
    TB = args.tree_batch
    oa_tree = {} if args.no_oa_tree else tls4_oa_tree(ctx, dev, rank, world, args)
    progress(rank, f"tls4_oa_tree done: {oa_tree.get('nodes_per_s', 0.0) / 1e6:.2f} M nodes/s")
    rel_tree = {} if args.no_oa_tree else tls4_oa_rel_tree(ctx, dev, rank, world, args)
    progress(rank, f"tls4_oa_rel_tree done: {rel_tree}")
    supp = {}
    for key, skip, fn in (
            ("fixed_batch", args.no_fixed, lambda: fixed_batch(ctx, dev, rank, world, args)),
            ("tree_search", args.no_bnb, lambda: tree_search(ctx, dev, rank, world, TB, args)),
            ("convex_batch", args.no_convex,
             lambda: convex_batch(ctx, dev, rank, world, TB, args)),
            ("qp_relaxation", args.no_qp, lambda: qp_relaxation(ctx, dev, rank, world, args)),
            ("qp_tree", args.no_qp, lambda: qp_tree(ctx, dev, rank, world, args)),
            ("knapsack_nodes", args.no_knapsack,
             lambda: knapsack_nodes(ctx, dev, rank, world, args)),
            ("glob_batch", args.no_glob, lambda: glob_batch(ctx, dev, rank, world, args)),
            ("glob_tree", args.no_glob, lambda: glob_tree(ctx, dev, rank, world, args))):
        supp[key] = None if skip else fn()
        progress(rank, f"{key} done")

    if rank == 0:
        kernels = h["kernels"]
        dom = max(("fbbt", "lp_pfi"), key=lambda k: kernels[k]["ms"])
        kd = kernels[dom]
        traffic, tsrc, fresh = pmc_traffic(dom, B, args.eta_cap, tree=True)
        roofline = {"kernel": dom, "bound": "hbm" if dom == "fbbt" else "fp64",
                    "achieved": kd["achieved"], "peak": kd["peak"], "unit": kd["unit"],
                    "frac": kd["frac"], "traffic": traffic}
        if tsrc:
            roofline["traffic_source"] = (f"profiles/{tsrc} (PMC, bytes per launch; " +
                                          {True: "same engine sources)",
                                           False: "STALE: measured on other engine sources)",
                                           None: "engine sources not recorded)"}[fresh])
        if dom != "fbbt":
            roofline["note"] = ("FP64 VALU (no MFMA: per-node pivots); achieved = SURVEY 8(d) "
                                "2m(n+m) flops per pivot K3P ran / its HIP-event time")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(p, LB, UB, args.cpu_seconds, "tls4-oa",
                               pool=(h["pool_sample"], h["incumbent"], args.eta_cap))
            # the same instance's tree on one core by the reference's own
            # BranchAndBound (nodes/s like value; not the same node boxes)
            cpu["reference_tree_one_core"] = tree_cpu_baseline(p, 0, 2 * args.tree_cpu_seconds)
        full = {"headline_kernels": kernels, "cpu_baseline": cpu, "tls4_oa_tree": oa_tree,
                "tls4_oa_rel_tree": rel_tree}
        full.update(supp)
        supp_path = os.path.abspath(args.supp_out)
        try:
            os.makedirs(os.path.dirname(supp_path), exist_ok=True)
            with open(supp_path, 'w') as fh:
                json.dump(full, fh, indent=1)
        except OSError as e:
            supp_path = f"not written ({e})"
        line = compact_line(args, world, B, p, h, elapsed, nodes, lps, roofline, kernels, cpu,
                            oa_tree, supp, supp_path, rel_tree)
        if rehearse:
            line["rehearsal"] = "all ranks on device 0 over gloo (not a scaling number)"
        print(json.dumps(line), flush=True)
    COMM = None
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
