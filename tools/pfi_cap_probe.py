"""K3P eta-file cap A/B on the bench's two node workloads (GPU box):

* the headline's tree rounds on tls4-oa (deep nodes: 15-20 pivots from the
  root basis), a few rounds per cap;
* the fixed batch of tls4-lin boxes (5.9 pivots on average).

Prints one JSON line per (workload, cap): per-round K3P main / overflow /
LP-call ms and nodes/s.  Usage: python tools/pfi_cap_probe.py [caps...]
"""
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)


def main():
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context
    caps = [int(a) for a in sys.argv[1:]] or [16, 24, 32]
    dev = torch.device('cuda', 0)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = int(os.environ.get('PROBE_BATCH', '524288'))
    LB, UB = random_boxes(p, B, 20261017)
    for cap in caps:
        ctx.load(p)
        ctx.set_lp_pfi(cap)
        ctx.bnb_config(0, 0)
        ctx.bnb_brancher(0)
        ctx.bnb_init(B * 10 + 2)
        ctx.bnb_import(LB, UB, np.full(B, -math.inf), np.zeros(B, dtype=np.int32))
        rows = []
        for r in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = ctx.bnb_round(B)
            torch.cuda.synchronize()
            rows.append({"round": r, "ms": 1e3 * (time.perf_counter() - t0),
                         "fbbt_ms": ctx.last_kernel_ms('fbbt'),
                         "k3p_ms": ctx.last_kernel_ms('lp_main'),
                         "ovf_ms": ctx.last_kernel_ms('lp_tail'),
                         "lp_ms": ctx.last_kernel_ms('lp'), "nodes": st.nodes, "lps": st.lps,
                         "pivots": st.pivots, "pfi_pivots": st.pfi_pivots})
        print(json.dumps({"workload": "tree_rounds", "cap": cap, "rounds": rows}), flush=True)




def iter_census(rounds=4, cap=16):
    """Per-LP pivot counts of the next batch after each tree round: the top
    B boxes are exported (and put back unchanged), FBBT'd with the round's
    incumbent and solved from the root basis; LPs with > 200 pivots are saved
    for the CPU oracle (gpurun_out/pfi_census_long.npz)."""
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context
    ctx = Context(0)
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = int(os.environ.get('PROBE_BATCH', '524288'))
    LB, UB = random_boxes(p, B, 20261017)
    ctx.load(p)
    ctx.set_lp_pfi(cap)
    root, ws = ctx.root_solve()
    ctx.bnb_config(0, 0)
    ctx.bnb_brancher(0)
    ctx.bnb_init(B * (rounds + 3) + 2)
    ctx.bnb_import(LB, UB, np.full(B, -math.inf), np.zeros(B, dtype=np.int32))
    inc = math.inf
    longs = []
    for r in range(rounds):
        lb, ub, nlb, dep = ctx.bnb_export(B)
        ctx.bnb_import(lb, ub, nlb, dep)
        f = ctx.fbbt(lb, ub, inc)
        keep = f.infeasible == 0
        t0 = time.perf_counter()
        o = ctx.lp_solve(f.lb[keep], f.ub[keep], ws)
        dt = time.perf_counter() - t0
        it = o.iters
        big = np.nonzero(it > 200)[0]
        print(json.dumps({"census_round": r, "lps": int(keep.sum()), "s": dt,
                          "mean": float(it.mean()), "max": int(it.max()),
                          "p99": float(np.percentile(it, 99)), "gt32": float((it > 32).mean()),
                          "gt200": int(big.size), "status": np.bincount(o.status).tolist()}),
              flush=True)
        for i in big[:64]:
            longs.append((f.lb[keep][i], f.ub[keep][i], int(it[i]), int(o.status[i])))
        st = ctx.bnb_round(B, inc)
        inc = min(inc, st.incumbent)
    if longs:
        os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
        np.savez(os.path.join(ROOT, 'gpurun_out', 'pfi_census_long.npz'),
                 lb=np.stack([a for a, _, _, _ in longs]), ub=np.stack([b for _, b, _, _ in longs]),
                 iters=np.array([c for _, _, c, _ in longs]),
                 status=np.array([d for _, _, _, d in longs]))


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'census':
        iter_census(cap=int(sys.argv[2]) if len(sys.argv) > 2 else 16)
    else:
        main()
