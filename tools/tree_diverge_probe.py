"""Where do the GPU tree and its CPU restatement part ways?  (GPU box)

Runs the CPU restatement (oracle/bnb.py) of a tree round by round, solves
each round's node LPs (the restatement's own inputs) on the GPU with the same
shared root basis and compares status / pivots / objective LP by LP, and runs
the GPU tree (mgpu_bnb_round) beside it comparing the per-round statistics.
The first mismatching LP is saved to gpurun_out/diverge_lp.npz.

Usage: python tools/tree_diverge_probe.py [instance] [order] [batch] [cap]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))


def main():
    import oracle
    import bnb as ob
    from minotaur_amd.problem import LinProblem
    from minotaur_amd.runtime import Context, WarmStart
    name = sys.argv[1] if len(sys.argv) > 1 else 'tls4_oa'
    order = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    cap = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', f'{name}.npz'))
    ctx = Context(0)
    ctx.load(p)
    ctx.set_lp_pfi(cap)
    rec = []
    orig = oracle.dual_simplex

    def spy(P, lb, ub, ws, *a, **k):
        r = orig(P, lb, ub, ws, *a, **k)
        rec.append((np.array(lb), np.array(ub), r))
        return r
    ob.oracle.dual_simplex = spy
    cpu = ob.CpuBnbContext(p, pfi=cap)
    cpu.bnb_config(order, 0)
    cpu.bnb_init(1 << 20)
    ctx.bnb_config(order, 0)
    ctx.bnb_brancher(0)
    ctx.bnb_init(1 << 20)
    ws = cpu.ws
    gws = WarmStart(ws.head, ws.st, ws.d, np.ascontiguousarray(ws.binv.T))
    first = True
    for rnd in range(10000):
        sc = cpu.bnb_round(batch)
        sg = ctx.bnb_round(batch)
        a = (sc.nodes, list(sc.ndec), sc.lps, sc.pivots)
        b = (sg.nodes, list(sg.ndec), sg.lps, sg.pivots)
        if rec:
            lb, ub, (st, obj, it, _) = rec[-1]
            rec.clear()
            g = ctx.lp_solve(lb, ub, gws)
            bad = np.nonzero((g.status != st) | (g.iters != it) |
                             (np.abs(g.obj - obj) > 1e-9 * np.maximum(1, np.abs(obj))) &
                             (st == 0))[0]
            if bad.size and first:
                i = bad[0]
                print(f"round {rnd}: LP {i} of {len(st)}: cpu st {st[i]} it {it[i]} obj {obj[i]!r}"
                      f" | gpu st {g.status[i]} it {g.iters[i]} obj {g.obj[i]!r}"
                      f" ({bad.size} mismatching)", flush=True)
                os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
                np.savez(os.path.join(ROOT, 'gpurun_out', 'diverge_lp.npz'), lb=lb[bad],
                         ub=ub[bad], st=st[bad], it=it[bad], obj=obj[bad],
                         gst=g.status[bad], git=g.iters[bad], gobj=g.obj[bad])
                first = False
        if a != b:
            print(f"round {rnd}: stats differ cpu {a} gpu {b}", flush=True)
            break
        if sc.open == 0:
            print(f"identical trees: {rnd + 1} rounds, {sc.nodes} nodes", flush=True)
            break


if __name__ == '__main__':
    main()
