"""Which node LP optima are degenerate or non-unique?

Clp is absent, so LP parity is pinned on statuses and objectives; where an
optimum is non-unique the vertex (and so the integrality verdict and the
branching variable) of any two simplex codes may legitimately differ.  This
counts, over the golden LP sets and over bench boxes, the optimal node LPs
whose final basis (the dense restatement, warm-started from the root basis
as the bench does) is
  * primal degenerate: a basic column sits at one of its bounds;
  * dual degenerate (non-unique primal optimum possible): a nonbasic column
    that is not fixed has a zero reduced cost;
with tolerance 1e-9.  Writes profiles/<tag>_degeneracy.json.
Usage: python tools/degeneracy_census.py [tag]"""
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import oracle  # noqa: E402
from golden_io import load_lp  # noqa: E402
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402

TOL = 1e-9


def census(p, LB, UB):
    st0, _, _, _, _, ws = oracle.dual_simplex_root(p)
    if st0 != 0:
        return None
    B = LB.shape[0]
    tile = oracle.WarmStart(np.tile(ws.head, (B, 1)), np.tile(ws.st, (B, 1)),
                            np.tile(ws.binv, (B, 1, 1)), np.tile(ws.d, (B, 1)))
    st, obj, it, x, wo = oracle.dual_simplex_nodes(p, LB, UB, tile)
    A = p.dense()
    opt = np.nonzero(st == 0)[0]
    prim = dual = both = 0
    for b in opt:
        act = A @ x[b]
        val = np.concatenate([x[b], act])
        lo = np.concatenate([LB[b], p.rlo])
        hi = np.concatenate([UB[b], p.rhi])
        basic = wo.head[b]
        at_bound = (np.abs(val[basic] - lo[basic]) <= TOL * np.maximum(1, np.abs(lo[basic]))) | \
                   (np.abs(val[basic] - hi[basic]) <= TOL * np.maximum(1, np.abs(hi[basic])))
        pd = bool(at_bound.any())
        nonbasic = np.setdiff1d(np.arange(p.n + p.m), basic)
        free_nb = nonbasic[hi[nonbasic] - lo[nonbasic] > TOL]
        dd = bool(np.any(np.abs(wo.d[b][free_nb]) <= TOL))
        prim += pd
        dual += dd
        both += pd and dd
    return {"instance": p.name, "lps": int(B), "optimal": int(opt.size),
            "primal_degenerate": int(prim), "dual_degenerate_nonunique": int(dual),
            "both": int(both)}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r02'
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, 'tests', 'golden', 'lp_*.npz'))):
        name = os.path.basename(f)[3:-4]
        p, g = load_lp(name)
        r = census(p, g['lb'], g['ub'])
        if r:
            r["set"] = f"tests/golden/lp_{name}.npz"
            out.append(r)
            print(r)
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    LB, UB = random_boxes(p, 4096, 20261015)
    f = oracle.linear_fbbt(p, LB, UB)
    keep = f.infeas == 0
    r = census(p, f.lb[keep], f.ub[keep])
    r["set"] = "bench boxes (first 4096 rank-0 tls4-lin boxes after FBBT)"
    out.append(r)
    print(r)
    with open(os.path.join(ROOT, 'profiles', f'{tag}_degeneracy.json'), 'w') as fh:
        json.dump({"tolerance": TOL, "sets": out}, fh, indent=1)


if __name__ == '__main__':
    main()
