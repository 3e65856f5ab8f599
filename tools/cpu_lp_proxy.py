"""Is the CPU LP baseline a strawman?  

Clp is unavailable, so the CPU baseline's LP leg is this repo's bounded dual
simplex restatement (oracle/lp_dual.c).  This times, on the same tls4-lin
node LPs (after the reference FBBT), one core each:

  * scipy HiGHS (linprog method='highs', cold: HiGHS has no warm start
    through scipy) — total per call, and the same with an empty LP to
    estimate scipy's per-call overhead;
  * the restatement cold (slack basis) and warm (root basis, as the bench).

Writes profiles/<tag>_cpu_lp_proxy.json (run in this container or on the GPU
box's host: python tools/cpu_lp_proxy.py [tag] [nodes]).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402
from bench import host_cpu  # noqa: E402
from minotaur_amd.problem import LinProblem, from_rows, random_boxes  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r02'
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    LB, UB = random_boxes(p, N, 20261015)
    f = oracle.linear_fbbt(p, LB, UB)
    keep = f.infeas == 0
    lb, ub = f.lb[keep], f.ub[keep]
    n_lp = int(keep.sum())
    _, _, _, _, _, ws = oracle.dual_simplex_root(p)

    t0 = time.perf_counter()
    hs = np.array([oracle.highs(p, lb[b], ub[b])[1] for b in range(n_lp)])
    t_highs = time.perf_counter() - t0
    # scipy per-call overhead: a 1-variable LP through the same wrapper
    tiny = from_rows('tiny', 1, [[(0, 1.0)]], [0.0], [1.0], [0.0], [1.0], [4], [1.0])
    t0 = time.perf_counter()
    for _ in range(n_lp):
        oracle.highs(tiny)
    t_over = time.perf_counter() - t0

    t0 = time.perf_counter()
    sc, oc, ic, _ = oracle.dual_simplex(p, lb, ub, None, nthreads=1)
    t_cold = time.perf_counter() - t0
    t0 = time.perf_counter()
    sw, ow, iw, _ = oracle.dual_simplex(p, lb, ub, ws, nthreads=1)
    t_warm = time.perf_counter() - t0
    ok = sc == 0
    err = float(np.max(np.abs(oc[ok] - hs[ok]) / np.maximum(1.0, np.abs(hs[ok]))))
    model, _ = host_cpu()
    out = {
        "instance": f"tls4-lin ({p.m} rows, {p.n} cols)", "node_lps": n_lp,
        "cpu_model": model, "cores": 1,
        "highs_scipy_us_per_lp": 1e6 * t_highs / n_lp,
        "scipy_call_overhead_us": 1e6 * t_over / n_lp,
        "highs_net_us_per_lp": 1e6 * (t_highs - t_over) / n_lp,
        "restatement_cold_us_per_lp": 1e6 * t_cold / n_lp,
        "restatement_cold_pivots_per_lp": float(ic.mean()),
        "restatement_warm_us_per_lp": 1e6 * t_warm / n_lp,
        "restatement_warm_pivots_per_lp": float(iw.mean()),
        "max_rel_obj_diff_vs_highs": err,
        "note": ("HiGHS net = HiGHS through scipy minus scipy's per-call overhead (timed on a "
                 "1-variable LP); HiGHS solves cold (no warm start through scipy), the bench's "
                 "CPU leg warm-starts from the root basis as NodeIncRelaxer does"),
    }
    path = os.path.join(ROOT, 'profiles', f'{tag}_cpu_lp_proxy.json')
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
