"""A/B on the CPU restatement: the batched tree's warm mode 2 with node
warm starts kept as pivot paths from the root basis (round 3) vs as the
parent's basis (statuses + the basic columns outside the root basis, rebuilt
by column replacement; round 4).  Rounds of the headline's shape (root plus B
seeded random-branching boxes, depth-first over batches) on tls4-oa at a
reduced batch; prints pivots per LP, warm-start lengths and the LPs whose
warm start plus own pivots overflow the eta file.

    python tools/basis_ws_probe.py [--batch 4096] [--rounds 8] [--inherit 24]
"""
import argparse
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

import oracle  # noqa: E402
import bnb as obnb  # noqa: E402  (oracle/bnb.py)
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402


def run(p, LB, UB, batch, rounds, pivots_mode, inherit, pfi=32):
    oracle.lib().orc_set_path_pivots(int(pivots_mode))
    obnb.PATH_INHERIT = inherit
    stats = {"k": [], "iters": [], "ovf": 0, "lps": 0}
    real = oracle.dual_simplex_path

    def spy(p_, LB_, UB_, ws, k_in, path_in, st_in, pfi_, inh, **kw):
        out = real(p_, LB_, UB_, ws, k_in, path_in, st_in, pfi_, inh, **kw)
        ok = out[0] != 12
        stats["k"].append(np.asarray(k_in)[ok])
        stats["iters"].append(out[2][ok])
        stats["ovf"] += int(((np.asarray(k_in) + out[2]) > pfi_)[ok].sum())
        stats["lps"] += int(ok.sum())
        return out
    oracle.dual_simplex_path = spy
    try:
        c = obnb.CpuBnbContext(p, pfi, order=0, warm=2)
        c.bnb_init(1 << 22)
        c.pool += [obnb._Node(LB[i].copy(), UB[i].copy(), -math.inf, 0, c.ws)
                   for i in range(LB.shape[0])]
        t0 = time.perf_counter()
        inc = math.inf
        for _ in range(rounds):
            st = c.bnb_round(batch, inc)
            inc = st.incumbent
        el = time.perf_counter() - t0
    finally:
        oracle.dual_simplex_path = real
    k = np.concatenate(stats["k"])
    it = np.concatenate(stats["iters"])
    return {"mode": "pivot paths" if pivots_mode else "bases (column replacement)",
            "nodes": st.nodes, "lps": stats["lps"], "pivots_per_lp": float(it.mean()),
            "warm_len_mean": float(k.mean()), "warm_len_p99": float(np.percentile(k, 99)),
            "from_root_frac": float((k == 0).mean()), "overflow_lps": stats["ovf"],
            "incumbent": inc, "seconds": el}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--rounds', type=int, default=8)
    ap.add_argument('--inherit', type=int, default=24)
    a = ap.parse_args()
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    LB, UB = random_boxes(p, a.batch, 20261017)
    for mode in (1, 0):
        print(run(p, LB, UB, a.batch, a.rounds, mode, a.inherit), flush=True)


if __name__ == '__main__':
    main()
