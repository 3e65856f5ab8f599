"""A/B of the reliability tree's strong-branching launches (mgpu_set_sb_chain):
config 2's tls4-OA tree as bench.py's tls4_oa_rel_tree runs it (best-first,
parent warm starts, reliability branching, growth 2), timed with chained
launches (1) and per-position launches (0), alternating, after a warm-up of
each.  Prints one JSON line per run and a summary."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from minotaur_amd import bnb  # noqa: E402
from minotaur_amd.problem import LinProblem  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx = Context(0)
    ctx.load(p)
    res = {0: [], 1: []}
    for chain in (1, 0):   # warm-up of each mode
        ctx.set_sb_chain(chain)
        bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1, brancher=1, growth=2)
    torch.cuda.synchronize()
    for _ in range(reps):
        for chain in (1, 0):
            ctx.set_sb_chain(chain)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            obj, _, st, _ = bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1,
                                      brancher=1, growth=2)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            res[chain].append(el)
            print(json.dumps({"chain": chain, "seconds": el, "nodes": st.nodes, "rounds": st.rounds,
                              "sb_lps": st.sb_lps, "sb_pivots": st.sb_pivots, "optimum": obj}),
                  flush=True)
    ctx.set_sb_chain(1)
    ctx.close()
    print(json.dumps({"median_chain_s": sorted(res[1])[len(res[1]) // 2],
                      "median_steps_s": sorted(res[0])[len(res[0]) // 2]}), flush=True)


if __name__ == '__main__':
    main()
