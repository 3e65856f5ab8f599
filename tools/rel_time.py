"""Time config 2's reliability tree (tls4-OA; best-first, parent warm starts,
reliability branching, growth 2, as bench.py's tls4_oa_rel_tree) with the
library MGPU_LIB selects: a warm-up solve, then REPS timed solves; prints the
nodes, LPs and the median / min time."""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx = Context(0)
    ctx.load(p)
    bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1, brancher=1, growth=2)
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        obj, _, st, _ = bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1, brancher=1,
                                  growth=2)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{os.path.basename(os.path.dirname(os.environ.get('MGPU_LIB', 'base/x')))}: obj {obj} "
          f"nodes {st.nodes} lps {st.lps} sb_lps {st.sb_lps} pivots {st.pivots} median "
          f"{1e3 * ts[len(ts) // 2]:.2f} ms min {1e3 * ts[0]:.2f} ms", flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
