"""One tls4-OA reliability tree (best-first; argv: batch cap, warm, growth)
after a warm-up solve, for a kernel trace of its rounds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from minotaur_amd import bnb  # noqa: E402
from minotaur_amd.problem import LinProblem  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

ctx = Context(0)
p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
ctx.load(p)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
growth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for k in range(2):
    t = time.perf_counter()
    o, x, st, _ = bnb.solve(ctx, batch=B, capacity=1 << 20, order=1, warm=warm, brancher=1,
                            growth=growth)
    print(k, st.rounds, st.nodes, st.sb_lps, f"{(time.perf_counter() - t) * 1e3:.1f} ms",
          flush=True)
ctx.close()
