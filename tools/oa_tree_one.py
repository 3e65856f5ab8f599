"""Config 2's complete MaxVio tree as the bench runs it (tls4-OA, batch
16384, depth-first, parent bases, the 48-eta K3P build), twice: a target
for a kernel trace of its rounds."""
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
ctx.set_lp_pfi(48)
for k in range(2):
    t = time.perf_counter()
    o, x, st, _ = bnb.solve(ctx, batch=16384, capacity=1 << 20, order=0, warm=2)
    print(k, st.rounds, st.nodes, f"{(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
ctx.close()
