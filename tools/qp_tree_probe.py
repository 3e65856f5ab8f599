"""How deep the color_lab2 QP tree must dive for a first incumbent: batched
depth-first rounds of K1 + K5, batch and round cap from argv."""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd import qp as qpm  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
ctx = Context(0)
for B, R in [(16, 400), (64, 400), (256, 200)]:
    t0 = time.perf_counter()
    obj, x, st, secs = qpm.solve_tree(ctx, P, batch=B, capacity=1 << 18, max_rounds=R)
    print(f"B={B} rounds={st.rounds} nodes={st.nodes} open={st.open} incumbent={obj} "
          f"dec={list(st.ndec)} secs={secs:.3f} wall={time.perf_counter() - t0:.2f}", flush=True)
