"""K5 alone on color_lab2_4x0 node boxes (B from argv, default 1024), two
timed batches: a target for rocprofv3 counter passes over qp_* kernels."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd import qp as qpm  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
ctx = Context(0)
ctx.load_qp(P)
LB, UB = qpm.random_node_boxes(P, B, 17)
ctx.qp_solve(LB[:8], UB[:8])
for _ in range(2):
    st, ob, it, x = ctx.qp_solve(LB, UB)
    print(f"qp B={B} ok={int((st == 0).sum())} iters={int(it.sum())} {ctx.last_kernel_ms('qp'):.3f} ms",
          flush=True)
