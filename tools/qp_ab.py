"""K5 timing probe for A/B builds (MGPU_LIB selects the library): color_lab2
node boxes, per-kernel times (qp_potrf / qp_trsm / qp_step) and QP/s."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd import qp as qpm  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
ctx = Context(0)
ctx.load_qp(P)
LB, UB = qpm.random_node_boxes(P, B, 17)
ctx.qp_solve(LB[:8], UB[:8])
ctx.set_qp_ktime(1)
for _ in range(3):
    st, ob, it, x = ctx.qp_solve(LB, UB)
    ms = ctx.last_kernel_ms('qp')
    print(f"{os.environ.get('TAG', '')} B={B} ok={int((st == 0).sum())} iters={int(it.sum())} "
          f"{ms:.3f} ms {B / ms * 1e3:.0f} QP/s potrf {ctx.last_kernel_ms('qp_potrf'):.3f} "
          f"trsm {ctx.last_kernel_ms('qp_trsm'):.3f} step {ctx.last_kernel_ms('qp_step'):.3f} "
          f"obj0 {ob[0]!r}", flush=True)
