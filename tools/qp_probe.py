"""GPU timing of K5 (batched QP relaxation, MFMA KKT) on color_lab2_4x0
node boxes: time per batch, IPM iterations, QP solves/s and the MFMA f64
rate of the factorizations (algorithmic flops: n^3/3 Cholesky + n^2 m
TRSM + n m^2 Gram per node per iteration, on the padded sizes)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd import qp as qpm  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def main():
    P = qpm.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'color_lab2_qp.npz'))
    ctx = Context(0)
    ctx.load_qp(P)
    np_, mp = 304, 64
    for B in [64, 256, 1024]:
        LB, UB = qpm.random_node_boxes(P, B, 17)
        ctx.qp_solve(LB[:8], UB[:8])
        t0 = time.perf_counter()
        st, ob, it, x = ctx.qp_solve(LB, UB)
        wall = time.perf_counter() - t0
        ms = ctx.last_kernel_ms('qp')
        iters = it.sum()
        flops = iters * (np_ ** 3 / 3 + np_ ** 2 * mp + np_ * mp ** 2)
        print(f"B={B:5d} ok={int((st == 0).sum())} iters/node={it.mean():.1f} max={it.max()} "
              f"gpu {ms:8.2f} ms wall {wall * 1e3:8.2f} ms  {B / (ms * 1e-3):9.1f} QP/s  "
              f"KKT f64 {flops / (ms * 1e-3) / 1e12:6.3f} TF/s", flush=True)


if __name__ == '__main__':
    main()
