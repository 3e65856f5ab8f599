"""GPU timing of K3 alone: tls4-lin node boxes (FBBT applied first, as in
the bench), warm-started from the root basis; kernel ms from hipEvents."""
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402
from minotaur_amd.runtime import Context, WarmStart  # noqa: E402


def main():
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    ctx = Context(0)
    ctx.load(p)
    root, wsh = ctx.root_solve()
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    ws = WarmStart(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (wsh.head, wsh.st, wsh.d, wsh.binv)))
    for B in [4096, 16384, 65536, 262144]:
        LB, UB = random_boxes(p, B, 20261015)
        lb0 = torch.from_numpy(LB).to(dev)
        ub0 = torch.from_numpy(UB).to(dev)
        lb = torch.empty_like(lb0)
        ub = torch.empty_like(ub0)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        obj = torch.zeros(B, dtype=torch.float64, device=dev)
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx.fbbt_dev(lb0, ub0, lb, ub, inf, nm)
        ms = []
        for _ in range(5):
            ctx.lp_solve_dev(lb, ub, st, obj, it, ws=ws, skip=inf)
            ctx.sync()
            ms.append(ctx.last_kernel_ms('lp'))
        k = float(np.median(ms))
        piv = int(it.sum().item())
        print(f"B={B:7d} lp kernel {k:8.3f} ms  {B / k / 1e3:8.2f} M LP/s  pivots/LP "
              f"{piv / max(1, int((st != 12).sum().item())):.2f}", flush=True)


if __name__ == '__main__':
    main()
