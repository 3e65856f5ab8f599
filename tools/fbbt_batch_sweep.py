"""K1 variants against batch size on config 2's instance (tls4-oa, random-
branching boxes, with and without an incumbent): the auto choice of
mgpu_fbbt_dev (K1: LDS / global / persistent lane-per-node), the persistent
K1 (variant 3) and K1G with 16 / 8 / 4 lanes per node (variants 4 / 5 / 6).
Median kernel ms of 5 launches.

    python tools/fbbt_batch_sweep.py
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


VARIANTS = (0, 3, 4, 5, 6)


def main():
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx = Context(0)
    ctx.load(p)
    dev = torch.device('cuda', 0)
    LBa, UBa = random_boxes(p, 524288, 20261017)
    for B in (1024, 4096, 16384, 65536, 262144, 524288):
        lb = torch.from_numpy(LBa[:B]).to(dev)
        ub = torch.from_numpy(UBa[:B]).to(dev)
        lo, uo = torch.empty_like(lb), torch.empty_like(ub)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        row = [B]
        for inc in (math.inf, 3.2):
            for v in VARIANTS:
                ctx.set_fbbt_variant(v)
                ms = []
                for _ in range(5):
                    ctx.fbbt_dev(lb, ub, lo, uo, inf, nm, inc)
                    torch.cuda.synchronize()
                    ms.append(ctx.last_kernel_ms('fbbt'))
                row.append(round(float(np.median(ms)), 3))
        ctx.set_fbbt_variant(0)
        print("B %7d " % B + "  ".join(
            "%s v%d %.3f" % ("inc" if i >= len(VARIANTS) else "noinc", VARIANTS[i % len(VARIANTS)], t)
            for i, t in enumerate(row[1:])), flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
