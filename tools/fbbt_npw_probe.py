"""K1 timing vs nodes per wave (MGPU_FBBT_NPW) and variant, tls4-lin."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def main():
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    ctx = Context(0)
    ctx.load(p)
    dev = torch.device('cuda', 0)
    for B in [65536, 262144]:
        LB, UB = random_boxes(p, B, 20261015)
        lb = torch.from_numpy(LB).to(dev)
        ub = torch.from_numpy(UB).to(dev)
        olb = torch.empty_like(lb)
        oub = torch.empty_like(ub)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        ref = None
        for npw in (64, 32, 16, 8):
            os.environ['MGPU_FBBT_NPW'] = str(npw)
            for variant in (2, 1):
                ctx.set_fbbt_variant(variant)
                ms = []
                for _ in range(4):
                    ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, math.inf)
                    ctx.sync()
                    ms.append(ctx.last_kernel_ms('fbbt'))
                out = olb.cpu().numpy()
                if ref is None:
                    ref = out
                same = np.array_equal(out.view(np.int64), ref.view(np.int64))
                k = float(np.median(ms[1:]))
                print(f"B={B:7d} npw={npw:3d} variant={variant} {k:8.3f} ms "
                      f"{B / k / 1e3:8.2f} M nodes/s same={same}", flush=True)
    ctx.set_fbbt_variant(0)


if __name__ == '__main__':
    main()
