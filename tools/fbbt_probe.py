"""Quick GPU timing sweep of K1 (batched FBBT) on tls4-lin: device time per
batch from hipEvents around the launch, both kernel variants."""
import math
import os
import sys
import time

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
    LB0, UB0 = random_boxes(p, 4096, 20261015)
    for B in [64, 256, 1024, 4096, 16384, 65536, 262144]:
        reps = (B + 4095) // 4096
        LB = np.tile(LB0, (reps, 1))[:B]
        UB = np.tile(UB0, (reps, 1))[:B]
        lb = torch.from_numpy(LB).to(dev)
        ub = torch.from_numpy(UB).to(dev)
        olb = torch.empty_like(lb)
        oub = torch.empty_like(ub)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        for variant in (1, 2):
            ctx.set_fbbt_variant(variant)
            for inc in (math.inf, 20.0):
                ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, inc)
                ctx.sync()
                t0 = time.perf_counter()
                K = 5
                ms = []
                for _ in range(K):
                    ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, inc)
                    ctx.sync()
                    ms.append(ctx.last_kernel_ms('fbbt'))
                wall = (time.perf_counter() - t0) / K
                kms = float(np.median(ms))
                print(f"B={B:7d} variant={variant} inc={inc:5} kernel {kms:9.3f} ms "
                      f"wall {wall*1e3:9.3f} ms  {B / (kms * 1e-3) / 1e6:9.2f} Mnodes/s",
                      flush=True)
    ctx.set_fbbt_variant(0)


if __name__ == '__main__':
    main()
