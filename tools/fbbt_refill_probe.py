"""K1 persistent-refill variant (3) against the one-node-per-lane global
variant (2): bit-exact outputs and kernel time over batch sizes and
persistent grid sizes (MGPU_FBBT_WAVES), tls4-lin, with and without an
incumbent.  Usage: python tools/fbbt_refill_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)


def main():
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    ctx = Context(0)
    ctx.load(p)
    dev = torch.device('cuda', 0)
    for B in [int(b) for b in os.environ.get('PROBE_B', '131072,262144,524288').split(',')]:
        LB, UB = random_boxes(p, B, 20261015)
        lb = torch.from_numpy(LB).to(dev)
        ub = torch.from_numpy(UB).to(dev)
        olb, oub = torch.empty_like(lb), torch.empty_like(ub)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        for inc in (float('inf'), 11.3):
            ref = None
            cfgs = [(int(a), int(b)) for a, b in (c.split(':') for c in os.environ.get(
                'PROBE_CFG', '2:0,3:1024,3:2048,3:3072,3:4096').split(','))]
            for variant, waves in cfgs:
                if waves:
                    os.environ['MGPU_FBBT_WAVES'] = str(waves)
                ctx.set_fbbt_variant(variant)
                ms = []
                for _ in range(4):
                    ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, inc)
                    ctx.sync()
                    ms.append(ctx.last_kernel_ms('fbbt'))
                out = (olb.cpu().numpy().view(np.int64).copy(), oub.cpu().numpy().view(np.int64).copy(),
                       inf.cpu().numpy().copy(), nm.cpu().numpy().copy())
                if ref is None:
                    ref = out
                same = all(np.array_equal(a, b) for a, b in zip(out, ref))
                k = float(np.median(ms[1:]))
                print(f"{os.environ.get('PROBE_TAG', ''):8s} B={B:7d} inc={inc:5} variant={variant} waves={waves:5d} {k:8.3f} ms "
                      f"{B / k / 1e3:8.2f} M nodes/s same={same}", flush=True)
    ctx.set_fbbt_variant(0)


if __name__ == '__main__':
    main()
