"""K1 timing over (row/term records staged in LDS or read from HBM,
MGPU_FBBT_NOTL) x (nodes per wave, MGPU_FBBT_NPW) x (LDS / global scratch),
tls4-lin, with a bit-exact check against the first configuration.
Usage: python tools/fbbt_variant_probe.py            (spawns both row paths)"""
import math
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)


def run_one(tag):
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context
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
        ref = os.path.join('/tmp', f'fbbt_probe_ref_{B}.npy')
        for npw in (64, 32):
            os.environ['MGPU_FBBT_NPW'] = str(npw)
            for variant in (2, 1):
                ctx.set_fbbt_variant(variant)
                ms = []
                for _ in range(4):
                    ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, 1.2)
                    ctx.sync()
                    ms.append(ctx.last_kernel_ms('fbbt'))
                out = np.concatenate([olb.cpu().numpy().view(np.int64).ravel(),
                                      oub.cpu().numpy().view(np.int64).ravel()])
                if not os.path.exists(ref):
                    np.save(ref, out)
                same = np.array_equal(out, np.load(ref))
                k = float(np.median(ms[1:]))
                print(f"{tag:5s} B={B:7d} npw={npw:3d} variant={variant} {k:8.3f} ms "
                      f"{B / k / 1e3:8.2f} M nodes/s same={same}", flush=True)
    ctx.set_fbbt_variant(0)


if __name__ == '__main__':
    if len(sys.argv) > 1:
        run_one(sys.argv[1])
    else:
        for tag, extra in (('tl', {}), ('notl', {'MGPU_FBBT_NOTL': '1'})):
            env = dict(os.environ, **extra)
            r = subprocess.run([sys.executable, '-u', __file__, tag], env=env)
            if r.returncode != 0:
                sys.exit(r.returncode)
