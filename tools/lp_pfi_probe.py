"""GPU timing of the LP step of the bench (tls4-lin node boxes after FBBT,
warm-started from the root basis): dense K3 against K3P at several eta-file
caps (K3P time includes the dense re-solve of its overflow list)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402
from minotaur_amd.runtime import LP_PFI_MAX, Context, WarmStart  # noqa: E402


def main():
    B = int(os.environ.get('PROBE_B', 131072))
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
    modes = [(1, LP_PFI_MAX)] + [(0, k) for k in (LP_PFI_MAX, 12, 8)]
    if os.environ.get('PROBE_MODES'):   # e.g. "0:24" (variant:kmax, comma separated)
        modes = [tuple(int(v) for v in mkv.split(':')) for mkv in
                 os.environ['PROBE_MODES'].split(',')]
    ref = None
    for variant, kmax in modes:
        ctx.set_lp_variant(variant)
        ctx.set_lp_pfi(kmax)
        ms = []
        for _ in range(5):
            ctx.lp_solve_dev(lb, ub, st, obj, it, ws=ws, skip=inf)
            ctx.sync()
            ms.append(ctx.last_kernel_ms('lp'))
        k = float(np.median(ms))
        o = obj.cpu().numpy()
        if ref is None:
            ref = o.copy()
        fin = np.isfinite(ref)
        dev_obj = float(np.max(np.abs(o[fin] - ref[fin]))) if fin.any() else 0.0
        over = int((it > kmax).sum().item()) if variant == 0 else 0
        name = 'K3 dense' if variant == 1 else f'K3P kmax={kmax:2d}'
        print(f"{name}: {k:7.3f} ms  {B / k / 1e3:7.2f} M LP/s  overflow {over:6d}  "
              f"max|dobj| vs dense {dev_obj:.2e}", flush=True)
    ctx.set_lp_variant(0)
    ctx.set_lp_pfi(LP_PFI_MAX)


if __name__ == '__main__':
    main()
