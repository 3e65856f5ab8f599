"""Do K1 (FBBT of one node batch) and K3P (LPs of another) overlap on two
streams?  Times each alone and both issued together (two engine contexts,
one stream each), tls4-lin, B nodes per batch."""
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
    B = int(os.environ.get('PROBE_B', 131072))
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    dev = torch.device('cuda', 0)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ca, cb = Context(0), Context(0)
    for c, s in ((ca, sa), (cb, sb)):
        c.load(p)
        c.set_stream(s.cuda_stream)
    root, wsh = cb.root_solve()
    ws = WarmStart(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                     for a in (wsh.head, wsh.st, wsh.d, wsh.binv)))
    LB, UB = random_boxes(p, B, 20261015)
    t = lambda a: torch.from_numpy(a).to(dev)
    lb0, ub0 = t(LB), t(UB)
    lb1, ub1, lb2, ub2 = (torch.empty_like(lb0) for _ in range(4))
    i32 = lambda: torch.zeros(B, dtype=torch.int32, device=dev)
    inf1, nm1, inf2, nm2, st, it = i32(), i32(), i32(), i32(), i32(), i32()
    obj = torch.zeros(B, dtype=torch.float64, device=dev)
    ca.fbbt_dev(lb0, ub0, lb2, ub2, inf2, nm2)   # the batch K3P solves
    torch.cuda.synchronize()

    def k1():
        ca.fbbt_dev(lb0, ub0, lb1, ub1, inf1, nm1)

    def k3():
        cb.lp_solve_dev(lb2, ub2, st, obj, it, ws=ws, skip=inf2)

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    a = timed(k1)
    b = timed(k3)
    both = timed(lambda: (k1(), k3()))
    seq = timed(lambda: (k1(), torch.cuda.synchronize(), k3()))
    print(f"B={B}: K1 alone {a:.3f} ms, K3P alone {b:.3f} ms, sequential {seq:.3f} ms, "
          f"two streams {both:.3f} ms", flush=True)


if __name__ == '__main__':
    main()
