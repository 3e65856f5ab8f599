"""K1 size sweep ("run the size sweep (n up to 1e5, B up to
1e4) to show the bandwidth regime"): seeded sparse MILP rows (3-8 terms per
row, m = n / 2, half binaries, a quarter integers, a quarter continuous),
node boxes by random branching, K1 on the device with the auto variant.
Per size: kernel time (HIP events), algorithmic bytes (bench.fbbt_bytes),
achieved GB/s and fraction of the 8 TB/s HBM peak, and a bit-exact spot check
of 32 nodes against the C restatement.  Prints one JSON line per size."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

from minotaur_amd.problem import (BINARY, CONTINUOUS, INTEGER, LinProblem,  # noqa: E402
                                  random_boxes)

HBM_PEAK_GBS = 8000.0


def sweep_problem(seed, n):
    rng = np.random.default_rng(seed)
    m = max(1, n // 2)
    u = rng.random(n)
    vtype = np.where(u < 0.5, BINARY, np.where(u < 0.75, INTEGER, CONTINUOUS)).astype(np.int32)
    vlb = np.where(vtype == BINARY, 0.0, np.where(vtype == INTEGER, 0.0, -5.0))
    vub = np.where(vtype == BINARY, 1.0, np.where(vtype == INTEGER, 20.0, 30.0))
    x = np.where(vtype == CONTINUOUS, rng.uniform(vlb, vub),
                 np.floor(rng.uniform(vlb, vub + 1)))
    k = rng.integers(3, 9, size=m)
    rowptr = np.zeros(m + 1, dtype=np.int32)
    np.cumsum(k, out=rowptr[1:])
    colidx = np.empty(rowptr[-1], dtype=np.int32)
    for i in range(m):   # distinct ascending columns per row
        colidx[rowptr[i]:rowptr[i + 1]] = np.sort(rng.choice(n, size=k[i], replace=False))
    val = np.round(rng.uniform(-5, 5, size=colidx.size), 3)
    val[val == 0.0] = 1.0
    act = np.add.reduceat(val * x[colidx], rowptr[:-1])
    slack = rng.uniform(0, 4, size=m)
    kind = rng.random(m)
    rlo = np.where(kind < 0.5, -np.inf, act - slack)
    rhi = np.where(kind < 0.5, act + slack, np.where(kind < 0.8, np.inf, act + slack))
    obj = np.round(rng.uniform(-3, 3, n), 2)
    return LinProblem(name=f'sweep-n{n}', n=n, m=m, rowptr=rowptr, colidx=colidx, val=val,
                      rlo=rlo, rhi=rhi, vlb=vlb.astype(np.float64), vub=vub.astype(np.float64),
                      vtype=vtype, obj=obj, obj_const=0.0).validate()


def main():
    import torch
    import oracle
    from bench import fbbt_bytes
    from minotaur_amd.runtime import Context
    ctx = Context(0)
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    for n in (1000, 10000, 100000):
        p = sweep_problem(7, n)
        B = int(min(10000, max(64, 1e8 // n)))
        LB, UB = random_boxes(p, B, 11, max_depth=20)
        ctx.load(p)
        lb, ub = torch.from_numpy(LB).to(dev), torch.from_numpy(UB).to(dev)
        lb2, ub2 = torch.empty_like(lb), torch.empty_like(ub)
        inf = torch.zeros(B, dtype=torch.int32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        ctx.fbbt_dev(lb, ub, lb2, ub2, inf, nm)      # warm-up
        torch.cuda.synchronize()
        ms = []
        for _ in range(3):
            ctx.fbbt_dev(lb, ub, lb2, ub2, inf, nm)
            ms.append(ctx.last_kernel_ms('fbbt'))
        t = float(np.median(ms))
        byt = fbbt_bytes(p, B)
        o = oracle.linear_fbbt(p, LB[:32], UB[:32], None, nthreads=8)
        gl, gu = lb2[:32].cpu().numpy(), ub2[:32].cpu().numpy()
        exact = bool(np.array_equal(gl.view(np.uint64), o.lb.view(np.uint64)) and
                     np.array_equal(gu.view(np.uint64), o.ub.view(np.uint64)) and
                     np.array_equal(inf[:32].cpu().numpy(), o.infeas))
        print(json.dumps({"n": n, "m": p.m, "nnz": p.nnz, "batch": B, "fbbt_ms": t,
                          "bytes_per_launch": byt, "achieved_gbs": byt / (t * 1e-3) / 1e9,
                          "frac_of_hbm_peak": byt / (t * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "node_passes_per_s": B / (t * 1e-3),
                          "spot_check_32_nodes_bit_exact": exact}), flush=True)
        del lb, ub, lb2, ub2
    ctx.reset_stream()
    ctx.close()


if __name__ == '__main__':
    main()
