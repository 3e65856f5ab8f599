"""Where does a B = 1 LP through HipLPEngine spend its time?  (GPU box)

* ``mgpu_lp_solve`` at B = 1 in a loop, each LP from the previous LP's warm
  start with the warm start back (what HipLPEngine::solve asks for), on the
  LP relaxation of the instance: wall us per call;
* the reference's own BranchAndBound with HipLPEngine (integ_bnb_tree:
  MaxVio, bfs; integ_bnb: ReliabilityBrancher): wall seconds per LP and the
  engine's own seconds per LP (HipLPEngine::fillStats).
Prints JSON lines.  Usage: python tools/b1_probe.py [instance ...]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
from minotaur_amd import runtime  # noqa: E402
from minotaur_amd.problem import LinProblem, random_mkp  # noqa: E402

P = ctypes.c_void_p


def _p(a):
    return a.ctypes.data_as(P)


def instances():
    return {'mkp-18-3': random_mkp(2, 18, 3), 'mkp-24-4': random_mkp(3, 24, 4),
            'nvs08_oa': LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances',
                                                     'nvs08_oa.npz'))}


def lp_loop(ctx, p, calls=2000):
    ctx.load(p)
    rng = np.random.default_rng(1)
    lb, ub = p.vlb.copy(), p.vub.copy()
    ws = None
    r = ctx.lp_solve(lb[None], ub[None], want_x=True, want_ws=True)
    ws = runtime.WarmStart(r.ws.head[0], r.ws.st[0], r.ws.d[0], r.ws.binv[0])
    t0 = time.perf_counter()
    piv = 0
    for k in range(calls):
        l, u = lb.copy(), ub.copy()
        j = rng.integers(p.n)
        if p.vub[j] - p.vlb[j] >= 1:
            if k & 1:
                u[j] = p.vlb[j]
            else:
                l[j] = p.vub[j]
        r = ctx.lp_solve(l[None], u[None], ws, want_x=True, want_ws=True)
        piv += int(r.iters[0])
    el = time.perf_counter() - t0
    return {"us_per_call": 1e6 * el / calls, "pivots_per_call": piv / calls,
            "kernel_ms_last": ctx.last_kernel_ms('lp')}


def main():
    runtime.load_library()
    lib = ctypes.CDLL(os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so'),
                      mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_bnb_tree.argtypes = [ctypes.c_int] * 6 + [P] * 9 + [ctypes.c_double, P, P]
    lib.integ_bnb.argtypes = [ctypes.c_int] * 4 + [P] * 9 + [ctypes.c_double, P, P]
    names = sys.argv[1:] or list(instances())
    ctx = runtime.Context(0)
    for name in names:
        p = instances()[name]
        out = {"instance": name, "n": p.n, "m": p.m, "lp_loop": lp_loop(ctx, p)}
        for mode in ('maxvio_tree', 'reliability'):
            res = np.zeros(3)
            st = np.zeros(6)
            if mode == 'maxvio_tree':
                cnt = np.zeros(6, dtype=np.int64)
                lib.integ_bnb_tree(0, 0, 0, 1, p.n, p.m, _p(p.rowptr), _p(p.colidx), _p(p.val),
                                   _p(p.rlo), _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub),
                                   _p(p.obj), float(p.obj_const), _p(res), _p(cnt))
            else:
                cnt = np.zeros(5, dtype=np.int32)
                lib.integ_bnb(0, 0, p.n, p.m, _p(p.rowptr), _p(p.colidx), _p(p.val), _p(p.rlo),
                              _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub), _p(p.obj),
                              float(p.obj_const), _p(res), _p(cnt))
            lib.integ_last_lp_stats(_p(st))
            calls = max(int(st[0]), 1)
            out[mode] = {"ub": res[0], "seconds": res[2], "lp_calls": int(st[0]),
                         "us_per_lp_wall": 1e6 * res[2] / calls,
                         "us_per_lp_engine": 1e6 * st[2] / calls,
                         "pivots_per_lp": st[4] / calls}
        print(json.dumps(out), flush=True)
    ctx.close()




def split():
    """``split``: 400 LPs through mgpu_lp_solve (host arrays) then 400 through
    mgpu_lp_solve1 (device slots), for a kernel trace to tell them apart."""
    p = random_mkp(3, 24, 4)
    ctx = runtime.Context(0)
    ctx.load(p)
    rng = np.random.default_rng(1)
    boxes = []
    for k in range(400):
        l, u = p.vlb.copy(), p.vub.copy()
        j = rng.integers(p.n)
        if k & 1:
            u[j] = p.vlb[j]
        else:
            l[j] = p.vub[j]
        boxes.append((l, u))
    r = ctx.lp_solve(p.vlb[None], p.vub[None], want_x=True, want_ws=True)
    ws = runtime.WarmStart(r.ws.head[0], r.ws.st[0], r.ws.d[0], r.ws.binv[0])
    t0 = time.perf_counter()
    for l, u in boxes:
        ctx.lp_solve(l[None], u[None], ws, want_x=True, want_ws=True)
    t1 = time.perf_counter()
    s0 = ctx.ws_alloc()
    ctx.ws_write(s0, ws)
    out = ctx.ws_alloc()
    t2 = time.perf_counter()
    for l, u in boxes:
        ctx.lp_solve1(l, u, s0, True, out)
    t3 = time.perf_counter()
    print(json.dumps({"host_path_us": 1e6 * (t1 - t0) / 400,
                      "slot_path_us": 1e6 * (t3 - t2) / 400}), flush=True)
    ctx.close()


if __name__ == '__main__':
    if sys.argv[1:2] == ['split']:
        split()
    else:
        main()
