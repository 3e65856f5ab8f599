"""The unchanged-driver route at B = 1: the reference's own BranchAndBound
(ReliabilityBrancher, NodeIncRelaxer, PCBProcessor) with HipLPEngine and
HipLinearHandler plugged in (oracle/_ref/libminotaur_hip_integ.so), against
the batched tree (mgpu_bnb_*) on the same MILP.  Prints one JSON line:
wall microseconds per LP of the whole BranchAndBound::solve, and the
engine's own (HipLPEngine::solve: one mgpu_lp_solve1 launch from a device
warm-start slot) per LP.  tools/b1_probe.py breaks the route down."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
from minotaur_amd import bnb, runtime  # noqa: E402
from minotaur_amd.problem import random_mkp  # noqa: E402

P = ctypes.c_void_p


def main():
    runtime.load_library()
    lib = ctypes.CDLL(os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so'),
                      mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_bnb.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
        [P] * 9 + [ctypes.c_double, P, P]
    out = []
    _p = lambda a: a.ctypes.data_as(P)   # noqa: E731
    w = random_mkp(1, 12, 2)   # warm-up: kernel modules, pinned blocks, slot chunks
    for hip_fbbt in (0, 1):
        lib.integ_bnb(0, hip_fbbt, w.n, w.m, _p(w.rowptr), _p(w.colidx), _p(w.val), _p(w.rlo),
                      _p(w.rhi), _p(w.vtype), _p(w.vlb), _p(w.vub), _p(w.obj),
                      float(w.obj_const), _p(np.zeros(3)), _p(np.zeros(5, dtype=np.int32)))
    for p in (random_mkp(2, 20, 3), random_mkp(3, 24, 4)):
        row = {"instance": p.name}
        # hip_fbbt 0: the reference's own LinearHandler (node FBBT on the
        # CPU) + HipLPEngine; 1: HipLinearHandler (K1 at batch 1) + HipLPEngine
        for hip_fbbt, key in ((0, "reference_bnb_hiplp_b1"),
                              (1, "reference_bnb_hiplp_hipfbbt_b1")):
            res = np.zeros(3)
            cnt = np.zeros(5, dtype=np.int32)
            lib.integ_bnb(0, hip_fbbt, p.n, p.m, _p(p.rowptr), _p(p.colidx), _p(p.val),
                          _p(p.rlo), _p(p.rhi), _p(p.vtype), _p(p.vlb), _p(p.vub), _p(p.obj),
                          float(p.obj_const), _p(res), _p(cnt))
            est = np.zeros(6)
            lib.integ_last_lp_stats(_p(est))   # HipLPEngine::fillStats
            row[key] = {"ub": res[0], "seconds": res[2], "nodes": int(cnt[0]),
                        "lp_solves": int(cnt[1]), "gpu_fbbt_calls": int(cnt[2]),
                        "us_per_lp": 1e6 * res[2] / max(int(cnt[1]), 1),
                        "engine_us_per_lp": 1e6 * est[2] / max(int(est[0]), 1),
                        "pivots_per_lp": est[4] / max(int(est[0]), 1)}
        ctx = runtime.Context(0)
        ctx.load(p)
        bnb.solve(ctx, batch=64, capacity=1 << 16, order=1, brancher=1)   # warm-up
        t0 = time.perf_counter()
        ob, _, st, _ = bnb.solve(ctx, batch=4096, capacity=1 << 20, order=1, brancher=1)
        el = time.perf_counter() - t0
        ctx.close()
        row["batched_tree"] = {"ub": ob, "seconds": el, "nodes": st.nodes,
                               "lp_solves": st.lps + st.sb_lps,
                               "us_per_lp": 1e6 * el / max(st.lps + st.sb_lps, 1)}
        out.append(row)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
