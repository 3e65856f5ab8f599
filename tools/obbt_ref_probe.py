"""Root OBBT: the reference's QuadHandler::postSolveRootNode (HipLPEngine
as bte_, chained bound LPs) vs the batched replay (minotaur_amd/obbt.py), per
seed: tightened bounds, LPs used, and which variables differ."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))


def main():
    import oracle
    from minotaur_amd import obbt, runtime
    from minotaur_amd.quad import random_qcqp
    from minotaur_amd.runtime import Context
    runtime.load_library()
    lib = ctypes.CDLL(os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so'),
                      mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    P = ctypes.c_void_p
    lib.integ_obbt.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_double, P, P, P,
                               ctypes.c_int, P, P, P, P]
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        qp = random_qcqp(seed, nv0=8, ncon=4)
        spec = oracle.qspec(qp)
        rlb, rub = np.zeros(qp.nv), np.zeros(qp.nv)
        info = np.zeros(3, dtype=np.int32)
        cap = 4 * qp.nv
        lc, ls = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        lg, lv = np.zeros(cap), np.zeros(cap)
        lib.integ_obbt(0, ctypes.byref(spec), 0, 0.0, rlb.ctypes.data_as(P),
                       rub.ctypes.data_as(P), info.ctypes.data_as(P), cap, lc.ctypes.data_as(P),
                       lg.ctypes.data_as(P), ls.ctypes.data_as(P), lv.ctypes.data_as(P))
        rows = oracle.quad_root_rows(qp)
        p = obbt.relaxation_lp(qp, rows)
        ctx = Context(0)
        ctx.load(p)
        r, ws = ctx.root_solve()
        inf, lb, ub, mods, nlp, used = obbt.obbt(ctx, qp, rows, r.x[0], ws)
        itmp = obbt.select_vars(qp, r.x[0], qp.vlb, qp.vub)
        ctx.close()
        dl = np.nonzero(~np.isclose(lb, rlb, rtol=1e-6, atol=1e-6))[0]
        du = np.nonzero(~np.isclose(ub, rub, rtol=1e-6, atol=1e-6))[0]
        print(f"seed {seed}: root st {info[0]} ret {info[1]} ref LPs {info[2]} batch LPs {nlp} "
              f"used {used} flagged {int((itmp > 0).sum())} lb diff {dl.tolist()} "
              f"ub diff {du.tolist()}", flush=True)
        for v in list(dl) + list(du):
            print(f"   v{v}: ref [{rlb[v]:.9g}, {rub[v]:.9g}] batch [{lb[v]:.9g}, {ub[v]:.9g}] "
                  f"root [{qp.vlb[v]:.6g}, {qp.vub[v]:.6g}] itmp {itmp[v]}")


if __name__ == '__main__':
    main()
