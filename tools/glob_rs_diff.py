"""Diagnostic: the first main-engine solve where the GPU relstronger glob tree
(mgpu_glob_brancher 1) differs from the reference's own tree on HipLPEngine
(integ_glob_tree3, device 0) or from the CPU restatement (oracle/
glob_tree.py).  Arguments: seed,nv0,ncon[,obbt] per case (tests/
test_glob_pin_cpu.py PIN_CASES).  Values are compared bit for bit."""
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in (ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, d)

from glob_tree import CpuGlobContext  # noqa: E402
from minotaur_amd import glob as mglob  # noqa: E402
from minotaur_amd import runtime  # noqa: E402
from minotaur_amd.quad import random_qcqp  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def first_diff(a, b, exact):
    for k in range(max(len(a), len(b))):
        x = a[k] if k < len(a) else None
        y = b[k] if k < len(b) else None
        if x is None or y is None or x[0] != y[0] or x[2] != y[2]:
            return k
        if not (x[1] == y[1] or (math.isinf(x[1]) and math.isinf(y[1]))):
            if exact or abs(x[1] - y[1]) > 1e-9 * max(1.0, abs(x[1])):
                return k
    return None


def show(name, a, b, k):
    print(f"  {name}: first difference at solve {k}", flush=True)
    if k is None:
        return
    for i in range(max(0, k - 3), min(k + 4, max(len(a), len(b)))):
        print("   ", i, a[i] if i < len(a) else None, b[i] if i < len(b) else None, flush=True)


def main():
    cases = [tuple(int(v) for v in s.split(',')) for s in sys.argv[1:]]
    runtime.load_library()
    from test_simplex_cuts_cpu import glob_tree3, load_integ
    integ = load_integ()
    P = ctypes.c_void_p
    integ.integ_last_solve_log.argtypes = [ctypes.c_int, P, P, P]
    ctx = Context(0)
    for cs_ in cases:
        seed, nv0, ncon = cs_[:3]
        obbt = cs_[3] if len(cs_) > 3 else 0
        qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
        ub, cnt, _ = glob_tree3(integ, qp, 1 | 16 | (8 if obbt else 0), 0, 1)
        n = integ.integ_last_solve_log(0, None, None, None)
        ls, lv, li = np.zeros(n, np.int32), np.zeros(n), np.zeros(n, np.int32)
        integ.integ_last_solve_log(n, ls.ctypes.data, lv.ctypes.data, li.ctypes.data)
        ref = [(int(a), float(b), int(c)) for a, b, c in zip(ls, lv, li)]
        obj, _, st, _ = mglob.solve(ctx, qp, batch=1, capacity=1 << 14, order=2, warm=1, qt=0,
                                    lin=1, obbt=obbt, brancher=1, max_rounds=20000)
        gs, gv, gi = ctx.glob_lp_log()
        gpu = [(int(a), float(b), int(c)) for a, b, c in zip(gs, gv, gi)]
        c = CpuGlobContext(qp)
        c.glob_config(2, 1, 0, 1, obbt)
        c.glob_brancher(1)
        c.glob_init(1 << 16)
        for _ in range(20000):
            cst = c.glob_round(1)
            if cst.open == 0:
                break
        print(f"seed {seed} ({nv0},{ncon}) obbt {obbt}: ref nodes {cnt[0]} lps {cnt[2]} ub {ub!r}; "
              f"gpu nodes {st.nodes} lps {st.lps} obj {obj!r}; cpu nodes {cst.nodes} lps {cst.lps} "
              f"obj {c.inc!r}", flush=True)
        show("ref(HipLPEngine) vs gpu, bits", ref, gpu, first_diff(ref, gpu, True))
        show("cpu restatement vs gpu, 1e-9", c.lplog, gpu, first_diff(c.lplog, gpu, False))
    ctx.close()


if __name__ == '__main__':
    main()
