"""Diagnostic: where K3 (or K3P with --pfi) spends its cycles.  Builds a stamped variant of
libmgpu (-DMGPU_STAMPS) into /tmp, runs the LP probe workload and prints the
s_memtime share of each section (see cdna_hip_programming.md §7: read the
SHARES, not the run time, of a stamped build)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
OUT = os.environ.get('STAMP_LIB', os.path.join(ROOT, 'gpurun_out', 'libmgpu_stamps.so'))
NAMES = ['setup:primals', 'pricing', 'rho_write', 'pass1+min', 'pass2+argmax', 'column_q',
         'steps/updates', 'binv_update', 'tail', 'outputs', 'setup:skip',
         'setup:bounds', 'setup:basis', 'setup:place']
PFI_NAMES = ['setup', 'primals', 'pricing', 'btran+rho', 'pass1+min', 'pass2+argmax', 'ftran',
             'steps+eta', 'outputs', 'skip/empty', 'path replay', 'path duals']


def build():
    from minotaur_amd import build as b
    srcs = [os.path.join(b.CSRC, x) for x in b.SOURCES]
    cmd = [b.HIPCC] + b.FLAGS + ['-DMGPU_STAMPS', '-I', os.path.join(ROOT, 'include'),
                                 '-o', OUT] + srcs + ['-L/opt/rocm/lib', '-lrccl']
    subprocess.run(cmd, check=True)


def tree():
    """--tree: K3P's sections inside the headline's tree rounds (tls4-oa, path
    warm starts, batch PROBE_BATCH): stamps of round 4's LP call."""
    if not os.path.exists(OUT):
        build()
    os.environ['MGPU_LIB'] = OUT
    import math
    import numpy as np
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context, load_library
    lib = load_library()
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    B = int(os.environ.get('PROBE_BATCH', '262144'))
    LB, UB = random_boxes(p, B, 20261017)
    ctx = Context(0)
    ctx.load(p)
    ctx.bnb_config(0, int(os.environ.get('PROBE_WARM', '2')))
    ctx.bnb_init(B * 8 + 2)
    ctx.bnb_import(LB, UB, np.full(B, -math.inf), np.zeros(B, dtype=np.int32))
    buf = (ctypes.c_ulonglong * 16)()
    st = None
    for r in range(5):
        if r == 4:
            lib.mgpu_debug_pfi_stamps(buf, 1)
            prev = st.pivots
        st = ctx.bnb_round(B)
    lib.mgpu_debug_pfi_stamps(buf, 1)
    names = PFI_NAMES
    tot = sum(buf[i] for i in range(len(names)))
    piv = st.pivots - prev
    print(f"round 4: pivots {piv}  total wave-cycles {tot:.3e}  per pivot {tot / max(piv, 1):.0f}")
    for i, nme in enumerate(names):
        print(f"  {nme:14s} {100.0 * buf[i] / tot:6.2f} %   {buf[i] / max(piv, 1):9.0f} cyc/pivot")


def b1():
    """--b1: K3's sections for single LPs through mgpu_lp_solve1 (HipLPEngine's
    route; mkp-24-4, each LP from the previous LP's slot): wave-cycles per LP
    per section, the kernel's total and its prologue (matrix / warm-start
    staging before the node loop)."""
    if not os.path.exists(OUT):
        build()
    os.environ['MGPU_LIB'] = OUT
    import numpy as np
    from minotaur_amd.problem import random_mkp
    from minotaur_amd.runtime import Context, load_library
    lib = load_library()
    p = random_mkp(3, 24, 4)
    ctx = Context(0)
    ctx.load(p)
    rng = np.random.default_rng(1)
    s0, s1 = ctx.ws_alloc(), ctx.ws_alloc()
    ctx.lp_solve1(p.vlb, p.vub, -1, True, s0)
    buf = (ctypes.c_ulonglong * 16)()
    lib.mgpu_debug_lp_stamps(buf, 1)
    piv = 0
    L = 400
    for k in range(L):
        lb, ub = p.vlb.copy(), p.vub.copy()
        j = rng.integers(p.n)
        if k & 1:
            ub[j] = p.vlb[j]
        else:
            lb[j] = p.vub[j]
        piv += ctx.lp_solve1(lb, ub, s0, True, s1)[2]
    lib.mgpu_debug_lp_stamps(buf, 1)
    print(f"{L} LPs, {piv / L:.2f} pivots each; wave-cycles per LP:")
    for i, nme in enumerate(NAMES[:10]):
        print(f"  {nme:14s} {buf[i] / L:9.0f}")
    print(f"  {'kernel total':14s} {buf[10] / L:9.0f}   (prologue {buf[11] / L:.0f}; 4 waves summed)")


def rel():
    """--rel: K3's sections over config 2's whole reliability tree (tls4-oa,
    best-first, parent warm starts, growth 2; node LPs and chained strong
    branching): wave-cycles per LP and per pivot per section."""
    if not os.path.exists(OUT):
        build()
    os.environ['MGPU_LIB'] = OUT
    from minotaur_amd import bnb
    from minotaur_amd.problem import LinProblem
    from minotaur_amd.runtime import Context, load_library
    lib = load_library()
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx = Context(0)
    ctx.load(p)
    bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1, brancher=1, growth=2)
    buf = (ctypes.c_ulonglong * 16)()
    lib.mgpu_debug_lp_stamps(buf, 1)
    _, _, st, _ = bnb.solve(ctx, batch=131072, capacity=1 << 20, order=1, warm=1, brancher=1,
                            growth=2)
    lib.mgpu_debug_lp_stamps(buf, 1)
    lps = st.lps + st.sb_lps
    piv = st.pivots + st.sb_pivots
    tot = sum(buf[i] for i in range(10))
    print(f"{lps} LPs, {piv} pivots ({piv / max(lps, 1):.2f} per LP); section wave-cycles "
          f"{tot:.3e}; kernel total {buf[10]:.3e}, prologue {buf[11]:.3e}")
    names = NAMES[:10] + ['', '', 'setup:basis', 'setup:place', 'out:objective', 'out:x+ws']
    tot += sum(buf[i] for i in range(12, 16))
    for i, nme in enumerate(names):
        if not nme:
            continue
        print(f"  {nme:14s} {100.0 * buf[i] / tot:6.2f} %   {buf[i] / max(lps, 1):9.0f} cyc/LP"
              f"   {buf[i] / max(piv, 1):9.0f} cyc/pivot")


def main():
    if '--tree' in sys.argv:
        tree()
        return
    if '--rel' in sys.argv:
        rel()
        return
    if '--b1' in sys.argv:
        b1()
        return
    pfi = '--pfi' in sys.argv
    if not os.path.exists(OUT):
        build()
    os.environ['MGPU_LIB'] = OUT
    import numpy as np
    import torch
    from minotaur_amd.problem import LinProblem, random_boxes
    from minotaur_amd.runtime import Context, WarmStart, load_library
    lib = load_library()
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    ctx = Context(0)
    ctx.load(p)
    root, wsh = ctx.root_solve()
    B = 65536
    LB, UB = random_boxes(p, B, 20261015)
    f = ctx.fbbt(LB, UB)
    buf = (ctypes.c_ulonglong * 16)()
    if pfi:
        ctx.set_lp_variant(3)
        fn, names = lib.mgpu_debug_pfi_stamps, PFI_NAMES
    else:
        ctx.set_lp_variant(1)
        fn, names = lib.mgpu_debug_lp_stamps, NAMES
    fn(buf, 1)
    r = ctx.lp_solve(f.lb, f.ub, wsh, skip=f.infeasible)
    fn(buf, 1)
    tot = sum(buf[i] for i in range(len(names)))
    piv = int(r.iters.sum())
    print(f"pivots {piv}  total wave-cycles {tot:.3e}  per pivot {tot / max(piv, 1):.0f}")
    for i, nme in enumerate(names):
        print(f"  {nme:14s} {100.0 * buf[i] / tot:6.2f} %   {buf[i] / max(piv, 1):9.0f} cyc/pivot")


if __name__ == '__main__':
    main()
