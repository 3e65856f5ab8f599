"""K1G row-visit census ("Where K1G's time goes"): run with
MGPU_LIB pointing at an instrumented variant built by tools/variant_build.py
(the edits count row visits per wave, tightenings per node and s_memtime
cycles of the activity / update phases, written into the infeas / nmods /
lb_out[0..3] outputs), e.g.

    python tools/variant_build.py k1gprobe fbbt_group.hip '<old>' '<new>' ...
    MGPU_LIB=tools/_stamps/k1gprobe/libmgpu.so python tools/k1g_probe.py

The outputs of such a build are NOT FBBT results."""
import os, sys, math
import numpy as np, torch
ROOT = '/root/repo' if os.path.isdir('/root/repo') else os.getcwd()
sys.path.insert(0, ROOT)
from minotaur_amd.problem import LinProblem, random_boxes
from minotaur_amd.runtime import Context
p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
ctx = Context(0); ctx.load(p)
LBa, UBa = random_boxes(p, 524288, 20261017)
for B in (1024, 16384):
    for v in (4,):
        ctx.set_fbbt_variant(v)
        r = ctx.fbbt(LBa[:B], UBa[:B], math.inf)
        vis = r.infeasible // 16; it = r.infeasible % 16
        cyc = r.lb[:, 0]
        ta, tu, tr = r.lb[:, 1], r.lb[:, 2], r.lb[:, 3]
        print(f"   per node: row-tighten cycles {tr.mean():.0f} (activity {ta.mean():.0f}, update {tu.mean():.0f}) of wave {cyc.mean():.0f}; per tightening {tr.mean()/r.nmods.mean():.0f}")
        print(f"B {B} v{v}: visits/wave mean {vis.mean():.1f} max {vis.max()}  tight/node {r.nmods.mean():.1f}  sweeps(iters-1) mean {(it-1).mean():.2f} max {(it-1).max()}  wave cycles mean {cyc.mean():.0f}  cycles/visit {np.mean(cyc/np.maximum(vis,1)):.0f}  ms {ctx.last_kernel_ms('fbbt'):.3f}", flush=True)
