import sys, os, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'oracle')); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import oracle
from minotaur_amd.problem import knapsack_oa
from minotaur_amd.runtime import Context, WarmStart
ctx = Context(0)
p = knapsack_oa(f=24, N=72)
ctx.load(p)
st0, _, _, _, _, ows = oracle.dual_simplex_root(p)
ws = WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T))
cols = np.repeat(np.arange(p.n, dtype=np.int32), 2); signs = np.tile([1.0, -1.0], p.n)
for kmax in (32, 12, 4):
    ctx.set_lp_variant(3); ctx.set_lp_pfi_wide(kmax)
    g = ctx.lp_bound(cols, signs, ws=ws, want_x=True)
    st, ob, it, xs = oracle.lp_bound(p, cols, signs, ws=ows, pfi=kmax)
    bad = np.nonzero((g.status != st) | (g.iters != it))[0]
    print(kmax, 'mismatch', bad.size, [(int(b), int(g.status[b]), int(st[b]), int(g.iters[b]), int(it[b])) for b in bad[:10]])
    st2, ob2, it2, _ = oracle.lp_bound(p, cols, signs, ws=ows, pfi=0)
    print('   dense oracle iters for those', [int(it2[b]) for b in bad[:10]])
