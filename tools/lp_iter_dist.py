"""Pivot-count distribution of the bench's warm-started tls4-lin LPs (CPU
oracle): sizes the eta file of the product-form LP kernel (K3P)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402

p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
LB, UB = random_boxes(p, 20000, 20261015)
f = oracle.linear_fbbt(p, LB, UB, None)
keep = f.infeas == 0
_, _, _, _, _, ws = oracle.dual_simplex_root(p)
st, obj, it, _ = oracle.dual_simplex(p, f.lb[keep], f.ub[keep], ws, nthreads=8)
it = np.asarray(it)
print('solved', int(keep.sum()), 'mean pivots', it.mean(),
      'p50/90/95/99/99.9', np.percentile(it, [50, 90, 95, 99, 99.9]), 'max', it.max())
for K in (8, 12, 16, 20, 24, 32):
    print(f'> {K} pivots: {(it > K).mean():.4f}')

# product form (K3P) vs dense: objectives and pivot counts
for K in (16, 24):
    s2, o2, i2, _ = oracle.dual_simplex(p, f.lb[keep], f.ub[keep], ws, nthreads=8, pfi=K)
    ok = st == 0
    print(f'pfi={K}: status equal {np.array_equal(st, s2)}, max |dobj| '
          f'{np.max(np.abs(obj[ok] - o2[ok])):.3g}, pivot counts differ on '
          f'{(it != i2).mean():.4f}')
