"""K1 persistent kernel on one golden case through a bounds-checking build
(MGPU_LIB=tools/_stamps/k1dbg/libmgpu.so): nodes whose view saw an
out-of-range column report nmods = -1000 - code."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from golden_io import bits_equal, load_fbbt  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'random1'
p, g = load_fbbt(name)
ctx = Context(0)
ctx.load(p)
ctx.set_fbbt_variant(3)
os.environ['MGPU_FBBT_WAVES'] = '2'
inc = np.inf if g['incumbent'] is None else g['incumbent']
r = ctx.fbbt(g['lb_in'], g['ub_in'], inc, mod_cap=g['mod_cap'])
bad = r.nmods <= -1000
print(name, 'nodes', len(r.nmods), 'oob nodes', int(bad.sum()), 'codes', sorted(set((-1000 - r.nmods[bad]).tolist())))
print('lb equal', bits_equal(r.lb, g['lb_out']), 'ub equal', bits_equal(r.ub, g['ub_out']),
      'nmods equal', bool(np.array_equal(r.nmods, g['nmods'])), 'infeas equal', bool(np.array_equal(r.infeasible, g['infeas'])))
if not bits_equal(r.lb, g['lb_out']) or not bits_equal(r.ub, g['ub_out']):
    d = np.nonzero(~((r.lb.view(np.int64) == g['lb_out'].view(np.int64)) & (r.ub.view(np.int64) == g['ub_out'].view(np.int64))))
    print('first diffs', list(zip(d[0][:10].tolist(), d[1][:10].tolist())))
