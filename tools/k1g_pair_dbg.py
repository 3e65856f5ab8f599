"""K1G (variant 4, G = 16) against every FBBT golden with the library in
MGPU_LIB: mismatching cases and, for the first, the differing nodes/columns
(paired-row walk debugging)."""
import os
import sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from golden_io import cases, load_fbbt  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402
ctx = Context(0)
tag = os.environ.get('TAG', '')
bad = []
for name in cases():
    p, g = load_fbbt(name)
    if p.m > 64:
        continue
    ctx.load(p)
    inc = np.inf if g['incumbent'] is None else g['incumbent']
    ctx.set_fbbt_variant(4)
    r = ctx.fbbt(g['lb_in'], g['ub_in'], inc)
    dl = np.nonzero(r.lb.view(np.int64) != g['lb_out'].view(np.int64))
    du = np.nonzero(r.ub.view(np.int64) != g['ub_out'].view(np.int64))
    ok = len(dl[0]) == 0 and len(du[0]) == 0 and np.array_equal(r.infeasible, g['infeas']) \
        and np.array_equal(r.nmods, g['nmods'])
    if not ok:
        nodes = sorted(set(dl[0].tolist()) | set(du[0].tolist()))
        bad.append(name)
        print(tag, name, 'lb', len(dl[0]), 'ub', len(du[0]), 'nodes', len(nodes), nodes[:6],
              'infeq', bool(np.array_equal(r.infeasible, g['infeas'])), flush=True)
print(tag, 'bad', bad, flush=True)
ctx.close()
