"""Load the committed golden fixtures (tests/golden/*.npz)."""
import glob
import math
import os

import numpy as np

from minotaur_amd.problem import LinProblem

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def cases(prefix='fbbt_'):
    return sorted(os.path.basename(p)[len(prefix):-4]
                  for p in glob.glob(os.path.join(GOLDEN, prefix + '*.npz')))


def load_fbbt(name):
    z = np.load(os.path.join(GOLDEN, f'fbbt_{name}.npz'), allow_pickle=False)
    p = LinProblem(name=str(z['name']), n=int(z['n']), m=int(z['m']),
                   rowptr=z['rowptr'].astype(np.int32), colidx=z['colidx'].astype(np.int32),
                   val=z['val'], rlo=z['rlo'], rhi=z['rhi'], vlb=z['vlb'], vub=z['vub'],
                   vtype=z['vtype'].astype(np.int32), obj=z['obj'],
                   obj_const=float(z['obj_const'])).validate()
    inc = float(z['incumbent'])
    g = {k: z[k] for k in ('lb_in', 'ub_in', 'lb_out', 'ub_out', 'infeas', 'nmods',
                           'mod_var', 'mod_lu', 'mod_val')}
    g['incumbent'] = None if math.isnan(inc) else inc
    g['mod_cap'] = g['mod_var'].shape[1]
    return p, g


def bits_equal(a, b):
    """Bit-exact f64 comparison (NaN payloads included)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def assert_mods_equal(nmods, mv, ml, mval, g, cap):
    for b in range(len(nmods)):
        k = min(int(nmods[b]), cap)
        assert np.array_equal(mv[b, :k], g['mod_var'][b, :k].astype(np.int32)), b
        assert np.array_equal(ml[b, :k], g['mod_lu'][b, :k].astype(np.int32)), b
        assert bits_equal(mval[b, :k], g['mod_val'][b, :k]), b


def load_lp(name):
    z = np.load(os.path.join(GOLDEN, f'lp_{name}.npz'), allow_pickle=False)
    p = LinProblem(name=str(z['name']), n=int(z['n']), m=int(z['m']),
                   rowptr=z['rowptr'].astype(np.int32), colidx=z['colidx'].astype(np.int32),
                   val=z['val'], rlo=z['rlo'], rhi=z['rhi'], vlb=z['vlb'], vub=z['vub'],
                   vtype=z['vtype'].astype(np.int32), obj=z['obj_c'],
                   obj_const=float(z['obj_const'])).validate()
    return p, {k: z[k] for k in ('lb', 'ub', 'status', 'obj')}


OBJ_TOL = 1e-6   # north star: relaxation objectives within 1e-6


def assert_lp_matches(status, obj, g, mask=None):
    """Status identical; objective within 1e-6 (relative for |obj| > 1) of the
    golden HiGHS value.  HiGHS 'unknown' entries (status 12) are skipped."""
    ok = g['status'] != 12
    if mask is not None:
        ok &= mask
    assert np.array_equal(np.asarray(status)[ok], g['status'][ok])
    opt = ok & (g['status'] == 0)
    err = np.abs(np.asarray(obj)[opt] - g['obj'][opt]) / np.maximum(1.0, np.abs(g['obj'][opt]))
    assert err.size == 0 or err.max() <= OBJ_TOL, err.max()


def load_quad(name):
    """QuadProblem + reference outputs of a quad_<name>.npz fixture."""
    from minotaur_amd.quad import QuadProblem
    z = np.load(os.path.join(GOLDEN, f'quad_{name}.npz'), allow_pickle=False)
    qp = QuadProblem.load(os.path.join(GOLDEN, f'quad_{name}.npz'))
    g = {k: z[k] for k in ('lb_in', 'ub_in', 'rows_in', 'lb_out', 'ub_out', 'rows_out',
                           'infeas', 'nmods', 'mod_kind', 'mod_idx', 'mod_v1', 'mod_v2')}
    inc = float(z['incumbent'])
    g['incumbent'] = None if math.isnan(inc) else inc
    g['qt'] = int(z['qt'])
    g['mod_cap'] = g['mod_kind'].shape[1]
    return qp, g


def assert_quad_equal(r_lb, r_ub, r_rows, r_inf, r_nmods, kind, idx, v1, v2, g):
    """Bit-exact comparison with a reference quad fixture (mod log included)."""
    assert bits_equal(r_lb, g['lb_out'])
    assert bits_equal(r_ub, g['ub_out'])
    assert np.array_equal(np.asarray(r_inf), g['infeas'])
    assert np.array_equal(np.asarray(r_nmods), g['nmods'])
    assert bits_equal(r_rows, g['rows_out'])
    cap = g['mod_cap']
    for b in range(len(r_nmods)):
        k = min(int(r_nmods[b]), cap)
        assert np.array_equal(kind[b, :k], g['mod_kind'][b, :k].astype(np.int32)), b
        assert np.array_equal(idx[b, :k], g['mod_idx'][b, :k].astype(np.int32)), b
        assert bits_equal(v1[b, :k], g['mod_v1'][b, :k]), b
        assert bits_equal(v2[b, :k], g['mod_v2'][b, :k]), b
