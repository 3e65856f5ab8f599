"""CPU: the LPEngine tableau extras (src/base/LPEngine.h:39-73) and the
reference's own simplex-tableau cut generator running on them (VERDICT r05
"next" #1).

mglob sets simplex_cut (src/solvers/Glob.cpp:311) and makes the main LP
engine QuadHandler's cut engine (SimpleTransformer.cpp:953-954), so at the
root QuadHandler::separate (QuadHandler.cpp:1691-1703) runs
SimplexQuadCutGen::generateCuts on that engine: getBasicInfo_ reads the
engine's matrix, bounds and right-hand side (SimplexQuadCutGen.cpp:285-304),
sortVariables_ its basis (:593-629), substituteAndRelax_ its tableau rows
(:366-418).  The harness (oracle/_ref/libminotaur_hip_integ.so,
integ_simplex_cuts) builds Glob's root relaxation with the reference's own
NodeIncRelaxer + IntVar / Linear / Quad handlers, solves it on the engine
(here CpuLPEngine: the dual-simplex restatement; tests/test_simplex_cuts_gpu.py
runs HipLPEngine), reads every extra and then calls the reference's
SimplexQuadCutGen on it.

Checks:
* the views are OsiLPEngine's (OsiLPEngine.cpp:328-360 over Clp): the row-major
  matrix is the relaxation's rows term for term; infinite bounds are
  +-DBL_MAX; rhs follows Osi's convertBoundToSense; row activity = A x;
* every getBInvARow row equals numpy's B^-1 [A I] for the reported basis
  (Osi's slack convention, slacks s = rhs - Ax), within 1e-12;
* the generated cuts are violated at the root LP point (each was kept for
  its depth, :203-219) and hold at the QCQP optimum the reference's own glob
  tree proves (they relax products over the root box).  The generator keeps
  maxCuts_ of its candidates after sorting the cut POINTERS (:204, a
  reference quirk: the choice follows heap addresses), so engines are
  compared on the whole candidate set (``lift``: maxCuts_ raised to its cap);
* Glob's real options -- simplex cuts, root OBBT, the relstronger brancher --
  prove the same optimum as the bare tree (a global optimum is unique in
  value), on the bilinear instances where neither tree closes a node at
  NoCandToBranch (no NLP engine in the image, QuadHandler.cpp:356-420)."""
import ctypes
import math
import os

import numpy as np
import pytest

from minotaur_amd.quad import random_qcqp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
LIB = os.path.join(ROOT, 'oracle', '_ref', 'libminotaur_hip_integ.so')
P = ctypes.c_void_p
DBL_MAX = np.finfo(np.float64).max

# (seed, nv0, ncon, squares)
TABLEAU_CASES = [(s, 8, 5, sq) for s in (0, 1, 2, 5, 9, 13) for sq in (False, True)] + \
                [(16, 5, 3, False), (31, 8, 5, True)]
# bilinear instances on which neither the bare tree nor the tree with Glob's
# options closes a node at NoCandToBranch
GLOB_CASES = [(16, 5, 3), (17, 6, 4), (26, 6, 4), (30, 5, 3), (31, 8, 5), (33, 8, 5)]
GLOB_OPTS = 1 | 4 | 8 | 16   # bfs, simplex_cut, root OBBT, relstronger

_ORDER = ('rowstart', 'rowlen', 'ind', 'val', 'clo', 'chi', 'rlo', 'rhi', 'rhs', 'act', 'rrow',
          'rcol', 'rval', 'rlb', 'rub', 'vlb', 'vub', 'basics', 'z', 'slack', 'x', 'cut_coef',
          'cut_lb', 'cut_ub')


@pytest.fixture(scope='module')
def integ():
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    return load_integ()


def load_integ():
    # torch (which libmgpu's loader imports) before the integration library:
    # loaded RTLD_GLOBAL first, the reference objects' symbols would bind
    # torch's libraries too, and the process would destroy an object twice
    # at exit ("double free", exit 134)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    lib.integ_simplex_cuts.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P] + \
        [P] * len(_ORDER)
    lib.integ_glob_tree3.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, P, P]
    return lib


def simplex_cuts(integ, qp, device, cap=160, lift=False):
    """integ_simplex_cuts -> dict of the engine's views, tableau and cuts
    (lift: every candidate cut is added, see integ_driver.cpp)."""
    import oracle
    spec = oracle.qspec(qp)
    dims = np.zeros(7, dtype=np.int64)
    i32 = lambda k: np.zeros(k, dtype=np.int32)
    f64 = lambda k: np.zeros(k)
    a = dict(rowstart=i32(cap + 1), rowlen=i32(cap), ind=i32(cap * cap), val=f64(cap * cap),
             clo=f64(cap), chi=f64(cap), rlo=f64(cap), rhi=f64(cap), rhs=f64(cap), act=f64(cap),
             rrow=i32(cap * cap), rcol=i32(cap * cap), rval=f64(cap * cap), rlb=f64(cap),
             rub=f64(cap), vlb=f64(cap), vub=f64(cap), basics=i32(cap), z=f64(cap * cap),
             slack=f64(cap * cap), x=f64(cap), cut_coef=f64(cap * cap), cut_lb=f64(cap),
             cut_ub=f64(cap))
    rc = integ.integ_simplex_cuts(device, ctypes.byref(spec), cap, int(lift),
                                  dims.ctypes.data_as(P),
                                  *[a[k].ctypes.data_as(P) for k in _ORDER])
    assert rc == 0, rc
    n, m, nnz = (int(v) for v in dims[:3])
    k = int(dims[6])
    out = {'n': n, 'm': m, 'nnz': nnz, 'status': int(dims[3]), 'optimal_basis': int(dims[4]),
           'site': int(dims[5]), 'ncuts': k}
    for key, ln in (('rowstart', m + 1), ('rowlen', m), ('ind', nnz), ('val', nnz), ('clo', n),
                    ('chi', n), ('rlo', m), ('rhi', m), ('rhs', m), ('act', m), ('rrow', nnz),
                    ('rcol', nnz), ('rval', nnz), ('rlb', m), ('rub', m), ('vlb', n), ('vub', n),
                    ('basics', m), ('x', n), ('cut_lb', k), ('cut_ub', k)):
        out[key] = a[key][:ln].copy()
    out['z'] = a['z'][:m * n].reshape(m, n).copy()
    out['slack'] = a['slack'][:m * m].reshape(m, m).copy()
    out['cuts'] = a['cut_coef'][:k * n].reshape(k, n).copy()
    return out


def glob_tree3(integ, qp, opts, device, pres_freq=5):
    """integ_glob_tree3 -> (ub, counts, incumbent x)."""
    import oracle
    spec = oracle.qspec(qp)
    res = np.zeros(3)
    cnt = np.zeros(8, dtype=np.int64)
    x = np.zeros(qp.nv)
    assert integ.integ_glob_tree3(device, ctypes.byref(spec), opts, pres_freq,
                                  res.ctypes.data_as(P), cnt.ctypes.data_as(P),
                                  x.ctypes.data_as(P)) == 0
    return res[0], cnt, x


def osi_bound(v):
    return np.where(v <= -1e27, -DBL_MAX, np.where(v >= 1e27, DBL_MAX, v))


def osi_rhs(lo, hi):
    lo, hi = osi_bound(lo), osi_bound(hi)
    return np.where(lo > -DBL_MAX, np.where(hi < DBL_MAX, hi, lo), np.where(hi < DBL_MAX, hi, 0.0))


def check_views_and_tableau(r, tol=1e-12):
    n, m, nnz = r['n'], r['m'], r['nnz']
    assert r['status'] == 0 and r['optimal_basis'] == 1
    # the matrix by row: the relaxation's rows, term for term, in order
    rs = r['rowstart']
    assert rs[0] == 0 and rs[-1] == nnz and np.array_equal(np.diff(rs), r['rowlen'])
    rows = np.repeat(np.arange(m), r['rowlen'])
    assert np.array_equal(rows, r['rrow'])
    assert np.array_equal(r['ind'], r['rcol']) and np.array_equal(r['val'], r['rval'])
    assert np.array_equal(r['clo'], osi_bound(r['vlb'])) and np.array_equal(r['chi'], osi_bound(r['vub']))
    assert np.array_equal(r['rlo'], osi_bound(r['rlb'])) and np.array_equal(r['rhi'], osi_bound(r['rub']))
    assert np.array_equal(r['rhs'], osi_rhs(r['rlb'], r['rub']))
    A = np.zeros((m, n))
    np.add.at(A, (rows, r['ind']), r['val'])
    assert np.allclose(r['act'], A @ r['x'], rtol=0, atol=1e-12 * max(1.0, np.abs(A @ r['x']).max()))
    # the tableau: row i of B^-1 [A I] with B the basis columns of [A I]
    M = np.hstack([A, np.eye(m)])
    bas = r['basics']
    assert sorted(bas.tolist()) == sorted(set(bas.tolist())) and bas.min() >= 0 and bas.max() < n + m
    T = np.linalg.solve(M[:, bas], M)
    G = np.hstack([r['z'], r['slack']])
    scale = max(1.0, np.abs(T).max())
    err = np.abs(G - T).max()
    assert err <= tol * scale, err
    # the basic columns of the tableau are the identity
    assert np.abs(G[:, bas] - np.eye(m)).max() <= tol * scale
    return err


def cut_violation(coef, lb, ub, x):
    """> 0 where the cut lb <= coef x <= ub is violated at x."""
    v = coef @ x
    return np.maximum(np.where(np.isfinite(ub), v - ub, -np.inf),
                      np.where(np.isfinite(lb), lb - v, -np.inf))


@pytest.mark.parametrize('case', TABLEAU_CASES)
def test_tableau_extras_equal_numpy(integ, case):
    seed, nv0, ncon, sq = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=sq)
    r = simplex_cuts(integ, qp, -1)
    check_views_and_tableau(r)


def test_simplex_cuts_cut_off_the_root_point(integ):
    total = 0
    for seed, nv0, ncon, sq in TABLEAU_CASES:
        qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=sq)
        r = simplex_cuts(integ, qp, -1)
        k = r['ncuts']
        total += k
        if k:
            # each cut has exactly one infinite side (SimplexQuadCutGen.cpp:210)
            assert np.all(np.isinf(r['cut_lb']) ^ np.isinf(r['cut_ub']))
            viol = cut_violation(r['cuts'], r['cut_lb'], r['cut_ub'], r['x'])
            assert np.all(viol > 0), viol
    assert total >= 20


@pytest.mark.parametrize('case', GLOB_CASES)
def test_cuts_valid_at_the_proven_optimum(integ, case):
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    r = simplex_cuts(integ, qp, -1)
    ub, cnt, xs = glob_tree3(integ, qp, 1, -1)
    assert math.isfinite(ub) and cnt[3] == 0
    if r['ncuts']:
        viol = cut_violation(r['cuts'], r['cut_lb'], r['cut_ub'], xs)
        scale = 1.0 + np.abs(r['cuts']).sum(axis=1) * (1.0 + np.abs(xs).max())
        assert np.all(viol <= 1e-6 * scale), (viol, scale)


@pytest.mark.parametrize('case', GLOB_CASES)
def test_glob_options_prove_the_same_optimum(integ, case):
    """Glob's real configuration (simplex_cut, root OBBT, relstronger) on the
    reference's own tree over CpuLPEngine proves the optimum of the bare
    MaxVio tree; the options do act (cuts at the root or OBBT LPs)."""
    seed, nv0, ncon = case
    qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
    ub0, c0, _ = glob_tree3(integ, qp, 1, -1)
    ub1, c1, _ = glob_tree3(integ, qp, GLOB_OPTS, -1)
    assert c0[3] == 0 and c1[3] == 0
    assert math.isfinite(ub0) and abs(ub1 - ub0) <= 1e-6 * max(1.0, abs(ub0)), (ub0, ub1)


def test_glob_options_act(integ):
    """Across the instances, the options change the search: root cut rows
    and OBBT bound LPs occur, and the trees are not the bare ones."""
    rows = lps = differ = 0
    for seed, nv0, ncon in GLOB_CASES:
        qp = random_qcqp(seed, nv0=nv0, ncon=ncon, squares=False)
        _, c0, _ = glob_tree3(integ, qp, 1, -1)
        _, c1, _ = glob_tree3(integ, qp, GLOB_OPTS, -1)
        rows += int(c1[4])
        lps += int(c1[5])
        differ += int(c1[0] != c0[0])
    assert rows > 0 and lps > 0 and differ >= len(GLOB_CASES) // 2, (rows, lps, differ)
