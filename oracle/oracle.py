"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings for the two CPU checkers:

* ``liboracle.so``        — this repo's plain-C restatements (oracle/*.c);
* ``_ref/libref_fbbt.so`` — the reference's own LinearHandler, compiled from
  /root/reference/src/base by oracle/Makefile (built in the container, shipped
  prebuilt to the GPU box; loaded RTLD_LAZY because the unused LAPACK symbol
  ``dsyevr_`` referenced by Eigen.cpp stays unresolved).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  Nothing in minotaur_amd/ does.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_ORACLE = os.path.join(HERE, 'liboracle.so')
LIB_REF = os.path.join(HERE, '_ref', 'libref_fbbt.so')

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_lib = None
_ref = None


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_P)


def build_oracle():
    """(Re)build liboracle.so from oracle/*.c (gcc; a second or two)."""
    import subprocess
    subprocess.run(['make', '-s', '-C', HERE, 'oracle'], check=True)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(('.c', '.h'))]
        if (not os.path.exists(LIB_ORACLE) or
                os.path.getmtime(LIB_ORACLE) < max(os.path.getmtime(s) for s in srcs)):
            build_oracle()
        _lib = ctypes.CDLL(LIB_ORACLE)
        _lib.orc_linear_fbbt.restype = _I
        _lib.orc_linear_fbbt.argtypes = [_I, _I] + [_P] * 8 + [_I, _P, _P, _I, _I,
                                          _P, _P, _P, _P, _I, _D, _P, _P, _I,
                                          _P, _P, _P, _I]
        if hasattr(_lib, 'orc_simplex_solve'):
            pass
    return _lib


def have_ref() -> bool:
    return os.path.exists(LIB_REF)


def ref_lib():
    global _ref
    if _ref is None:
        _ref = ctypes.CDLL(LIB_REF, mode=os.RTLD_LAZY)
        _ref.ref_linear_fbbt.restype = _I
        _ref.ref_linear_fbbt.argtypes = [_I, _I] + [_P] * 7 + [_P, _I, _P, _P, _D,
                                          _I, _D, _I, _P, _P, _P, _P, _P, _P, _I,
                                          _P, _P, _P, _P]
    return _ref


class FbbtResult:
    def __init__(self, lb, ub, infeas, nmods, mod_var=None, mod_lu=None,
                 mod_val=None, seconds=None):
        self.lb, self.ub, self.infeas, self.nmods = lb, ub, infeas, nmods
        self.mod_var, self.mod_lu, self.mod_val = mod_var, mod_lu, mod_val
        self.seconds = seconds

    def mods(self, b):
        """Mod log of node ``b`` as [(var, lu, value)] (capped at mod_cap)."""
        k = min(int(self.nmods[b]), self.mod_var.shape[1])
        return [(int(self.mod_var[b, t]), int(self.mod_lu[b, t]),
                 float(self.mod_val[b, t])) for t in range(k)]


def _inc_ub(p, incumbent):
    # LinearHandler.cpp:1637: spool->getBestSolutionValue() - obj constant
    if incumbent is None or not math.isfinite(incumbent):
        return 0, 0.0
    return 1, float(incumbent) - float(p.obj_const)


def linear_fbbt(p, lb, ub, incumbent=None, mod_cap=0, nthreads=1):
    """C restatement of LinearHandler::presolveNode over a batch of boxes."""
    lb = np.ascontiguousarray(lb, dtype=np.float64)
    ub = np.ascontiguousarray(ub, dtype=np.float64)
    B = lb.shape[0]
    colptr, rowidx = p.csc_pattern()
    oidx, oval = p.obj_sparse()
    olb = np.empty_like(lb)
    oub = np.empty_like(ub)
    infeas = np.zeros(B, dtype=np.int32)
    nmods = np.zeros(B, dtype=np.int32)
    mv = ml = mval = None
    if mod_cap > 0:
        mv = np.full((B, mod_cap), -1, dtype=np.int32)
        ml = np.full((B, mod_cap), -1, dtype=np.int32)
        mval = np.zeros((B, mod_cap))
    has, incv = _inc_ub(p, incumbent)
    lib().orc_linear_fbbt(p.n, p.m, _ptr(p.rowptr), _ptr(p.colidx), _ptr(p.val),
                          _ptr(p.rlo), _ptr(p.rhi), _ptr(colptr), _ptr(rowidx),
                          _ptr(p.vtype), len(oidx), _ptr(oidx), _ptr(oval),
                          p.cons_bad(), B, _ptr(lb), _ptr(ub), _ptr(olb),
                          _ptr(oub), has, incv, _ptr(infeas), _ptr(nmods),
                          mod_cap, _ptr(mv), _ptr(ml), _ptr(mval), nthreads)
    return FbbtResult(olb, oub, infeas, nmods, mv, ml, mval)


def ref_linear_fbbt(p, lb, ub, incumbent=None, mod_cap=0):
    """The reference's own LinearHandler::presolveNode, node by node."""
    lb = np.ascontiguousarray(lb, dtype=np.float64)
    ub = np.ascontiguousarray(ub, dtype=np.float64)
    B = lb.shape[0]
    oidx, oval = p.obj_sparse()
    olb = np.empty_like(lb)
    oub = np.empty_like(ub)
    infeas = np.zeros(B, dtype=np.int32)
    nmods = np.zeros(B, dtype=np.int32)
    mv = ml = mval = None
    if mod_cap > 0:
        mv = np.full((B, mod_cap), -1, dtype=np.int32)
        ml = np.full((B, mod_cap), -1, dtype=np.int32)
        mval = np.zeros((B, mod_cap))
    secs = np.zeros(1)
    has = 0 if incumbent is None or not math.isfinite(incumbent) else 1
    inc = float(incumbent) if has else 0.0
    ref_lib().ref_linear_fbbt(p.n, p.m, _ptr(p.rowptr), _ptr(p.colidx), _ptr(p.val),
                              _ptr(p.rlo), _ptr(p.rhi), _ptr(p.vtype), _ptr(p.vlb),
                              _ptr(p.vub), len(oidx), _ptr(oidx), _ptr(oval),
                              float(p.obj_const), has, inc, B, _ptr(lb), _ptr(ub),
                              _ptr(olb), _ptr(oub), _ptr(infeas), _ptr(nmods),
                              mod_cap, _ptr(mv), _ptr(ml), _ptr(mval), _ptr(secs))
    return FbbtResult(olb, oub, infeas, nmods, mv, ml, mval, float(secs[0]))


# ---------------------------------------------------------------------------
# LP: bounded dual simplex restatement (liboracle) and scipy HiGHS
# ---------------------------------------------------------------------------
def lp_csc(p):
    """CSC of the constraint matrix (rows ascending inside each column)."""
    colptr, rowidx = p.csc_pattern()
    cval = np.empty(p.nnz)
    fill = colptr[:-1].copy()
    for i in range(p.m):
        for k in range(p.rowptr[i], p.rowptr[i + 1]):
            j = p.colidx[k]
            cval[fill[j]] = p.val[k]
            fill[j] += 1
    return colptr, rowidx, cval


class WarmStart:
    """Optimal basis of an LP: basic column per row, status of every column
    (0 at lb, 1 at ub, 2 free, 3 basic) and the dense basis inverse."""

    def __init__(self, head, st, binv, d):
        self.head, self.st, self.binv, self.d = head, st, binv, d


def _lp_sig(l):
    l.orc_dual_simplex_batch.restype = _I
    l.orc_dual_simplex_batch.argtypes = [_I, _I] + [_P] * 6 + [_I, _P, _P, _P, _P, _P, _P,
                                         _I, _P, _P, _P, _P, _I, _I]
    l.orc_dual_simplex_root.restype = _I
    l.orc_dual_simplex_root.argtypes = [_I, _I] + [_P] * 8 + [_I] + [_P] * 8


def dual_simplex(p, LB, UB, ws=None, iter_limit=10000, nthreads=1, want_x=False, pfi=0):
    """Per-node LP solves; returns (status[B], obj[B] incl. constant, iters[B], x).
    pfi > 0 (with a shared ``ws``): the product-form arithmetic of K3P with an
    eta file of ``pfi`` columns, and the dense solve for an LP that fills it
    (what the GPU runs for a shared warm start)."""
    l = lib()
    _lp_sig(l)
    LB = np.ascontiguousarray(LB, dtype=np.float64)
    UB = np.ascontiguousarray(UB, dtype=np.float64)
    B = LB.shape[0]
    colptr, rowidx, cval = lp_csc(p)
    st = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    it = np.zeros(B, dtype=np.int32)
    x = np.zeros((B, p.n)) if want_x else None
    h = s = bi = dd = None
    if ws is not None:
        h = np.ascontiguousarray(ws.head, dtype=np.int32)
        s = np.ascontiguousarray(ws.st, dtype=np.int8)
        bi = np.ascontiguousarray(ws.binv, dtype=np.float64)
        if ws.d is not None:
            dd = np.ascontiguousarray(ws.d, dtype=np.float64)
        else:
            pfi = 0  # no d: reduced costs rebuilt for this objective, dense K3 on the GPU
    l.orc_dual_simplex_batch(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval), _ptr(p.obj),
                             _ptr(p.rlo), _ptr(p.rhi), B, _ptr(LB), _ptr(UB), _ptr(h),
                             _ptr(s), _ptr(bi), _ptr(dd), iter_limit, _ptr(st), _ptr(obj), _ptr(x),
                             _ptr(it), nthreads, int(pfi))
    obj = obj + p.obj_const
    return st, obj, it, x


def dual_simplex_nodes(p, LB, UB, ws, iter_limit=10000, nthreads=1):
    """Per-node warm starts in and out (dense arithmetic, K3/K3L): ws is a
    WarmStart whose arrays carry a leading batch axis (binv row-major), or
    None (slack basis); ws.d None rebuilds the reduced costs for p.obj;
    returns (status, obj incl. constant, iters, x, WarmStart out)."""
    l = lib()
    l.orc_dual_simplex_nodes.restype = _I
    l.orc_dual_simplex_nodes.argtypes = [_I, _I] + [_P] * 6 + [_I] + [_P] * 6 + [_I] + \
        [_P] * 8 + [_I]
    LB = np.ascontiguousarray(LB, dtype=np.float64)
    UB = np.ascontiguousarray(UB, dtype=np.float64)
    B = LB.shape[0]
    colptr, rowidx, cval = lp_csc(p)
    N = p.n + p.m
    h = s = bi = dd = None
    if ws is not None:    # None: slack basis
        h = np.ascontiguousarray(ws.head, dtype=np.int32)
        s = np.ascontiguousarray(ws.st, dtype=np.int8)
        bi = np.ascontiguousarray(ws.binv, dtype=np.float64)
        if ws.d is not None:  # None: reduced costs rebuilt for p's objective
            dd = np.ascontiguousarray(ws.d, dtype=np.float64)
    st = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    it = np.zeros(B, dtype=np.int32)
    x = np.zeros((B, p.n))
    wo = WarmStart(np.zeros((B, p.m), np.int32), np.zeros((B, N), np.int8),
                   np.zeros((B, p.m, p.m)), np.zeros((B, N)))
    l.orc_dual_simplex_nodes(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval), _ptr(p.obj),
                             _ptr(p.rlo), _ptr(p.rhi), B, _ptr(LB), _ptr(UB), _ptr(h), _ptr(s),
                             _ptr(bi), _ptr(dd), iter_limit, _ptr(st), _ptr(obj), _ptr(x),
                             _ptr(it), _ptr(wo.head), _ptr(wo.st), _ptr(wo.binv), _ptr(wo.d),
                             nthreads)
    return st, obj + p.obj_const, it, x, wo


def chain_solve(p, ws, iter_limit=10000):
    """One LP of p from the single warm start ws (None: slack basis; ws.d
    None: reduced costs rebuilt for p.obj) with its final basis back when
    optimal / at the iteration limit: minotaur_amd.obbt.obbt_chained's solve
    step restated on the CPU (K3's dense arithmetic)."""
    W = None if ws is None else WarmStart(ws.head[None], ws.st[None], ws.binv[None], None)
    st, obj, it, x, wo = dual_simplex_nodes(p, p.vlb[None], p.vub[None], W, iter_limit)
    out = None
    if st[0] in (0, 6):
        out = WarmStart(wo.head[0], wo.st[0], wo.binv[0], None)
    return int(st[0]), float(obj[0]), x[0], out


PATH_MAX = 32     # ORC_PATH_MAX = MGPU_PATH_MAX: pivots per path warm start


def dual_simplex_path(p, LB, UB, ws, k_in, path_in, st_in, pfi, inherit, iter_limit=10000,
                      nthreads=1, want_x=True):
    """Basis warm starts (the batched tree's warm mode 2; orc_dual_simplex_path_batch):
    node b starts from its parent's basis: statuses st_in[b] and the k_in[b]
    basic columns outside the shared root basis ``ws`` (path_in[b], ascending),
    rebuilt from the root inverse by column replacement with partial pivoting;
    k_in <= 0 = the root basis.  Product form with ``pfi`` etas (the GPU's
    K3P), dense continuation past it.  Returns (status, obj incl. constant,
    own pivots, x, k_out, path_out, st_out): the node's final basis in the
    same form for its children (k_out 0 = restart from the root)."""
    l = lib()
    f = l.orc_dual_simplex_path_batch
    f.restype = _I
    f.argtypes = [_I, _I] + [_P] * 6 + [_I, _P, _P] + [_P] * 7 + [_I] + [_P] * 7 + [_I, _I, _I]
    LB = np.ascontiguousarray(LB, dtype=np.float64)
    UB = np.ascontiguousarray(UB, dtype=np.float64)
    B = LB.shape[0]
    N = p.n + p.m
    colptr, rowidx, cval = lp_csc(p)
    h = np.ascontiguousarray(ws.head, dtype=np.int32)
    s = np.ascontiguousarray(ws.st, dtype=np.int8)
    bi = np.ascontiguousarray(ws.binv, dtype=np.float64)
    dd = np.ascontiguousarray(ws.d, dtype=np.float64)
    k_in = np.ascontiguousarray(k_in, dtype=np.int32)
    path_in = np.ascontiguousarray(path_in, dtype=np.uint32).reshape(B, PATH_MAX)
    st_in = np.ascontiguousarray(st_in, dtype=np.int8).reshape(B, N)
    st = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    it = np.zeros(B, dtype=np.int32)
    x = np.zeros((B, p.n)) if want_x else None
    k_out = np.zeros(B, dtype=np.int32)
    path_out = np.zeros((B, PATH_MAX), dtype=np.uint32)
    st_out = np.zeros((B, N), dtype=np.int8)
    f(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval), _ptr(p.obj), _ptr(p.rlo), _ptr(p.rhi),
      B, _ptr(LB), _ptr(UB), _ptr(h), _ptr(s), _ptr(bi), _ptr(dd), _ptr(k_in), _ptr(path_in),
      _ptr(st_in), iter_limit, _ptr(st), _ptr(obj), _ptr(x), _ptr(it), _ptr(k_out),
      _ptr(path_out), _ptr(st_out), int(pfi), int(inherit), nthreads)
    return st, obj + p.obj_const, it, x, k_out, path_out, st_out


def dual_simplex_root(p, lb=None, ub=None, iter_limit=100000):
    l = lib()
    _lp_sig(l)
    lb = np.ascontiguousarray(p.vlb if lb is None else lb, dtype=np.float64)
    ub = np.ascontiguousarray(p.vub if ub is None else ub, dtype=np.float64)
    colptr, rowidx, cval = lp_csc(p)
    head = np.zeros(p.m, dtype=np.int32)
    st = np.zeros(p.n + p.m, dtype=np.int8)
    binv = np.zeros((p.m, p.m))
    dred = np.zeros(p.n + p.m)
    obj = np.zeros(1)
    x = np.zeros(p.n)
    y = np.zeros(p.m)
    it = np.zeros(1, dtype=np.int32)
    status = l.orc_dual_simplex_root(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval),
                                     _ptr(p.obj), _ptr(p.rlo), _ptr(p.rhi), _ptr(lb), _ptr(ub),
                                     iter_limit, _ptr(head), _ptr(st), _ptr(binv), _ptr(dred),
                                     _ptr(obj), _ptr(x), _ptr(y), _ptr(it))
    return (status, float(obj[0]) + p.obj_const, x, y, int(it[0]),
            WarmStart(head, st, binv, dred))


def highs(p, lb=None, ub=None):
    """scipy HiGHS: (EngineStatus numeric, objective incl. constant)."""
    from scipy.optimize import linprog
    from scipy.sparse import csr_matrix
    lb = p.vlb if lb is None else lb
    ub = p.vub if ub is None else ub
    A = csr_matrix((p.val, p.colidx, p.rowptr), shape=(p.m, p.n))
    fin_hi = np.isfinite(p.rhi)
    fin_lo = np.isfinite(p.rlo)
    eq = fin_hi & fin_lo & (p.rlo == p.rhi)
    ub_rows = fin_hi & ~eq
    lo_rows = fin_lo & ~eq
    import scipy.sparse as sp
    A_ub = sp.vstack([A[ub_rows], -A[lo_rows]]) if (ub_rows.any() or lo_rows.any()) else None
    b_ub = np.concatenate([p.rhi[ub_rows], -p.rlo[lo_rows]]) if A_ub is not None else None
    A_eq = A[eq] if eq.any() else None
    b_eq = p.rlo[eq] if eq.any() else None
    bounds = [(None if not np.isfinite(a) else a, None if not np.isfinite(b) else b)
              for a, b in zip(lb, ub)]
    if np.any(np.asarray(lb) > np.asarray(ub)):
        return 2, math.inf
    r = linprog(p.obj, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=bounds,
                method='highs')
    if r.status == 0:
        return 0, float(r.fun) + p.obj_const
    if r.status == 2:
        return 2, math.inf
    if r.status == 3:
        return 4, -math.inf
    return 12, math.nan


# ---------------------------------------------------------------------------
# Quadratic node FBBT: C restatement (liboracle) and the reference's own
# QuadHandler::presolveNode (_ref/libref_fbbt.so, oracle/ref/ref_quad.cpp)
# ---------------------------------------------------------------------------
class _QSpec(ctypes.Structure):
    _fields_ = [('nv0', _I), ('nv', _I), ('vtype', _P), ('vlb', _P), ('vub', _P),
                ('nsq', _I), ('sq_x', _P), ('sq_y', _P),
                ('nbil', _I), ('bil_x0', _P), ('bil_x1', _P), ('bil_y', _P),
                ('ncon', _I), ('lptr', _P), ('lvar', _P), ('lval', _P),
                ('qptr', _P), ('qv1', _P), ('qv2', _P), ('qval', _P),
                ('clb', _P), ('cub', _P), ('has_obj', _I), ('obj_const', _D)]


def qspec(qp):
    """ctypes view of a minotaur_amd.quad.QuadProblem (arrays stay owned by qp)."""
    f = {}
    for k in ('vtype', 'sq_x', 'sq_y', 'bil_x0', 'bil_x1', 'bil_y', 'lptr', 'lvar', 'qptr',
              'qv1', 'qv2'):
        a = np.ascontiguousarray(getattr(qp, k), dtype=np.int32)
        qp._keep.append(a)
        f[k] = _ptr(a)
    for k in ('vlb', 'vub', 'lval', 'qval', 'clb', 'cub'):
        a = np.ascontiguousarray(getattr(qp, k), dtype=np.float64)
        qp._keep.append(a)
        f[k] = _ptr(a)
    return _QSpec(nv0=qp.nv0, nv=qp.nv, nsq=qp.nsq, nbil=qp.nbil, ncon=qp.ncon,
                  has_obj=int(qp.has_obj), obj_const=float(qp.obj_const), **f)


class QuadFbbtResult:
    def __init__(self, lb, ub, infeas, nmods, rows, kind=None, idx=None, v1=None, v2=None,
                 seconds=None):
        self.lb, self.ub, self.infeas, self.nmods, self.rows = lb, ub, infeas, nmods, rows
        self.kind, self.idx, self.v1, self.v2 = kind, idx, v1, v2
        self.seconds = seconds


def _quad_out(qp, B, mod_cap):
    olb = np.empty((B, qp.nv))
    oub = np.empty((B, qp.nv))
    rows = np.empty((B, qp.nrow_state))
    infeas = np.zeros(B, dtype=np.int32)
    nmods = np.zeros(B, dtype=np.int32)
    kind = idx = v1 = v2 = None
    if mod_cap > 0:
        kind = np.full((B, mod_cap), -1, dtype=np.int32)
        idx = np.full((B, mod_cap), -1, dtype=np.int32)
        v1 = np.zeros((B, mod_cap))
        v2 = np.zeros((B, mod_cap))
    return olb, oub, rows, infeas, nmods, kind, idx, v1, v2


def quad_root_rows(qp, lb=None, ub=None):
    """Secant / McCormick row state of QuadHandler::relax_ at a box (C)."""
    L = lib()
    L.orc_quad_rows.restype = None
    L.orc_quad_rows.argtypes = [ctypes.POINTER(_QSpec), _P, _P, _P]
    lb = np.ascontiguousarray(qp.vlb if lb is None else lb, dtype=np.float64)
    ub = np.ascontiguousarray(qp.vub if ub is None else ub, dtype=np.float64)
    rows = np.empty(qp.nrow_state)
    s = qspec(qp)
    L.orc_quad_rows(ctypes.byref(s), _ptr(lb), _ptr(ub), _ptr(rows))
    return rows


def quad_update_rows(qp, lb, ub, rows):
    """upSqCon_ / upBilCon_ over every product at box lb/ub on a copy of the
    row state rows (C); postSolveRootNode's rewrite after OBBT."""
    L = lib()
    L.orc_quad_update_rows.restype = None
    L.orc_quad_update_rows.argtypes = [ctypes.POINTER(_QSpec), _P, _P, _P]
    lb = np.ascontiguousarray(lb, dtype=np.float64).copy()
    ub = np.ascontiguousarray(ub, dtype=np.float64).copy()
    out = np.ascontiguousarray(rows, dtype=np.float64).copy()
    s = qspec(qp)
    L.orc_quad_update_rows(ctypes.byref(s), _ptr(lb), _ptr(ub), _ptr(out))
    return out


def quad_fbbt(qp, lb, ub, incumbent=None, qt=1, rows=None, mod_cap=0):
    """C restatement of QuadHandler::presolveNode over a batch of boxes.
    rows: [R] shared or [B, R] per node (default: root rows)."""
    L = lib()
    L.orc_quad_fbbt_batch.restype = _I
    L.orc_quad_fbbt_batch.argtypes = [ctypes.POINTER(_QSpec), _I, _P, _P, _D, _I, _P,
                                      ctypes.c_long, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P]
    lb = np.ascontiguousarray(lb, dtype=np.float64)
    ub = np.ascontiguousarray(ub, dtype=np.float64)
    B = lb.shape[0]
    if rows is None:
        rows = quad_root_rows(qp)
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    stride = 0 if rows.ndim == 1 else qp.nrow_state
    best = math.inf if incumbent is None else float(incumbent)
    olb, oub, orows, infeas, nmods, kind, idx, v1, v2 = _quad_out(qp, B, mod_cap)
    s = qspec(qp)
    r = L.orc_quad_fbbt_batch(ctypes.byref(s), B, _ptr(lb), _ptr(ub), best, int(qt),
                              _ptr(rows), stride, _ptr(olb), _ptr(oub), _ptr(infeas),
                              _ptr(nmods), _ptr(orows), mod_cap, _ptr(kind), _ptr(idx),
                              _ptr(v1), _ptr(v2))
    if r != 0:
        raise RuntimeError('orc_quad_fbbt_batch: propagation cap hit')
    return QuadFbbtResult(olb, oub, infeas, nmods, orows, kind, idx, v1, v2)


def ref_quad_root_rows(qp):
    R = ref_lib()
    R.ref_quad_root_rows.restype = _I
    R.ref_quad_root_rows.argtypes = [ctypes.POINTER(_QSpec), _P]
    rows = np.empty(qp.nrow_state)
    s = qspec(qp)
    R.ref_quad_root_rows(ctypes.byref(s), _ptr(rows))
    return rows


def ref_quad_fbbt(qp, lb, ub, incumbent=None, qt=1, rows=None, mod_cap=0):
    """The reference's own QuadHandler::presolveNode, node by node (shared
    row state `rows`, default the reference's relax_ rows at the root)."""
    R = ref_lib()
    R.ref_quad_fbbt.restype = _I
    R.ref_quad_fbbt.argtypes = [ctypes.POINTER(_QSpec), _I, _D, _I, _P, _I, _P, _P, _P, _P,
                                _P, _P, _P, _I, _P, _P, _P, _P, _P]
    lb = np.ascontiguousarray(lb, dtype=np.float64)
    ub = np.ascontiguousarray(ub, dtype=np.float64)
    B = lb.shape[0]
    if rows is None:
        rows = ref_quad_root_rows(qp)
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    assert rows.ndim == 1
    olb, oub, orows, infeas, nmods, kind, idx, v1, v2 = _quad_out(qp, B, mod_cap)
    secs = np.zeros(1)
    has = 0 if incumbent is None or not math.isfinite(incumbent) else 1
    s = qspec(qp)
    R.ref_quad_fbbt(ctypes.byref(s), has, float(incumbent) if has else 0.0, int(qt),
                    _ptr(rows), B, _ptr(lb), _ptr(ub), _ptr(olb), _ptr(oub), _ptr(infeas),
                    _ptr(nmods), _ptr(orows), mod_cap, _ptr(kind), _ptr(idx), _ptr(v1),
                    _ptr(v2), _ptr(secs))
    return QuadFbbtResult(olb, oub, infeas, nmods, orows, kind, idx, v1, v2, float(secs[0]))


def lp_bound(p, cols, signs, lb=None, ub=None, ws=None, iter_limit=100000, nthreads=1, pfi=0):
    """C restatement of the bound LPs (min sign_b * x[col_b] on one box,
    warm-started from ws = oracle WarmStart, binv row-major); pfi as in
    dual_simplex."""
    L = lib()
    L.orc_lp_bound_batch.restype = _I
    L.orc_lp_bound_batch.argtypes = ([_I, _I] + [_P] * 7 + [_I] + [_P] * 5 + [_I] + [_P] * 4
                                     + [_I, _I])
    colptr, rowidx, cval = lp_csc(p)
    lb = np.ascontiguousarray(p.vlb if lb is None else lb, dtype=np.float64)
    ub = np.ascontiguousarray(p.vub if ub is None else ub, dtype=np.float64)
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    signs = np.ascontiguousarray(signs, dtype=np.float64)
    B = cols.size
    st = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    it = np.zeros(B, dtype=np.int32)
    x = np.zeros((B, p.n))
    wh = wst = wb = None
    if ws is not None:
        wh = np.ascontiguousarray(ws.head, dtype=np.int32)
        wst = np.ascontiguousarray(ws.st, dtype=np.int8)
        wb = np.ascontiguousarray(ws.binv, dtype=np.float64)
    L.orc_lp_bound_batch(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval), _ptr(p.rlo),
                         _ptr(p.rhi), _ptr(lb), _ptr(ub), B, _ptr(cols), _ptr(signs), _ptr(wh),
                         _ptr(wst), _ptr(wb), iter_limit, _ptr(st), _ptr(obj), _ptr(x), _ptr(it),
                         nthreads, int(pfi))
    return st, obj, it, x


def highs_obj(p, c, lb=None, ub=None):
    """scipy HiGHS with objective vector c (no constant)."""
    import dataclasses
    q = dataclasses.replace(p, obj=np.asarray(c, dtype=np.float64), obj_const=0.0)
    return highs(q, lb, ub)


def highs_milp(p, time_limit=60.0):
    """scipy HiGHS MILP (Binary/Integer columns integral): (status, objective
    incl. constant); status 0 optimal, 2 infeasible, 4 unbounded, 12 other."""
    from scipy.optimize import Bounds, LinearConstraint, milp
    from scipy.sparse import csr_matrix
    A = csr_matrix((p.val, p.colidx, p.rowptr), shape=(p.m, p.n))
    cons = [LinearConstraint(A, p.rlo, p.rhi)] if p.m > 0 else []
    integ = np.isin(p.vtype, (0, 1)).astype(int)
    r = milp(p.obj, constraints=cons, integrality=integ, bounds=Bounds(p.vlb, p.vub),
             options={'time_limit': time_limit, 'mip_rel_gap': 1e-9})
    if r.status == 0:
        return 0, float(r.fun) + p.obj_const
    if r.status == 2:
        return 2, math.inf
    if r.status == 3:
        return 4, -math.inf
    return 12, math.nan


# ---------------------------------------------------------------------------
# Node decision: PCBProcessor::shouldPrune_ + IntVarHandler::isFeasible
# ---------------------------------------------------------------------------
DEC_BRANCH, DEC_INFEAS, DEC_PRUNED, DEC_FEASIBLE, DEC_ENGINE = 0, 1, 2, 3, 4
NODE_INFEASIBLE, NODE_HIT_UB, NODE_CONTINUE = 1, 2, 5   # NodeStatus (Types.h:184-194)


def ref_node_decide(vtype, status, obj, x, incumbent=None):
    """The reference's own PCBProcessor::shouldPrune_ (PCBProcessor.cpp:400-523)
    then, for kept nodes, IntVarHandler::isFeasible (IntVarHandler.cpp:54-84)
    (_ref/libref_fbbt.so, oracle/ref/ref_decide.cpp).  Returns (prune,
    node_status, feas (-1 = not evaluated), inf_meas) per node."""
    R = ref_lib()
    R.ref_node_decide.restype = _I
    R.ref_node_decide.argtypes = [_I, _P, _I, _P, _P, _P, _I, _D, _P, _P, _P, _P]
    vtype = np.ascontiguousarray(vtype, dtype=np.int32)
    status = np.ascontiguousarray(status, dtype=np.int32)
    obj = np.ascontiguousarray(obj, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    B = status.size
    prune = np.zeros(B, np.int32)
    nstat = np.zeros(B, np.int32)
    feas = np.zeros(B, np.int32)
    meas = np.zeros(B)
    has = 0 if incumbent is None or not math.isfinite(incumbent) else 1
    R.ref_node_decide(vtype.size, _ptr(vtype), B, _ptr(status), _ptr(obj), _ptr(x), has,
                      float(incumbent) if has else 0.0, _ptr(prune), _ptr(nstat), _ptr(feas),
                      _ptr(meas))
    return prune, nstat, feas, meas


def decision_from_ref(prune, nstat, feas):
    """The engine's decision code (include/mgpu.h mgpu_node_decide_dev) for a
    reference (shouldPrune_, NodeStatus, isFeasible) outcome."""
    dec = np.full(prune.size, DEC_ENGINE, np.int32)
    dec[(prune == 1) & (nstat == NODE_INFEASIBLE)] = DEC_INFEAS
    dec[(prune == 1) & (nstat == NODE_HIT_UB)] = DEC_PRUNED
    dec[(prune == 0) & (nstat == NODE_CONTINUE) & (feas == 1)] = DEC_FEASIBLE
    dec[(prune == 0) & (nstat == NODE_CONTINUE) & (feas == 0)] = DEC_BRANCH
    return dec


def node_decide(vtype, status, obj, x, incumbent=math.inf, fbbt_infeas=None, abs_tol=1e-6,
                rel_tol=1e-6, cutoff=math.inf, int_tol=1e-6):
    """CPU restatement of node_decide_kernel: shouldPrune_'s status switch
    (PCBProcessor.cpp:409-520, contOnErr_ false) and IntVarHandler::isFeasible
    with its sequential inf_meas (IntVarHandler.cpp:64-79).  Returns
    (decision, inf_meas)."""
    ints = np.isin(np.asarray(vtype), (0, 1))
    B = len(status)
    dec = np.full(B, DEC_ENGINE, np.int32)
    meas = np.zeros(B)
    for b in range(B):
        st, sv = int(status[b]), float(obj[b])
        if fbbt_infeas is not None and fbbt_infeas[b]:
            dec[b] = DEC_INFEAS
        elif st in (2, 3, 8, 10, 11):
            dec[b] = DEC_INFEAS
        elif st == 5:
            dec[b] = DEC_PRUNED
        else:
            cut = incumbent
            if st in (0, 1, 6) and (sv >= cut - abs_tol or sv >= cut - abs(cut) * rel_tol
                                    or sv >= cutoff):
                dec[b] = DEC_PRUNED
            else:   # 7 / 9: NodeContinue with the parent's bound (:444-467)
                s, frac = 0.0, False
                for j in np.nonzero(ints)[0]:
                    v = float(x[b, j])
                    f = abs(v - math.floor(v + 0.5))
                    if f > int_tol:
                        frac = True
                        s += f
                meas[b] = s
                # 4 / 12 / others: shouldPrune_ keeps the node, isFeasible
                # runs, the engine reports a problem
                dec[b] = (DEC_ENGINE if st not in (0, 1, 6, 7, 9) else
                          DEC_BRANCH if frac else DEC_FEASIBLE)
    return dec, meas


def dual_simplex_rows(p, LB, UB, nr, vals, ws=None, iter_limit=10000, nthreads=1,
                      want_x=False, want_ws=False):
    """Per-node rows (mgpu_lp_solve_rows): node b solves ``p`` with the entries
    and row bounds of ``nr`` (a quad.NodeRows) taken from ``vals[b]``, from
    the warm basis ``ws`` (head/st; 1-D shared or per node) refactored for
    its matrix: from ws.binv (the shared root inverse, row-major) by column
    replacement, else by Gauss-Jordan.  Returns (status, obj incl.
    constant, iters, x)."""
    l = lib()
    l.orc_dual_simplex_rows.restype = _I
    l.orc_dual_simplex_rows.argtypes = ([_I, _I] + [_P] * 6 + [_I] + [_P] * 3 + [_I, _I]
                                        + [_P] * 2 + [_I] + [_P] * 5 + [_I, _I] + [_P] * 4
                                        + [_I, _P, _P, _P])
    LB = np.ascontiguousarray(LB, dtype=np.float64)
    UB = np.ascontiguousarray(UB, dtype=np.float64)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    B = LB.shape[0]
    colptr, rowidx, cval = lp_csc(p)
    # CSR entry -> CSC position (lp_csc fills in CSR order)
    csc_of = np.empty(p.nnz, dtype=np.int32)
    fill = colptr[:-1].copy()
    for k in range(p.nnz):
        j = p.colidx[k]
        csc_of[k] = fill[j]
        fill[j] += 1
    cpos = np.ascontiguousarray(csc_of[nr.coef_pos], dtype=np.int32)
    csrc = np.ascontiguousarray(nr.coef_src, dtype=np.int32)
    row = np.ascontiguousarray(nr.row_idx, dtype=np.int32)
    lo = np.ascontiguousarray(nr.lo_src, dtype=np.int32)
    hi = np.ascontiguousarray(nr.hi_src, dtype=np.int32)
    h = s = b0 = None
    shared = 1
    if ws is not None:
        h = np.ascontiguousarray(ws.head, dtype=np.int32)
        s = np.ascontiguousarray(ws.st, dtype=np.int8)
        shared = 1 if h.ndim == 1 else 0
        # the root inverse (row-major) of a shared warm start: the column
        # replacement of K3R / K3L; without it, the Gauss-Jordan refactor
        if ws.binv is not None and shared:
            b0 = np.ascontiguousarray(ws.binv, dtype=np.float64)
    st = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    it = np.zeros(B, dtype=np.int32)
    x = np.zeros((B, p.n)) if want_x else None
    ho = np.zeros((B, p.m), dtype=np.int32) if want_ws else None
    so = np.zeros((B, p.n + p.m), dtype=np.int8) if want_ws else None
    l.orc_dual_simplex_rows(p.n, p.m, _ptr(colptr), _ptr(rowidx), _ptr(cval), _ptr(p.obj),
                            _ptr(p.rlo), _ptr(p.rhi), B, _ptr(LB), _ptr(UB), _ptr(vals),
                            int(nr.stride), int(cpos.size), _ptr(cpos), _ptr(csrc), int(row.size),
                            _ptr(row), _ptr(lo), _ptr(hi), _ptr(h), _ptr(s), shared, iter_limit,
                            _ptr(st), _ptr(obj), _ptr(x), _ptr(it), nthreads, _ptr(b0),
                            _ptr(ho), _ptr(so))
    if want_ws:   # the final bases (head [B][m], statuses [B][n+m]; status 0 / 6)
        return st, obj + p.obj_const, it, x, ho, so
    return st, obj + p.obj_const, it, x
