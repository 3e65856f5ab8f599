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
