"""AMPL ``.nl`` reader (text ``g`` and binary ``b`` formats) -> linear data.

This is SURVEY §8(f) row 2 (the on-disk input format of the hot path).  The
reference reads ``.nl`` files through ASL in ``AMPLInterface::readInstance``
(src/interfaces/AMPLInterface.cpp); ASL is not vendored, so this module reads
the documented ``.nl`` layout directly and keeps only what the LP/FBBT path
consumes: variable bounds and types, constraint bounds, the linear
(Jacobian) part of every row, the linear objective gradient and constant, and
which rows / the objective carry a nonlinear expression.

Variable types follow the AMPL ordering rules the ``.nl`` header encodes
(nonlinear variables first, integers last inside each group; then linear
continuous, binary, integer) and use the reference's ``VariableType``
numerics (src/base/Types.h:83-89): 0 Binary, 1 Integer, 4 Continuous.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field

import numpy as np

BINARY, INTEGER, CONTINUOUS = 0, 1, 4

# Arity of AMPL expression opcodes (o<k>); -1 = n-ary with a count operand.
_BINARY_OPS = {0, 1, 2, 3, 4, 5, 6, 20, 21, 22, 23, 24, 28, 29, 30, 48, 49, 55,
               56, 57, 58, 73}
_UNARY_OPS = {13, 14, 15, 16, 34, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
              49, 50, 51, 52, 53, 74}
_NARY_OPS = {11, 12, 54, 59, 60, 61, 70, 71}


@dataclass
class NlModel:
    name: str
    n: int
    m: int
    var_lb: np.ndarray
    var_ub: np.ndarray
    var_type: np.ndarray          # int32, reference VariableType numerics
    con_lb: np.ndarray
    con_ub: np.ndarray
    rows: list                    # per row: list of (col, coef) in file order
    con_nonlinear: np.ndarray     # bool per row
    obj_sense: int = 0            # 0 minimize, 1 maximize
    obj_grad: list = field(default_factory=list)
    obj_const: float = 0.0
    obj_nonlinear: bool = False
    # raw expression trees (token lists), kept for OA / QP builders
    con_expr: dict = field(default_factory=dict)
    obj_expr: list = field(default_factory=list)

    def linear_rows(self):
        """Indices of rows without a nonlinear part."""
        return [i for i in range(self.m) if not self.con_nonlinear[i]]


class _TextStream:
    def __init__(self, text: str):
        self.lines = text.splitlines()
        self.pos = 0

    def line(self) -> str:
        s = self.lines[self.pos]
        self.pos += 1
        return s.split('#', 1)[0].strip()

    def eof(self) -> bool:
        return self.pos >= len(self.lines)

    # expression tokens -----------------------------------------------------
    def expr(self):
        """Read one expression tree in prefix form; returns a nested tuple."""
        tok = self.line()
        k, rest = tok[0], tok[1:]
        if k == 'n' or k == 'l' or k == 's':
            return ('n', float(rest))
        if k == 'v':
            return ('v', int(rest))
        if k == 'h':
            return ('h', rest)
        if k == 'f':
            fi, na = rest.split()
            return ('f', int(fi), [self.expr() for _ in range(int(na))])
        if k == 'o':
            op = int(rest)
            if op in _NARY_OPS:
                cnt = int(self.line())
                return ('o', op, [self.expr() for _ in range(cnt)])
            if op == 35:  # if-then-else
                return ('o', op, [self.expr() for _ in range(3)])
            if op == 65:  # if-symbolic
                return ('o', op, [self.expr() for _ in range(3)])
            if op in _UNARY_OPS:
                return ('o', op, [self.expr()])
            return ('o', op, [self.expr(), self.expr()])
        raise ValueError(f"unexpected expression token {tok!r}")


class _BinStream:
    def __init__(self, data: bytes, pos: int):
        self.d = data
        self.pos = pos

    def _take(self, fmt):
        v = struct.unpack_from(fmt, self.d, self.pos)
        self.pos += struct.calcsize(fmt)
        return v[0]

    def ch(self) -> str:
        c = chr(self.d[self.pos])
        self.pos += 1
        return c

    def i(self) -> int:
        return self._take('<i')

    def f(self) -> float:
        return self._take('<d')

    def expr(self):
        k = self.ch()
        if k == 'n':
            return ('n', self.f())
        if k == 'l':
            return ('n', float(self._take('<i')))
        if k == 's':
            return ('n', float(self._take('<h')))
        if k == 'v':
            return ('v', self.i())
        if k == 'h':
            ln = self.i()
            s = self.d[self.pos:self.pos + ln].decode()
            self.pos += ln
            return ('h', s)
        if k == 'f':
            fi = self.i()
            na = self.i()
            return ('f', fi, [self.expr() for _ in range(na)])
        if k == 'o':
            op = self.i()
            if op in _NARY_OPS:
                cnt = self.i()
                return ('o', op, [self.expr() for _ in range(cnt)])
            if op in (35, 65):
                return ('o', op, [self.expr() for _ in range(3)])
            if op in _UNARY_OPS:
                return ('o', op, [self.expr()])
            return ('o', op, [self.expr(), self.expr()])
        raise ValueError(f"unexpected binary expression token {k!r} at {self.pos}")


def _bound(code: int, vals):
    if code == 0:
        return vals[0], vals[1]
    if code == 1:
        return -math.inf, vals[0]
    if code == 2:
        return vals[0], math.inf
    if code == 3:
        return -math.inf, math.inf
    if code == 4:
        return vals[0], vals[0]
    raise ValueError(f"unsupported bound code {code}")


def _var_types(n, hdr):
    """AMPL variable ordering -> per-variable type (reference numerics)."""
    nlvc, nlvo, nlvb = hdr['nlvc'], hdr['nlvo'], hdr['nlvb']
    nbv, niv = hdr['nbv'], hdr['niv']
    nlvbi, nlvci, nlvoi = hdr['nlvbi'], hdr['nlvci'], hdr['nlvoi']
    t = np.full(n, CONTINUOUS, dtype=np.int32)
    # nonlinear in both: [0, nlvb) with the last nlvbi integer
    t[nlvb - nlvbi:nlvb] = INTEGER
    # nonlinear in constraints only: [nlvb, nlvc) with last nlvci integer
    t[nlvc - nlvci:nlvc] = INTEGER
    # nonlinear in objective only: [nlvc, max(nlvc,nlvo)) last nlvoi integer
    nlv = max(nlvc, nlvo)
    t[nlv - nlvoi:nlv] = INTEGER
    # linear variables: continuous, then nbv binary, then niv integer
    t[n - nbv - niv:n - niv] = BINARY
    t[n - niv:n] = INTEGER
    return t


def _header(lines):
    v = [list(map(int, ln.split('#')[0].split())) for ln in lines[1:10]]
    h = dict(n=v[0][0], m=v[0][1], nobj=v[0][2], nranges=v[0][3], neqns=v[0][4],
             nlc=v[1][0], nlo=v[1][1], nlvc=v[3][0], nlvo=v[3][1], nlvb=v[3][2],
             nbv=v[5][0], niv=v[5][1], nlvbi=v[5][2], nlvci=v[5][3], nlvoi=v[5][4],
             nzc=v[6][0], nzo=v[6][1])
    return h


def read_nl(path: str) -> NlModel:
    with open(path, 'rb') as fh:
        data = fh.read()
    # the 10 header lines are text in both formats
    hdr_end = 0
    for _ in range(10):
        hdr_end = data.index(b'\n', hdr_end) + 1
    header_lines = data[:hdr_end].decode().splitlines()
    kind = header_lines[0][0]
    h = _header(header_lines)
    name = header_lines[0].split('#')[-1].replace('problem', '').strip()
    n, m = h['n'], h['m']
    var_lb = np.full(n, -math.inf)
    var_ub = np.full(n, math.inf)
    con_lb = np.full(m, -math.inf)
    con_ub = np.full(m, math.inf)
    rows = [[] for _ in range(m)]
    con_nl = np.zeros(m, dtype=bool)
    model = NlModel(name=name, n=n, m=m, var_lb=var_lb, var_ub=var_ub,
                    var_type=_var_types(n, h), con_lb=con_lb, con_ub=con_ub,
                    rows=rows, con_nonlinear=con_nl)

    def is_zero_expr(e):
        return e[0] == 'n' and e[1] == 0.0

    if kind == 'g':
        s = _TextStream(data[hdr_end:].decode())
        while not s.eof():
            ln = s.line()
            if not ln:
                continue
            seg, rest = ln[0], ln[1:].split()
            if seg == 'C':
                i = int(rest[0])
                e = s.expr()
                if not is_zero_expr(e):
                    con_nl[i] = True
                    model.con_expr[i] = e
            elif seg == 'O':
                model.obj_sense = int(rest[1])
                e = s.expr()
                if e[0] == 'n':
                    model.obj_const = e[1]
                else:
                    model.obj_nonlinear = True
                    model.obj_expr = e
            elif seg in 'xd':
                for _ in range(int(rest[0])):
                    s.line()
            elif seg == 'r':
                for i in range(m):
                    p = s.line().split()
                    con_lb[i], con_ub[i] = _bound(int(p[0]), [float(x) for x in p[1:]])
            elif seg == 'b':
                for j in range(n):
                    p = s.line().split()
                    var_lb[j], var_ub[j] = _bound(int(p[0]), [float(x) for x in p[1:]])
            elif seg == 'k':
                for _ in range(int(rest[0])):
                    s.line()
            elif seg == 'J':
                i, cnt = int(rest[0]), int(rest[1])
                for _ in range(cnt):
                    p = s.line().split()
                    rows[i].append((int(p[0]), float(p[1])))
            elif seg == 'G':
                cnt = int(rest[1])
                for _ in range(cnt):
                    p = s.line().split()
                    model.obj_grad.append((int(p[0]), float(p[1])))
            elif seg == 'S':
                # suffix: "S<kind> <count> <name>" then count lines
                for _ in range(int(rest[1])):
                    s.line()
            elif seg == 'V':
                raise NotImplementedError("defined variables (V segments)")
            elif seg == 'F':
                continue
            else:
                raise ValueError(f"unknown .nl segment {ln!r}")
    elif kind == 'b':
        s = _BinStream(data, hdr_end)
        while s.pos < len(data):
            seg = s.ch()
            if seg == 'C':
                i = s.i()
                e = s.expr()
                if not is_zero_expr(e):
                    con_nl[i] = True
                    model.con_expr[i] = e
            elif seg == 'O':
                s.i()
                model.obj_sense = s.i()
                e = s.expr()
                if e[0] == 'n':
                    model.obj_const = e[1]
                else:
                    model.obj_nonlinear = True
                    model.obj_expr = e
            elif seg in 'xd':
                for _ in range(s.i()):
                    s.i(); s.f()
            elif seg in 'rb':
                cnt = m if seg == 'r' else n
                lo, hi = (con_lb, con_ub) if seg == 'r' else (var_lb, var_ub)
                for i in range(cnt):
                    code = int(s.ch())
                    if code == 0:
                        vals = [s.f(), s.f()]
                    elif code == 3:
                        vals = []
                    elif code == 5:
                        vals = [s.i(), s.i()]
                    else:
                        vals = [s.f()]
                    lo[i], hi[i] = _bound(code, vals)
            elif seg == 'k':
                for _ in range(s.i()):
                    s.i()
            elif seg == 'J':
                i, cnt = s.i(), s.i()
                for _ in range(cnt):
                    rows[i].append((s.i(), s.f()))
            elif seg == 'G':
                s.i()
                cnt = s.i()
                for _ in range(cnt):
                    model.obj_grad.append((s.i(), s.f()))
            elif seg == 'S':
                kind_s, cnt = s.i(), s.i()
                ln = s.i()
                s.pos += ln
                for _ in range(cnt):
                    s.i()
                    if kind_s & 4:
                        s.f()
                    else:
                        s.i()
            elif seg in '\n\r ':
                continue
            else:
                raise ValueError(f"unknown binary .nl segment {seg!r} at {s.pos}")
    else:
        raise ValueError(f"not an .nl file: {path}")
    # binary variables get [0,1] bounds in the file already; make sure
    for j in range(n):
        if model.var_type[j] == INTEGER and var_lb[j] > -1e-8 and var_ub[j] < 1 + 1e-8:
            model.var_type[j] = BINARY
    return model


def quadratic_form(expr, n):
    """Expand an expression tree of degree <= 2 (the ``o0`` plus, ``o1``
    minus, ``o2`` mult, ``o5`` pow with exponent 2, ``o16`` negation,
    ``o54`` sumlist, numbers and variables) into (Q, c, k) with
    f(x) = 1/2 x'Qx + c'x + k, Q symmetric.  Raises ValueError for anything
    else (the QP relaxation path takes quadratic objectives only)."""
    def poly(e):
        if e[0] == 'n':
            return {(): float(e[1])}
        if e[0] == 'v':
            return {(int(e[1]),): 1.0}
        op, args = e[1], e[2]
        if op == 54 or op == 0:
            out = {}
            for a in args:
                for k, v in poly(a).items():
                    out[k] = out.get(k, 0.0) + v
            return out
        if op == 1:
            a, b = poly(args[0]), poly(args[1])
            for k, v in b.items():
                a[k] = a.get(k, 0.0) - v
            return a
        if op == 16:
            return {k: -v for k, v in poly(args[0]).items()}
        if op == 2:
            a, b = poly(args[0]), poly(args[1])
            out = {}
            for ka, va in a.items():
                for kb, vb in b.items():
                    k = tuple(sorted(ka + kb))
                    if len(k) > 2:
                        raise ValueError('degree > 2')
                    out[k] = out.get(k, 0.0) + va * vb
            return out
        if op == 5 and args[1][0] == 'n' and float(args[1][1]) == 2.0:
            a = poly(args[0])
            return poly(('o', 2, [args[0], args[0]])) if a else {(): 0.0}
        raise ValueError(f'opcode {op} is not quadratic')

    Q = np.zeros((n, n))
    c = np.zeros(n)
    k0 = 0.0
    for key, v in poly(expr).items():
        if len(key) == 0:
            k0 += v
        elif len(key) == 1:
            c[key[0]] += v
        else:
            i, j = key
            if i == j:
                Q[i, i] += 2.0 * v
            else:
                Q[i, j] += v
                Q[j, i] += v
    return Q, c, k0


def evaluate(expr, x):
    """Value and gradient (dense, len(x)) of an ``.nl`` expression tree at x
    (forward mode).  Opcodes: o0 plus, o1 minus, o2 mult, o3 div, o5 pow,
    o16 negation, o39 sqrt, o54 sumlist, numbers and variables — the set
    tls4.nl, nvs08.nl and color_lab2_4x0.nl use.  The outer-approximation
    builders (minotaur_amd/problem.py) linearise rows with it."""
    x = np.asarray(x, dtype=np.float64)
    n = x.size

    def ev(e):
        if e[0] == 'n':
            return float(e[1]), np.zeros(n)
        if e[0] == 'v':
            g = np.zeros(n)
            g[int(e[1])] = 1.0
            return float(x[int(e[1])]), g
        if e[0] != 'o':
            raise ValueError(f'unsupported expression node {e[0]!r}')
        op, args = e[1], e[2]
        if op in (0, 54):
            v, g = 0.0, np.zeros(n)
            for a in args:
                va, ga = ev(a)
                v += va
                g = g + ga
            return v, g
        if op == 1:
            (va, ga), (vb, gb) = ev(args[0]), ev(args[1])
            return va - vb, ga - gb
        if op == 2:
            (va, ga), (vb, gb) = ev(args[0]), ev(args[1])
            return va * vb, vb * ga + va * gb
        if op == 3:
            (va, ga), (vb, gb) = ev(args[0]), ev(args[1])
            return va / vb, (ga * vb - va * gb) / (vb * vb)
        if op == 5:
            (va, ga), (vb, gb) = ev(args[0]), ev(args[1])
            if not gb.any():                        # constant exponent
                return va ** vb, vb * va ** (vb - 1.0) * ga
            v = va ** vb
            return v, v * (gb * math.log(va) + vb * ga / va)
        if op == 16:
            va, ga = ev(args[0])
            return -va, -ga
        if op == 39:
            va, ga = ev(args[0])
            s = math.sqrt(va)
            return s, ga / (2.0 * s)
        raise ValueError(f'opcode o{op} not supported by evaluate()')

    return ev(expr)


def row_value(model, i, x):
    """Value and gradient of row i's body: nonlinear part + linear (J) part."""
    x = np.asarray(x, dtype=np.float64)
    v, g = (evaluate(model.con_expr[i], x) if model.con_nonlinear[i]
            else (0.0, np.zeros(model.n)))
    for j, a in model.rows[i]:
        v += a * x[j]
        g[j] += a
    return v, g


def objective_value(model, x):
    """Value and gradient of the objective (nonlinear part + G gradient + constant)."""
    x = np.asarray(x, dtype=np.float64)
    v, g = (evaluate(model.obj_expr, x) if model.obj_nonlinear else (0.0, np.zeros(model.n)))
    for j, a in model.obj_grad:
        v += a * x[j]
        g[j] += a
    return v + model.obj_const, g
