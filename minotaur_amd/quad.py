"""Host-side data for the quadratic node FBBT (K2).

``QuadProblem`` is the flat form of what Minotaur's ``QuadHandler`` sees in
``mglob``:

* the transformed problem ``p_``: variables ``0..nv0-1`` are the original
  problem's, ``nv0..nv-1`` the auxiliaries that ``SimpleTransformer`` creates
  for every distinct product (``newBilVar_``, SimpleTransformer.cpp:178-215;
  squares and bilinears alike, ``-y + x0*x1 = 0``);
* the handler's registries: squares ``y = x^2`` in ascending ``x`` (the
  ``LinSqrMap``, QuadHandler.h:54) and bilinears ``y = x0*x1`` in ascending
  ``(x0, x1)`` with ``x0 < x1`` (``CompareLinBil``, LinBil.cpp:51-62);
* the ORIGINAL problem's quadratic constraints and objective, read by
  ``tightenQuad_`` (QuadHandler.cpp:2683-2924): per function a linear term
  list (ascending variable) and a quadratic term list (ascending ``(v1, v2)``,
  ``v1 <= v2``; CompareVariablePair, Types.cpp:56-66).  Function ``ncon`` is
  the objective when ``has_obj``.

Relaxation row state (one secant per square, four McCormick rows per
bilinear, all ``<= rhs``; QuadHandler::relax_, QuadHandler.cpp:1549-1592):
``[a_x, rhs]`` per square (row ``y + a_x x <= rhs``) then ``[a0, a1, rhs] x 4``
per bilinear (rows ``-y + ..`` for types 0/1, ``+y + ..`` for types 2/3).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .problem import BINARY, CONTINUOUS, INTEGER

LF_TOL = 1e-9   # LinearFunction.cpp:22 / :89-95 — smaller weights are not stored
QF_TOL = 1e-8   # QuadraticFunction.cpp:36 / :520-528


@dataclass
class QuadProblem:
    name: str
    nv0: int
    vtype: np.ndarray      # int32 [nv]
    vlb: np.ndarray        # f64 [nv] root box (aux y's included)
    vub: np.ndarray
    sq_x: np.ndarray       # int32 [nsq] ascending
    sq_y: np.ndarray
    bil_x0: np.ndarray     # int32 [nbil] ascending (x0, x1), x0 < x1
    bil_x1: np.ndarray
    bil_y: np.ndarray
    lptr: np.ndarray       # int32 [nfun+1]  (nfun = ncon + has_obj)
    lvar: np.ndarray
    lval: np.ndarray
    qptr: np.ndarray
    qv1: np.ndarray
    qv2: np.ndarray
    qval: np.ndarray
    clb: np.ndarray        # f64 [ncon]
    cub: np.ndarray
    has_obj: bool = False
    obj_const: float = 0.0
    _keep: list = field(default_factory=list, repr=False)

    @property
    def nv(self) -> int:
        return int(self.vtype.size)

    @property
    def nsq(self) -> int:
        return int(self.sq_x.size)

    @property
    def nbil(self) -> int:
        return int(self.bil_x0.size)

    @property
    def ncon(self) -> int:
        return int(self.clb.size)

    @property
    def nrow_state(self) -> int:
        return 2 * self.nsq + 12 * self.nbil

    def save(self, path):
        np.savez(path, **{k: getattr(self, k) for k in _ARRAYS},
                 nv0=self.nv0, has_obj=int(self.has_obj), obj_const=self.obj_const,
                 name=self.name)

    @staticmethod
    def load(path) -> 'QuadProblem':
        z = np.load(path, allow_pickle=False)
        kw = {k: z[k] for k in _ARRAYS}
        return QuadProblem(name=str(z['name']), nv0=int(z['nv0']), has_obj=bool(z['has_obj']),
                           obj_const=float(z['obj_const']), **kw)


_ARRAYS = ('vtype', 'vlb', 'vub', 'sq_x', 'sq_y', 'bil_x0', 'bil_x1', 'bil_y', 'lptr',
           'lvar', 'lval', 'qptr', 'qv1', 'qv2', 'qval', 'clb', 'cub')


def _bounds_on_product(l0, u0, l1, u1):
    """Root-box product bounds (Operations.cpp:122-177, finite boxes)."""
    c = [l0 * l1, l0 * u1, u0 * l1, u0 * u1]
    return min(c), max(c)


def from_functions(name, vtype, vlb, vub, funcs, clb, cub, obj=None, obj_const=0.0,
                   aux_bounds='product'):
    """Builds a QuadProblem from original functions.

    ``funcs[c] = (lin, quad)`` with ``lin = {var: coef}`` and
    ``quad = {(v1, v2): coef}``; ``obj`` the same for the objective (or None).
    Aux variables are created (continuous) for every distinct product, squares
    first then bilinears, each in registry order.  ``aux_bounds``: 'product'
    gives y the product bounds of the root box (what QuadHandler presolve
    propagation would set), 'free' leaves y in (-inf, inf)."""
    nv0 = len(vtype)
    allf = list(funcs) + ([obj] if obj is not None else [])
    pairs = set()
    for lin, quad in allf:
        for (a, b) in quad:
            pairs.add((min(a, b), max(a, b)))
    sq = sorted(a for (a, b) in pairs if a == b)
    bil = sorted((a, b) for (a, b) in pairs if a != b)
    vt = list(vtype)
    lb = list(map(float, vlb))
    ub = list(map(float, vub))
    sq_y, bil_y = [], []
    for x in sq:
        sq_y.append(len(vt))
        vt.append(CONTINUOUS)
        if aux_bounds == 'product':
            l, u = vlb[x], vub[x]
            lo = 0.0 if l <= 0.0 <= u else min(l * l, u * u)
            lb.append(lo)
            ub.append(max(l * l, u * u))
        else:
            lb.append(-np.inf)
            ub.append(np.inf)
    for (a, b) in bil:
        bil_y.append(len(vt))
        vt.append(CONTINUOUS)
        if aux_bounds == 'product':
            lo, hi = _bounds_on_product(vlb[a], vub[a], vlb[b], vub[b])
            lb.append(lo)
            ub.append(hi)
        else:
            lb.append(-np.inf)
            ub.append(np.inf)
    lptr, lvar, lval, qptr, qv1, qv2, qval = [0], [], [], [0], [], [], []
    for lin, quad in allf:
        for v in sorted(lin):
            if abs(lin[v]) > LF_TOL:
                lvar.append(v)
                lval.append(float(lin[v]))
        lptr.append(len(lvar))
        for (a, b) in sorted((min(a, b), max(a, b)) for (a, b) in quad):
            w = quad.get((a, b), quad.get((b, a)))
            if abs(w) >= QF_TOL:
                qv1.append(a)
                qv2.append(b)
                qval.append(float(w))
        qptr.append(len(qv1))
    i32 = lambda x: np.asarray(x, dtype=np.int32)
    f64 = lambda x: np.asarray(x, dtype=np.float64)
    return QuadProblem(name=name, nv0=nv0, vtype=i32(vt), vlb=f64(lb), vub=f64(ub),
                       sq_x=i32(sq), sq_y=i32(sq_y),
                       bil_x0=i32([a for a, _ in bil]), bil_x1=i32([b for _, b in bil]),
                       bil_y=i32(bil_y), lptr=i32(lptr), lvar=i32(lvar), lval=f64(lval),
                       qptr=i32(qptr), qv1=i32(qv1), qv2=i32(qv2), qval=f64(qval),
                       clb=f64(clb), cub=f64(cub), has_obj=obj is not None,
                       obj_const=float(obj_const))


def _eval(lin, quad, x):
    return (sum(c * x[v] for v, c in lin.items()) +
            sum(c * x[a] * x[b] for (a, b), c in quad.items()))


def random_qcqp(seed: int, nv0: int = 12, ncon: int = 8, with_obj: bool = True,
                aux_bounds: str = 'product', squares: bool = True):
    """Seeded synthetic QCQP exercising every branch of QuadHandler's node
    FBBT: univariate terms a x^2 + b x (x also linear), pure squares,
    bilinears, sign-definite and sign-changing boxes, integer and binary
    variables, one- and two-sided rows, equalities, rows without a linear
    part (skipped by tightenQuad_) and purely bilinear rows (type Bilinear,
    also skipped).  squares=False turns every square x_a^2 into the product
    x_a x_(a+1) (same random stream): a bilinear-only QCQP, whose McCormick
    relaxation needs no cut loop (the glob tree's instances)."""
    rng = np.random.default_rng(seed)
    vtype, vlb, vub = [], [], []
    for j in range(nv0):
        r = rng.random()
        if r < 0.15:
            vtype.append(BINARY); vlb.append(0.0); vub.append(1.0)
        elif r < 0.3:
            vtype.append(INTEGER)
            l = float(rng.integers(-4, 2)); vlb.append(l); vub.append(l + float(rng.integers(2, 8)))
        else:
            vtype.append(CONTINUOUS)
            kind = rng.integers(0, 4)
            if kind == 0:      # straddles zero
                vlb.append(-float(rng.uniform(0.5, 8))); vub.append(float(rng.uniform(0.5, 8)))
            elif kind == 1:    # nonnegative from 0
                vlb.append(0.0); vub.append(float(rng.uniform(1, 10)))
            elif kind == 2:    # strictly positive
                l = float(rng.uniform(0.25, 3)); vlb.append(l); vub.append(l + float(rng.uniform(0.5, 6)))
            else:              # strictly negative
                u = -float(rng.uniform(0.25, 3)); vub.append(u); vlb.append(u - float(rng.uniform(0.5, 6)))
    xs = np.array([rng.uniform(l, u) if t == CONTINUOUS else float(rng.integers(int(l), int(u) + 1))
                   for t, l, u in zip(vtype, vlb, vub)])
    coef = lambda: float(rng.choice([-1, 1]) * rng.uniform(0.5, 3.0))
    funcs, clb, cub = [], [], []
    for c in range(ncon):
        lin, quad = {}, {}
        style = rng.integers(0, 10)
        nq = int(rng.integers(1, 4))
        for _ in range(nq):
            a = int(rng.integers(0, nv0))
            if style == 9 or rng.random() < 0.45:
                b = int(rng.integers(0, nv0))
                if b == a:
                    b = (a + 1) % nv0
                quad[(min(a, b), max(a, b))] = coef()
            else:
                b2 = a if squares else (a + 1) % nv0
                quad[(min(a, b2), max(a, b2))] = coef()
                if rng.random() < 0.6 and style != 8:
                    lin[a] = coef()
        if style != 8:
            for _ in range(int(rng.integers(1, 4))):
                lin[int(rng.integers(0, nv0))] = coef()
        val = _eval(lin, quad, xs)
        kind = rng.integers(0, 4)
        slack = float(rng.uniform(0.0, 2.0))
        if kind == 0:
            clb.append(-np.inf); cub.append(val + slack)
        elif kind == 1:
            clb.append(val - slack); cub.append(np.inf)
        elif kind == 2:
            clb.append(val - slack); cub.append(val + slack)
        else:
            clb.append(val); cub.append(val)
        funcs.append((lin, quad))
    obj = None
    if with_obj:
        lin, quad = {}, {}
        for _ in range(int(rng.integers(2, 5))):
            a = int(rng.integers(0, nv0))
            b2 = a if squares else (a + 1) % nv0
            quad[(min(a, b2), max(a, b2))] = float(rng.uniform(0.5, 2.0))
            lin[a] = coef()
        for _ in range(int(rng.integers(0, 3))):
            a, b = rng.integers(0, nv0, size=2)
            if a != b:
                quad[(int(min(a, b)), int(max(a, b)))] = coef()
        obj = (lin, quad)
    qp = from_functions(f'qcqp-{seed}', vtype, vlb, vub, funcs, clb, cub, obj=obj,
                        obj_const=float(rng.uniform(-2, 2)), aux_bounds=aux_bounds)
    # the interior point every row was built around, with y = products
    xstar = np.zeros(qp.nv)
    xstar[:nv0] = xs
    for k in range(qp.nsq):
        xstar[qp.sq_y[k]] = xs[qp.sq_x[k]] ** 2
    for k in range(qp.nbil):
        xstar[qp.bil_y[k]] = xs[qp.bil_x0[k]] * xs[qp.bil_x1[k]]
    qp.xstar = xstar
    return qp


def objective_at(qp: QuadProblem, x) -> float:
    """Original objective value at x (original variables)."""
    assert qp.has_obj
    c = qp.ncon
    v = qp.obj_const
    for k in range(qp.lptr[c], qp.lptr[c + 1]):
        v += qp.lval[k] * x[qp.lvar[k]]
    for k in range(qp.qptr[c], qp.qptr[c + 1]):
        v += qp.qval[k] * x[qp.qv1[k]] * x[qp.qv2[k]]
    return float(v)


def random_quad_boxes(qp: QuadProblem, B: int, seed: int, max_depth: int = 8,
                      edge: bool = False):
    """Seeded node boxes by random branching on the ORIGINAL variables (glob
    branches on x; the aux y's keep the root bounds).  Integers split at
    floor(mid); continuous variables at a random interior point, keeping
    either side.  ``edge`` adds the interval-arithmetic corner cases of
    Operations.cpp:122-210: x pinned to [0, 0] or to |x| < 1e-10, aux y
    bounds shrunk (so y -> x propagation bites) or made infinite."""
    rng = np.random.default_rng(seed)
    LB = np.tile(qp.vlb, (B, 1))
    UB = np.tile(qp.vub, (B, 1))
    for b in range(B):
        if edge:
            for _ in range(int(rng.integers(0, 3))):
                j = int(rng.integers(0, qp.nv0))
                if qp.vtype[j] == CONTINUOUS and LB[b, j] <= 0.0 <= UB[b, j]:
                    if rng.random() < 0.5:
                        LB[b, j] = UB[b, j] = 0.0
                    else:
                        LB[b, j], UB[b, j] = -3e-11, 4e-11
            for _ in range(int(rng.integers(0, 3))):
                if qp.nv == qp.nv0:
                    break
                j = int(rng.integers(qp.nv0, qp.nv))
                l, u = LB[b, j], UB[b, j]
                r = rng.random()
                if r < 0.2:
                    LB[b, j], UB[b, j] = -np.inf, np.inf
                elif np.isfinite(l) and np.isfinite(u):
                    t0, t1 = np.sort(rng.uniform(0.0, 1.0, size=2))
                    LB[b, j], UB[b, j] = l + (u - l) * t0, l + (u - l) * t1
        for _ in range(int(rng.integers(0, max_depth + 1))):
            j = int(rng.integers(0, qp.nv0))
            l, u = LB[b, j], UB[b, j]
            if u - l <= 1e-6:
                continue
            if qp.vtype[j] in (BINARY, INTEGER):
                if u - l < 1.0:
                    continue
                m = np.floor(0.5 * (l + u))
                if rng.random() < 0.5:
                    UB[b, j] = m
                else:
                    LB[b, j] = m + 1.0
            else:
                t = l + (u - l) * float(rng.uniform(0.1, 0.9))
                if rng.random() < 0.5:
                    UB[b, j] = t
                else:
                    LB[b, j] = t
    return LB, UB


@dataclass
class NodeRows:
    """Per-node rows of an LP relaxation (``mgpu_set_node_rows``): entry
    ``coef_pos[k]`` of the loaded CSR takes a node record's value
    ``coef_src[k]``; row ``row_idx[q]`` takes bounds ``lo_src[q]`` /
    ``hi_src[q]`` of it (-1: the loaded bound).  ``stride`` = record length."""
    stride: int
    coef_pos: np.ndarray
    coef_src: np.ndarray
    row_idx: np.ndarray
    lo_src: np.ndarray
    hi_src: np.ndarray

    def node_problem(self, p, rec):
        """The LP of one node (a copy of ``p`` with the record applied;
        |a| <= 1e-9 dropped as LinearFunction::addTerm does)."""
        import copy
        q = copy.copy(p)
        val = p.val.copy()
        v = np.asarray(rec, dtype=np.float64)[self.coef_src]
        val[self.coef_pos] = np.where(np.abs(v) <= LF_TOL, 0.0, v)
        q.val = val
        q.rlo = p.rlo.copy()
        q.rhi = p.rhi.copy()
        for r, lo, hi in zip(self.row_idx, self.lo_src, self.hi_src):
            if lo >= 0:
                q.rlo[r] = rec[lo]
            if hi >= 0:
                q.rhi[r] = rec[hi]
        return q


def tangent_record(qp: QuadProblem, slots: int) -> np.ndarray:
    """The tangent part of a node record with every slot inactive: per square
    k and slot s the pair [2 xl, xl^2] of the cut 2 xl x - y <= xl^2
    (QuadHandler::addTangent_, QuadHandler.cpp:805-817); inactive = [0, +inf],
    the row 0 x - y <= +inf."""
    rec = np.zeros(2 * qp.nsq * slots)
    rec[1::2] = np.inf
    return rec


def relaxation_lp(qp: QuadProblem, rows=None, tan_slots: int = 0):
    """The LP relaxation of ``p_`` that mglob's engine solves at a node
    (QuadHandler::relax_, QuadHandler.cpp:1549-1592, plus the linear rows):

    * rows 0..ncon-1: the original constraints with every product replaced by
      its auxiliary (SimpleTransformer), bounds clb/cub;
    * one secant row per square, ``y + a_x x <= rhs`` (upSqCon_ rewrites a_x
      and rhs), then four McCormick rows per bilinear, ``-y + a0 x0 + a1 x1
      <= rhs`` (types 0, 1) and ``y + a0 x0 + a1 x1 <= rhs`` (types 2, 3)
      (upBilCon_ rewrites a0, a1, rhs);
    * ``tan_slots`` > 0: per square, that many tangent-cut rows
      ``2 xl x - y <= xl^2`` (QuadHandler::separate's cuts, addTangent_,
      QuadHandler.cpp:805-817), coefficient and bound from the node record
      after the row state (``tangent_record``: inactive slots are 0 x - y <=
      +inf); the record stride becomes R + 2 nsq tan_slots;
    * objective: the original objective with products replaced (0 if none).

    ``rows``: the row state at the root (``Context.quad_rows()`` layout,
    ``QuadProblem.nrow_state`` values).  Returns ``(LinProblem, NodeRows)``;
    the NodeRows map reads a node's K2 row state (``rows_out``) directly.
    The rewritten entries are always in the pattern (value 0 when dropped)."""
    from .problem import LinProblem
    nsq, nbil = qp.nsq, qp.nbil
    rows = np.zeros(qp.nrow_state) if rows is None else np.asarray(rows, dtype=np.float64)
    aux = {}
    for k in range(nsq):
        aux[(int(qp.sq_x[k]), int(qp.sq_x[k]))] = int(qp.sq_y[k])
    for k in range(nbil):
        aux[(int(qp.bil_x0[k]), int(qp.bil_x1[k]))] = int(qp.bil_y[k])

    def linearize(f):
        d = {}
        for t in range(qp.lptr[f], qp.lptr[f + 1]):
            d[int(qp.lvar[t])] = d.get(int(qp.lvar[t]), 0.0) + float(qp.lval[t])
        for t in range(qp.qptr[f], qp.qptr[f + 1]):
            y = aux[(int(qp.qv1[t]), int(qp.qv2[t]))]
            d[y] = d.get(y, 0.0) + float(qp.qval[t])
        return [(j, d[j]) for j in sorted(d) if abs(d[j]) > LF_TOL]

    rowptr, colidx, val, rlo, rhi = [0], [], [], [], []
    coef_pos, coef_src, row_idx, hi_src = [], [], [], []

    def add_row(terms, lo, hi, varying=()):
        # terms ascending by column; varying: {col: record offset}
        for j, a in terms:
            if j in varying:
                coef_pos.append(len(colidx))
                coef_src.append(varying[j])
            colidx.append(j)
            val.append(a)
        rowptr.append(len(colidx))
        rlo.append(lo)
        rhi.append(hi)

    for c in range(qp.ncon):
        add_row(linearize(c), float(qp.clb[c]), float(qp.cub[c]))
    for k in range(nsq):
        x, y = int(qp.sq_x[k]), int(qp.sq_y[k])
        row_idx.append(len(rlo))
        hi_src.append(2 * k + 1)
        add_row([(x, rows[2 * k]), (y, 1.0)], -np.inf, rows[2 * k + 1], {x: 2 * k})
    for k in range(nbil):
        x0, x1, y = int(qp.bil_x0[k]), int(qp.bil_x1[k]), int(qp.bil_y[k])
        for t in range(4):
            o = 2 * nsq + 12 * k + 3 * t
            row_idx.append(len(rlo))
            hi_src.append(o + 2)
            add_row([(x0, rows[o]), (x1, rows[o + 1]), (y, -1.0 if t < 2 else 1.0)],
                    -np.inf, rows[o + 2], {x0: o, x1: o + 1})
    R = qp.nrow_state
    for k in range(nsq):
        x, y = int(qp.sq_x[k]), int(qp.sq_y[k])
        for t in range(tan_slots):
            o = R + 2 * (k * tan_slots + t)
            row_idx.append(len(rlo))
            hi_src.append(o + 1)
            terms = sorted([(x, 0.0), (y, -1.0)])
            add_row(terms, -np.inf, np.inf, {x: o})
    obj = np.zeros(qp.nv)
    if qp.has_obj:
        for j, a in linearize(qp.ncon):
            obj[j] = a
    i32 = lambda a: np.asarray(a, dtype=np.int32)
    p = LinProblem(name=f'{qp.name}-relax', n=qp.nv, m=len(rlo), rowptr=i32(rowptr),
                   colidx=i32(colidx), val=np.asarray(val, dtype=np.float64),
                   rlo=np.asarray(rlo, dtype=np.float64), rhi=np.asarray(rhi, dtype=np.float64),
                   vlb=qp.vlb.copy(), vub=qp.vub.copy(), vtype=qp.vtype.copy(), obj=obj,
                   obj_const=float(qp.obj_const) if qp.has_obj else 0.0).validate()
    nr = NodeRows(stride=R + 2 * nsq * tan_slots, coef_pos=i32(coef_pos), coef_src=i32(coef_src),
                  row_idx=i32(row_idx), lo_src=i32([-1] * len(row_idx)), hi_src=i32(hi_src))
    return p, nr
