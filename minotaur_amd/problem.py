"""Host-side problem data for the batched relaxation path.

``LinProblem`` is the flat form of a Minotaur ``Relaxation`` with linear rows
that the engine loads once per batch (``OsiLPEngine::load``,
src/interfaces/OsiLPEngine.cpp:390-498, builds the same row-major CSR):

* rows in constraint-index order, terms inside a row in ascending column
  order (the reference's ``VariableGroup`` is a ``std::map`` ordered by
  variable id, src/base/Types.h:496 + Types.cpp:30-34, and ids follow
  creation order = column index, Problem.cpp:1854-1856);
* column bounds / types (reference ``VariableType`` numerics, Types.h:83-89);
* a linear objective (dense ``obj``) plus constant, minimisation.

Node boxes (``lb``/``ub`` per node) are the per-node data; everything here is
shared across the batch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

BINARY, INTEGER, CONTINUOUS = 0, 1, 4


@dataclass
class LinProblem:
    name: str
    n: int
    m: int
    rowptr: np.ndarray   # int32 [m+1]
    colidx: np.ndarray   # int32 [nnz]
    val: np.ndarray      # f64 [nnz]
    rlo: np.ndarray      # f64 [m]
    rhi: np.ndarray      # f64 [m]
    vlb: np.ndarray      # f64 [n] root box
    vub: np.ndarray      # f64 [n]
    vtype: np.ndarray    # int32 [n]
    obj: np.ndarray      # f64 [n] dense linear objective (minimise)
    obj_const: float = 0.0

    # ------------------------------------------------------------------
    @property
    def nnz(self) -> int:
        return int(self.rowptr[-1])

    def csc_pattern(self):
        """Column -> rows pattern (rows ascending) used by ``changeBFlag_``
        (LinearHandler.cpp:1229-1234 marks every row holding the column)."""
        counts = np.bincount(self.colidx, minlength=self.n)
        colptr = np.zeros(self.n + 1, dtype=np.int32)
        np.cumsum(counts, out=colptr[1:])
        rowidx = np.empty(self.nnz, dtype=np.int32)
        fill = colptr[:-1].copy()
        for i in range(self.m):
            for k in range(self.rowptr[i], self.rowptr[i + 1]):
                j = self.colidx[k]
                rowidx[fill[j]] = i
                fill[j] += 1
        return colptr, rowidx

    def obj_sparse(self):
        idx = np.nonzero(self.obj)[0].astype(np.int32)
        return idx, self.obj[idx].astype(np.float64)

    def cons_bad(self) -> int:
        """``checkBounds_`` second loop (LinearHandler.cpp:350-357)."""
        return int(np.any(self.rlo > self.rhi + 1e-8))

    def dense(self) -> np.ndarray:
        A = np.zeros((self.m, self.n))
        for i in range(self.m):
            s, e = self.rowptr[i], self.rowptr[i + 1]
            A[i, self.colidx[s:e]] = self.val[s:e]
        return A

    def validate(self):
        assert self.rowptr.dtype == np.int32 and self.colidx.dtype == np.int32
        assert self.rowptr.shape == (self.m + 1,) and self.rowptr[0] == 0
        for i in range(self.m):
            c = self.colidx[self.rowptr[i]:self.rowptr[i + 1]]
            assert np.all(np.diff(c) > 0), f"row {i} not strictly ascending"
        assert np.all((self.colidx >= 0) & (self.colidx < self.n))
        for a in (self.val, self.rlo, self.rhi, self.vlb, self.vub, self.obj):
            assert a.dtype == np.float64
        return self

    # ------------------------------------------------------------------
    def save(self, path: str):
        np.savez_compressed(path, name=self.name, n=self.n, m=self.m,
                            rowptr=self.rowptr, colidx=self.colidx, val=self.val,
                            rlo=self.rlo, rhi=self.rhi, vlb=self.vlb, vub=self.vub,
                            vtype=self.vtype, obj=self.obj,
                            obj_const=self.obj_const)

    @staticmethod
    def load(path: str) -> "LinProblem":
        z = np.load(path, allow_pickle=False)
        return LinProblem(name=str(z['name']), n=int(z['n']), m=int(z['m']),
                          rowptr=z['rowptr'].astype(np.int32),
                          colidx=z['colidx'].astype(np.int32),
                          val=z['val'].astype(np.float64),
                          rlo=z['rlo'].astype(np.float64),
                          rhi=z['rhi'].astype(np.float64),
                          vlb=z['vlb'].astype(np.float64),
                          vub=z['vub'].astype(np.float64),
                          vtype=z['vtype'].astype(np.int32),
                          obj=z['obj'].astype(np.float64),
                          obj_const=float(z['obj_const'])).validate()


def from_rows(name, n, rows, rlo, rhi, vlb, vub, vtype, obj, obj_const=0.0):
    """Build a LinProblem from per-row ``[(col, coef), ...]`` lists.  Terms are
    sorted by column and |coef| <= 1e-9 dropped (``LinearFunction::addTerm``
    keeps only |a| > tol_ = 1e-9, LinearFunction.cpp:22,89-95)."""
    rowptr = [0]
    colidx, val = [], []
    for r in rows:
        d = {}
        for j, a in r:
            d[int(j)] = d.get(int(j), 0.0) + float(a)
        for j in sorted(d):
            if abs(d[j]) > 1e-9:
                colidx.append(j)
                val.append(d[j])
        rowptr.append(len(colidx))
    return LinProblem(name=name, n=int(n), m=len(rows),
                      rowptr=np.asarray(rowptr, dtype=np.int32),
                      colidx=np.asarray(colidx, dtype=np.int32),
                      val=np.asarray(val, dtype=np.float64),
                      rlo=np.asarray(rlo, dtype=np.float64),
                      rhi=np.asarray(rhi, dtype=np.float64),
                      vlb=np.asarray(vlb, dtype=np.float64),
                      vub=np.asarray(vub, dtype=np.float64),
                      vtype=np.asarray(vtype, dtype=np.int32),
                      obj=np.asarray(obj, dtype=np.float64),
                      obj_const=float(obj_const)).validate()


def from_nl_linear(model, name=None) -> LinProblem:
    """Linear part of an ``.nl`` model: every row without a nonlinear
    expression ("tls4-lin" for tls4.nl)."""
    keep = model.linear_rows()
    obj = np.zeros(model.n)
    for j, a in model.obj_grad:
        obj[j] += a
    if model.obj_sense == 1:
        obj = -obj
    return from_rows(name or (model.name + "-lin"), model.n,
                     [model.rows[i] for i in keep],
                     model.con_lb[keep], model.con_ub[keep],
                     model.var_lb, model.var_ub, model.var_type, obj,
                     model.obj_const)


def knapsack_oa(f=9, N=64, a=None, b=None, points=(1.0, 8.0, 32.0, 64.0)):
    """Outer-approximation LP of the knapsack example
    (examples/knapsack/knapsack.cpp:68-114, data main.f:12-32):
    min sum a_i x_i^{b_i}, sum x_i <= N, x_i integer in [1, N].
    Columns: x_1..x_f (Integer), eta_1..eta_f (Continuous); rows: the
    capacity row, then for each term one tangent row per point t:
    eta_i - f_i'(t) x_i >= f_i(t) - f_i'(t) t  (the terms are convex for
    a > 0, b < 0, x > 0, so tangents under-estimate)."""
    if a is None:
        a = [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0, 9.0][:f]
    if b is None:
        b = [-1.0, -2.0, -1.5, -1.7, -1.2, -1.7, -1.4, -1.2, -1.5][:f]
    if len(a) < f:
        rng = np.random.default_rng(1234 + f)
        a = list(a) + list(rng.uniform(1.0, 9.0, f - len(a)))
        b = list(b) + list(rng.uniform(-2.0, -1.0, f - len(b)))
    n = 2 * f
    rows, rlo, rhi = [], [], []
    rows.append([(i, 1.0) for i in range(f)])
    rlo.append(-math.inf)
    rhi.append(float(N))
    for i in range(f):
        for t in points:
            if t > N:
                continue
            fv = a[i] * t ** b[i]
            g = a[i] * b[i] * t ** (b[i] - 1.0)
            rows.append([(i, -g), (f + i, 1.0)])
            rlo.append(fv - g * t)
            rhi.append(math.inf)
    vlb = [1.0] * f + [-math.inf] * f
    vub = [float(N)] * f + [math.inf] * f
    vtype = [INTEGER] * f + [CONTINUOUS] * f
    obj = [0.0] * f + [1.0] * f
    return from_rows(f"knapsack-oa-f{f}-N{N}", n, rows, rlo, rhi, vlb, vub,
                     vtype, obj)


def random_boxes(p: LinProblem, B: int, seed: int, max_depth: int = 20,
                 root_lb=None, root_ub=None):
    """Seeded node boxes by random branching from the root:
    each node gets a depth d in [1, max_depth]; each of the d steps picks a
    random integer column that is not fixed yet and either fixes a binary to
    0/1 or splits an integer (down: ub=floor(mid), up: lb=floor(mid)+1).
    Vectorised over nodes; the column is drawn uniformly among the node's
    free integer columns by rejection (round 4: 4 M boxes in seconds instead
    of minutes; earlier rounds drew it by an arg-min over random keys, the
    same distribution, other boxes).  Returns (lb[B,n], ub[B,n])."""
    rng = np.random.default_rng(seed)
    lb0 = p.vlb if root_lb is None else root_lb
    ub0 = p.vub if root_ub is None else root_ub
    ints = np.nonzero((p.vtype == BINARY) | (p.vtype == INTEGER))[0]
    LB = np.tile(np.asarray(lb0, dtype=np.float64), (B, 1))
    UB = np.tile(np.asarray(ub0, dtype=np.float64), (B, 1))
    if ints.size == 0 or B == 0:
        return LB, UB
    depth = rng.integers(1, max_depth + 1, size=B)
    rows = np.arange(B)
    nint = ints.size

    def is_free(r, c):
        jj = ints[c]
        return (UB[r, jj] - LB[r, jj]) >= 1.0

    for step in range(max_depth):
        # a uniformly random free integer column per node, by rejection from
        # uniform proposals (8 rounds; a node still without one -- most of
        # its columns fixed -- takes the exact draw over its free columns)
        pick = rng.integers(0, nint, size=B)
        ok = is_free(rows, pick)
        for _ in range(8):
            miss = np.nonzero(~ok)[0]
            if miss.size == 0:
                break
            cand = rng.integers(0, nint, size=miss.size)
            good = is_free(miss, cand)
            pick[miss[good]] = cand[good]
            ok[miss[good]] = True
        miss = np.nonzero(~ok)[0]
        if miss.size:
            fr = (UB[miss][:, ints] - LB[miss][:, ints]) >= 1.0
            keys = rng.random((miss.size, nint))
            keys[~fr] = 2.0
            pick[miss] = np.argmin(keys, axis=1)
            ok[miss] = fr[np.arange(miss.size), pick[miss]]
        act = (depth > step) & ok
        j = ints[pick]
        l = np.where(np.isfinite(LB[rows, j]), LB[rows, j], -1e3)
        h = np.where(np.isfinite(UB[rows, j]), UB[rows, j], 1e3)
        split = np.floor(0.5 * (l + h))
        down = rng.integers(0, 2, size=B) == 0
        sel = act & down
        UB[rows[sel], j[sel]] = split[sel]
        sel = act & ~down
        LB[rows[sel], j[sel]] = split[sel] + 1.0
    return LB, UB


def random_problem(seed: int, n: int = 40, m: int = 30, density: float = 0.15,
                   inf_frac: float = 0.15, int_frac: float = 0.5,
                   eq_frac: float = 0.1):
    """Synthetic edge-case generator: ragged rows (including empty and dense
    ones), infinite column bounds (exercising getSingLfBnds_), one-sided and
    two-sided rows, equality rows, tiny (|a|<=1e-8) and large coefficients,
    and a mix of binary / integer / continuous columns."""
    rng = np.random.default_rng(seed)
    vtype = np.full(n, CONTINUOUS, dtype=np.int32)
    r = rng.random(n)
    vtype[r < int_frac] = INTEGER
    vtype[r < int_frac * 0.5] = BINARY
    vlb = np.where(vtype == BINARY, 0.0, np.round(rng.uniform(-20, 5, n)))
    vub = np.where(vtype == BINARY, 1.0, vlb + np.round(rng.uniform(1, 40, n)))
    cont = vtype == CONTINUOUS
    vlb = np.where(cont, rng.uniform(-20, 5, n), vlb)
    vub = np.where(cont, vlb + rng.uniform(0.5, 40, n), vub)
    infl = (rng.random(n) < inf_frac) & (vtype != BINARY)
    infu = (rng.random(n) < inf_frac) & (vtype != BINARY)
    vlb[infl] = -math.inf
    vub[infu] = math.inf
    rows, rlo, rhi = [], [], []
    # one interior point shared by all rows, so the root box is feasible
    x = np.where(np.isfinite(vlb) & np.isfinite(vub),
                 rng.uniform(0, 1, n) * (np.where(np.isfinite(vub), vub, 0) -
                                         np.where(np.isfinite(vlb), vlb, 0)) +
                 np.where(np.isfinite(vlb), vlb, 0),
                 np.where(np.isfinite(vlb), vlb, np.where(np.isfinite(vub), vub, 0.0)))
    for i in range(m):
        if i == 0:
            k = 0
        elif i == 1:
            k = n
        else:
            k = max(1, rng.binomial(n, density))
        cols = rng.choice(n, size=k, replace=False) if k else []
        terms = []
        for j in cols:
            u = rng.random()
            if u < 0.03:
                c = float(rng.choice([-1, 1]) * 5e-9)  # ignored by updates
            elif u < 0.08:
                c = float(rng.choice([-1, 1]) * rng.uniform(50, 500))
            else:
                c = float(np.round(rng.uniform(-5, 5), 3)) or 1.0
            terms.append((int(j), c))
        rows.append(terms)
        act = sum(c * x[j] for j, c in terms)
        kind = rng.random()
        slack = float(rng.uniform(0, 10))
        if kind < eq_frac:
            rlo.append(act)
            rhi.append(act)
        elif kind < 0.45:
            rlo.append(-math.inf)
            rhi.append(act + slack)
        elif kind < 0.8:
            rlo.append(act - slack)
            rhi.append(math.inf)
        else:
            rlo.append(act - slack)
            rhi.append(act + slack)
    obj = np.round(rng.uniform(-3, 3, n), 2)
    obj[rng.random(n) < 0.3] = 0.0
    return from_rows(f"random-{seed}", n, rows, rlo, rhi, vlb, vub, vtype, obj,
                     obj_const=float(np.round(rng.uniform(-5, 5), 2)))


def random_mkp(seed: int, n: int = 40, m: int = 5, tight: float = 0.5):
    """Seeded multi-dimensional 0-1 knapsack (a classic weak-LP-bound MILP,
    for tree-search throughput): max c'x s.t. A x <= tight * A 1, x binary,
    written as min -c'x.  A, c integer in [1, 100] (c correlated with A)."""
    rng = np.random.default_rng(seed)
    A = rng.integers(1, 101, size=(m, n)).astype(np.float64)
    c = np.floor(A.mean(axis=0) + rng.integers(0, 21, size=n)).astype(np.float64)
    b = np.floor(tight * A.sum(axis=1))
    rows = [[(j, A[i, j]) for j in range(n)] for i in range(m)]
    return from_rows(f"mkp-{seed}-n{n}-m{m}", n, rows, np.full(m, -np.inf), b,
                     np.zeros(n), np.ones(n), np.full(n, BINARY, dtype=np.int32), -c)


def tls4_oa(model, ntan=1, seed=2, ratio_lo=0.5, ratio_hi=20.0):
    """Outer-approximation LP of test_instances/tls4.nl (BASELINE config 2,
    the MINLP itself rather than its linear rows only).

    tls4 has four nonlinear rows (tls4.nl:203-222, expression o16 o54 of four
    o39 o2 terms):

      C_i:  - sum_{k<4} sqrt(x_{4i+k} * y_k) + a_i' z <= b_i,   i = 0..3,

    with x_{4i+k} = column 4i+k (continuous, [1, inf)) and y_k = column 16+k
    (integer, [1, 100]); the linear part a_i' z is the row's own linear terms
    in the file.  -sqrt(x y) is convex on the positive orthant (sqrt(x y) is
    the geometric mean, concave), so every tangent plane under-estimates it
    and g(p) + grad g(p)'(x - p) <= b_i is a valid cut.  -sqrt(x y) is
    positively homogeneous of degree 1, so g(p) = grad g(p)'p (Euler) and the
    tangent at a point with ratio r = x/y is simply

      -1/2 (x / sqrt(r) + y sqrt(r)) + a_i' z <= b_i,

    exact on the ray x = r y.  Each nonlinear row becomes ``ntan`` tangent
    rows, each with its own seeded ratio per term (log-uniform in
    [ratio_lo, ratio_hi]); they take the place of C_i (rows 0..4*ntan-1), and
    the 60 linear rows follow in file order.  With ntan = 1 the LP keeps
    tls4's 64 rows (the K3P / K3 row range).

    The OA-MILP optimum is a lower bound on tls4's MINLP optimum (8.3,
    MINLPLib): 3.2 for the default seed (HiGHS, tools/make_instances.py)."""
    import math as _m
    assert model.n == 105 and model.m == 64, 'tls4 has 105 columns and 64 rows'
    rng = np.random.default_rng(seed)
    rows, rlo, rhi = [], [], []
    nl_rows = [i for i in range(model.m) if model.con_nonlinear[i]]
    assert nl_rows == [0, 1, 2, 3], nl_rows
    for i in nl_rows:
        lin = [(j, a) for j, a in model.rows[i] if a != 0.0]
        for _ in range(ntan):
            r = np.exp(rng.uniform(_m.log(ratio_lo), _m.log(ratio_hi), 4))
            extra = []
            for k in range(4):
                extra += [(4 * i + k, -0.5 / _m.sqrt(r[k])), (16 + k, -0.5 * _m.sqrt(r[k]))]
            rows.append(lin + extra)
            rlo.append(model.con_lb[i])
            rhi.append(model.con_ub[i])
    for i in model.linear_rows():
        rows.append(model.rows[i])
        rlo.append(model.con_lb[i])
        rhi.append(model.con_ub[i])
    obj = np.zeros(model.n)
    for j, a in model.obj_grad:
        obj[j] += a
    if model.obj_sense == 1:
        obj = -obj
    return from_rows('tls4-oa' if ntan == 1 else f'tls4-oa{ntan}', model.n, rows, rlo, rhi,
                     model.var_lb, model.var_ub, model.var_type, obj, model.obj_const)


def nvs08_oa(model, npts=4, nobj=8, seed=20261016):
    """Outer-approximation LP of test_instances/nvs08.nl (BASELINE config 1,
    SURVEY §0.1 / §8d: "OA-LP with tangent rows at seeded points").

    nvs08 is nonlinear in every row (nvs08.nl:2-44), so OsiLPEngine cannot
    load it (OsiLPEngine.cpp:420); the LP this engine solves for it is built
    from the model the .nl reader returns (nl.row_value / objective_value
    evaluate the file's own expression trees):

      columns  x0 (continuous, [1e-3, 200]), x1, x2 (integer, [0, 200]), eta;
      C0  sqrt(x0) + x1 + 2 x2 >= 10        concave: tangent rows at x0 = t_k
      C1  q x1^2 + a x0 - x2 >= -3          x1^2 convex: its secant over the
                                            root box [l1, u1] (over-estimates)
      C2  x2^2 - x0^-3.5 - 4 x1 >= -12      x2^2 by its secant, -x0^-3.5
                                            concave: tangent rows at x0 = t_k
      obj (x1-3)^2 + (x2-2)^2 + (x0+4)^2    convex: min eta, eta >= tangent
                                            planes at seeded points p_k

    Every row over-estimates its (>=) row body on the root box, so the LP is
    a relaxation of nvs08 and the OA-MILP optimum is a lower bound on the
    MINLP optimum (23.4497, MINLPLib; x = (0.63, 4, 3)).  The linearisation
    points sit around that region as an OA solver's NLP iterates would
    (seeded): t_k log-uniform in [0.3, 5]; p_k with x0 uniform in [0.3, 2],
    x1 integer in [2, 5], x2 integer in [1, 4]; eta >= 0 (the objective is a
    sum of squares)."""
    from .nl import objective_value, row_value
    assert model.n == 3 and model.m == 3, 'nvs08 has 3 variables and 3 rows'
    rng = np.random.default_rng(seed)
    n = 4                                          # x0, x1, x2, eta
    l1, u1 = float(model.var_lb[1]), float(model.var_ub[1])
    l2, u2 = float(model.var_lb[2]), float(model.var_ub[2])
    ts = np.exp(rng.uniform(math.log(0.3), math.log(5.0), npts))
    rows, rlo, rhi = [], [], []

    def tangent(i, p, extra=(), shift=0.0):
        v, g = row_value(model, i, p)
        terms = [(j, g[j]) for j in range(3) if g[j] != 0.0] + list(extra)
        rows.append(terms)
        rlo.append(model.con_lb[i] - v + float(np.dot(g, p)) + shift)
        rhi.append(math.inf)

    for t in ts:                                   # C0 tangents
        tangent(0, np.array([t, 0.0, 0.0]))
    # C1: the quadratic coefficient from the file's expression (value at x1 = 1)
    q = row_value(model, 1, np.array([0.0, 1.0, 0.0]))[0] - \
        row_value(model, 1, np.zeros(3))[0] - dict(model.rows[1]).get(1, 0.0)
    _, g1 = row_value(model, 1, np.zeros(3))      # the linear terms (x1^2' = 0 at 0)
    rows.append([(0, g1[0]), (1, q * (l1 + u1) + g1[1]), (2, g1[2])])
    rlo.append(model.con_lb[1] + q * l1 * u1)
    rhi.append(math.inf)
    for t in ts:                                   # C2: -x0^-3.5 tangent + x2^2 secant
        tangent(2, np.array([t, 0.0, 0.0]), extra=[(2, l2 + u2)], shift=l2 * u2)
    for _ in range(nobj):                          # objective tangent planes
        p = np.array([rng.uniform(0.3, 2.0), float(rng.integers(2, 6)),
                      float(rng.integers(1, 5))])
        f, g = objective_value(model, p)
        rows.append([(j, -g[j]) for j in range(3)] + [(3, 1.0)])
        rlo.append(f - float(np.dot(g, p)))
        rhi.append(math.inf)
    vlb = list(model.var_lb) + [0.0]            # the objective is a sum of squares
    vub = list(model.var_ub) + [math.inf]
    vtype = list(model.var_type) + [CONTINUOUS]
    obj = [0.0, 0.0, 0.0, 1.0]
    return from_rows('nvs08-oa', n, rows, rlo, rhi, vlb, vub, vtype, obj)
