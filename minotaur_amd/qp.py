"""Host-side data of the QP relaxation path.

``QpProblem``: min 1/2 x'Qx + c'x + k  s.t.  A x = b (equality rows),
l <= x <= u, dense Q (shared by every node), the node data being the box.
``from_nl`` builds it from an ``.nl`` model with a quadratic objective and
linear equality rows (color_lab2_4x0: 300 binaries, 61 rows, dense Q),
relaxing integrality (the QP relaxation QPDRelaxer hands to BQPD,
examples/QPDRelaxer.cpp:56-126).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import nl as nlmod


@dataclass
class QpProblem:
    name: str
    Q: np.ndarray      # [n, n] symmetric PSD
    c: np.ndarray      # [n]
    k: float
    A: np.ndarray      # [m, n] dense
    b: np.ndarray      # [m]
    l: np.ndarray      # [n] root box
    u: np.ndarray
    vtype: np.ndarray  # reference VariableType numerics

    @property
    def n(self):
        return self.Q.shape[0]

    @property
    def m(self):
        return self.A.shape[0]


def from_nl(path, name=None) -> QpProblem:
    """The QP of an ``.nl`` model with a quadratic objective and linear rows.
    Equality rows stay as they are; a ranged or one-sided row l <= a'x <= u
    becomes a'x - s = 0 with a slack column s in [l, u] (continuous, no
    objective term, appended after the model's columns in row order): BQPD
    takes the same model, general constraints carrying bounds bl / bu next
    to the variables' (BqpdEngine::setVarBounds_ / setConsBounds_,
    src/interfaces/BqpdEngine.cpp:601-641).  Infinite bounds stay infinite
    (presolve_box makes a node box finite for K5)."""
    m = nlmod.read_nl(path)
    Q, c, k = nlmod.quadratic_form(m.obj_expr, m.n)
    for j, a in m.obj_grad:
        c[j] += a
    k += m.obj_const
    if m.obj_sense == 1:
        Q, c, k = -Q, -c, -k
    ranged = [i for i in range(m.m) if m.con_lb[i] != m.con_ub[i]]
    n = m.n + len(ranged)
    A = np.zeros((m.m, n))
    for i, row in enumerate(m.rows):
        for j, a in row:
            A[i, j] += a
    b = m.con_lb.astype(np.float64).copy()
    l = np.concatenate([m.var_lb.astype(np.float64), np.zeros(len(ranged))])
    u = np.concatenate([m.var_ub.astype(np.float64), np.zeros(len(ranged))])
    for t, i in enumerate(ranged):
        A[i, m.n + t] = -1.0
        b[i] = 0.0
        l[m.n + t], u[m.n + t] = m.con_lb[i], m.con_ub[i]
    Qn = np.zeros((n, n))
    Qn[:m.n, :m.n] = Q
    cn = np.concatenate([c, np.zeros(len(ranged))])
    vtype = np.concatenate([np.asarray(m.var_type, dtype=np.int32),
                            np.full(len(ranged), 4, dtype=np.int32)])   # Continuous
    return QpProblem(name or m.name, Qn, cn, k, A, b, l, u, vtype)


def presolve_box(ctx, qp: QpProblem, lb=None, ub=None):
    """A finite node box for K5 (whose interior point needs one): the box
    (default: the root's) tightened by K1 on the QP's rows -- the batched
    tree's own presolve (LinearHandler::presolveNode, mgpu_fbbt) -- which
    derives bounds for free columns from their rows.  Raises when the rows
    prove the box infeasible or a bound stays infinite.  Loads the rows
    problem into ``ctx``."""
    ctx.load(rows_problem(qp))
    LB = np.atleast_2d(qp.l if lb is None else lb).astype(np.float64)
    UB = np.atleast_2d(qp.u if ub is None else ub).astype(np.float64)
    r = ctx.fbbt(LB, UB)
    if np.any(r.infeasible):
        raise ValueError(f'{qp.name}: the rows prove the box infeasible')
    if not (np.all(np.isfinite(r.lb)) and np.all(np.isfinite(r.ub))):
        raise ValueError(f'{qp.name}: FBBT leaves an infinite bound; K5 needs a finite box')
    return r.lb, r.ub


def feasible_binary_point(qp: QpProblem, seed: int):
    """A 0/1 point with A x = b for assignment-type rows (every row a
    sum of binaries = 1 with disjoint supports, plus coupling rows): greedy
    with random order, returns None if the greedy pick fails."""
    rng = np.random.default_rng(seed)
    x = np.zeros(qp.n)
    # rows  sum a_j x_j = 0  with all a_j > 0 force their binaries to 0
    zero = np.zeros(qp.n, dtype=bool)
    for i in range(qp.m):
        nz = np.nonzero(qp.A[i])[0]
        if qp.b[i] == 0.0 and np.all(qp.A[i, nz] > 0):
            zero[nz] = True
    for i in rng.permutation(qp.m):
        r = qp.A[i]
        need = qp.b[i] - r @ x
        if abs(need) < 1e-12:
            continue
        cand = [j for j in np.nonzero(r)[0]
                if x[j] == 0.0 and not zero[j] and abs(r[j] - need) < 1e-12]
        if not cand:
            return None
        x[rng.choice(cand)] = 1.0
    return x if np.allclose(qp.A @ x, qp.b) else None


def random_node_boxes(qp: QpProblem, B: int, seed: int, max_fix: int = 40):
    """Node boxes that fix a random subset of binaries to the values of a
    feasible 0/1 point (so every node QP is feasible); the rest keep the
    root box."""
    rng = np.random.default_rng(seed)
    LB = np.tile(qp.l, (B, 1))
    UB = np.tile(qp.u, (B, 1))
    for b in range(B):
        x = None
        s = int(rng.integers(0, 1 << 30))
        for _ in range(1000):
            x = feasible_binary_point(qp, s)
            s += 1
            if x is not None:
                break
        if x is None:
            raise ValueError('no feasible 0/1 point found for the node boxes')
        k = int(rng.integers(0, max_fix + 1))
        js = rng.choice(qp.n, size=k, replace=False)
        LB[b, js] = x[js]
        UB[b, js] = x[js]
    return LB, UB


def save(qp: QpProblem, path):
    np.savez_compressed(path, name=qp.name, Q=qp.Q, c=qp.c, k=qp.k, A=qp.A, b=qp.b, l=qp.l,
                        u=qp.u, vtype=qp.vtype)


def load(path) -> QpProblem:
    z = np.load(path, allow_pickle=False)
    return QpProblem(str(z['name']), z['Q'], z['c'], float(z['k']), z['A'], z['b'], z['l'],
                     z['u'], z['vtype'])


def rows_problem(qp: QpProblem):
    """The QP's equality rows as a LinProblem: what the batched tree's K1
    (LinearHandler::presolveNode on the linear rows) and node decision
    (IntVarHandler column types) read when the node relaxation is the QP
    (mgpu_bnb_relaxation 1).  No linear objective: LinearHandler does not
    propagate a quadratic objective."""
    from .problem import LinProblem
    rows, cols, vals = np.nonzero(qp.A)[0], np.nonzero(qp.A)[1], qp.A[np.nonzero(qp.A)]
    rowptr = np.zeros(qp.m + 1, dtype=np.int32)
    np.add.at(rowptr, rows + 1, 1)
    rowptr = np.cumsum(rowptr).astype(np.int32)
    return LinProblem(f'{qp.name}-rows', qp.n, qp.m, rowptr, cols.astype(np.int32),
                      vals.astype(np.float64), qp.b.astype(np.float64), qp.b.astype(np.float64),
                      qp.l.astype(np.float64), qp.u.astype(np.float64),
                      qp.vtype.astype(np.int32), np.zeros(qp.n), 0.0)


def solve_tree(ctx, qp: QpProblem, batch=1024, capacity=None, max_rounds=10**9, order=0,
               incumbent=float('inf')):
    """Branch-and-bound over QP relaxations (the batched tree with K5 as its
    node relaxation, mgpu_bnb_relaxation 1): returns (incumbent, x, stats,
    seconds).  QPDRelaxer (examples/QPDRelaxer.cpp:56-126) hands each node's
    QP to BqpdEngine; here a round's nodes go to K5 in one batch."""
    from . import bnb
    ctx.load(rows_problem(qp))
    ctx.load_qp(qp)
    ctx.bnb_relaxation(1)
    try:
        return bnb.solve(ctx, batch=batch, capacity=capacity, max_rounds=max_rounds,
                         incumbent=incumbent, order=order, warm=0)
    finally:
        ctx.bnb_relaxation(0)


def random_miqp(seed: int, nbin: int = 8, ncont: int = 4, m: int = 2) -> QpProblem:
    """A small convex MIQP whose optimum brute force over the binaries can
    check: binaries x, continuous y in [0, 2], rows sum_j a_ij x_j +
    sum_k c_ik y_k = b_i (some binary assignments infeasible), Q = G G'/n +
    0.01 I."""
    rng = np.random.default_rng(seed)
    n = nbin + ncont
    G = rng.normal(size=(n, n))
    Q = G @ G.T / n + 0.01 * np.eye(n)
    c = rng.normal(size=n)
    A = np.zeros((m, n))
    A[:, :nbin] = rng.uniform(0.5, 1.5, size=(m, nbin)) * (rng.random((m, nbin)) < 0.6)
    A[:, nbin:] = rng.uniform(0.5, 1.5, size=(m, ncont))
    b = A[:, :nbin].sum(axis=1) * 0.4 + A[:, nbin:].sum(axis=1) * 0.7
    l = np.zeros(n)
    u = np.concatenate([np.ones(nbin), np.full(ncont, 2.0)])
    vtype = np.array([0] * nbin + [4] * ncont, dtype=np.int32)   # Binary, Continuous
    return QpProblem(f'miqp{seed}', Q, c, 0.0, A, b, l, u, vtype)
