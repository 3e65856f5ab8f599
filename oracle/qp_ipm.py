"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy, float64) of the batched QP relaxation solve of
minotaur_amd/csrc/qp_kkt.hip: the node QP of QPDRelaxer /
BqpdEngine (src/interfaces/BqpdEngine.cpp:449-534, examples/QPDRelaxer.cpp)

    min 1/2 x'Qx + c'x + k   s.t.  A x = b,  l <= x <= u   (node box)

solved by a Mehrotra predictor-corrector primal-dual interior point method
whose Newton systems are the KKT block [Q + D, A'; A, 0] reduced through the
Schur complement: K = Q + D = L L' (dense Cholesky, the MFMA part on the
GPU), W = L^-1 A', M = W'W (+ tiny regularisation), M = Lm Lm'.  Fixed
variables (l = u) keep x = l; their rows/columns of K are the identity and
their columns of A are moved to the right-hand side.

BQPD itself is binary-only Fortran and absent: the objective
of a convex QP is unique, so parity is pinned by the solution's KKT
certificate (primal/dual residuals and the duality gap, checked in the
tests) rather than by BQPD's iterates — "parity unpinned" for iterates.
"""
from __future__ import annotations

import numpy as np

MAXIT = 80
STEP = 0.995
TOL_P = 1e-9
TOL_D = 1e-9
TOL_MU = 1e-10
REG = 1e-12


def _chol(K):
    return np.linalg.cholesky(K)


def _fwd(L, r):
    from scipy.linalg import solve_triangular
    return solve_triangular(L, r, lower=True, check_finite=False)


def _bwd(L, r):
    from scipy.linalg import solve_triangular
    return solve_triangular(L.T, r, lower=False, check_finite=False)


def _max_step(s, ds):
    neg = ds < 0
    if not neg.any():
        return 1.0
    return min(1.0, float(np.min(-s[neg] / ds[neg])))


def solve_node(Q, c, A, b, l, u, maxit=MAXIT):
    """One node: returns dict(status, obj, x, y, zl, zu, iters).
    status 0 converged, 6 iteration limit."""
    n = Q.shape[0]
    fixed = l >= u
    free = ~fixed
    nf = int(free.sum())
    x = np.where(free, 0.5 * (l + u), l)
    y = np.zeros(A.shape[0])
    zl = np.where(free, 1.0, 0.0)
    zu = np.where(free, 1.0, 0.0)
    Af = A.copy()
    Af[:, fixed] = 0.0
    tp = TOL_P * (1.0 + np.max(np.abs(b), initial=0.0))
    td = TOL_D * (1.0 + np.max(np.abs(c), initial=0.0))
    status = 6
    it = 0
    for it in range(maxit):
        sl = np.where(free, x - l, 1.0)
        su = np.where(free, u - x, 1.0)
        rd = np.where(free, Q @ x + c - A.T @ y - zl + zu, 0.0)
        rp = b - A @ x
        mu = float((sl[free] @ zl[free] + su[free] @ zu[free]) / max(2 * nf, 1))
        # the primal tolerance also scales with the iterate: a ranged row's
        # slack column carries the row's activity while b is 0 (hs021)
        tpx = max(tp, TOL_P * (1.0 + float(np.max(np.abs(x), initial=0.0))))
        if np.max(np.abs(rp), initial=0.0) <= tpx and np.max(np.abs(rd), initial=0.0) <= td \
                and mu <= TOL_MU:
            status = 0
            break
        D = np.where(free, zl / sl + zu / su, 0.0)
        K = Q + np.diag(D)
        K[fixed, :] = 0.0
        K[:, fixed] = 0.0
        K[fixed, fixed] = 1.0
        L = _chol(K)
        W = _fwd(L, Af.T)
        M = W.T @ W
        M += REG * (1.0 + np.max(np.diag(M), initial=0.0)) * np.eye(M.shape[0])
        Lm = _chol(M)

        def solve(r1):
            v = _fwd(L, r1)
            dy = _bwd(Lm, _fwd(Lm, rp - W.T @ v))
            dx = _bwd(L, v + W @ dy)
            return np.where(free, dx, 0.0), dy

        # predictor (affine scaling)
        r1 = np.where(free, -rd - zl + zu, 0.0)
        dx, dy = solve(r1)
        dzl = np.where(free, -zl - (zl / sl) * dx, 0.0)
        dzu = np.where(free, -zu + (zu / su) * dx, 0.0)
        ap = min(_max_step(sl[free], dx[free]), _max_step(su[free], -dx[free]))
        ad = min(_max_step(zl[free], dzl[free]), _max_step(zu[free], dzu[free]))
        mu_aff = float(((sl + ap * dx)[free] @ (zl + ad * dzl)[free]
                        + (su - ap * dx)[free] @ (zu + ad * dzu)[free]) / max(2 * nf, 1))
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        # corrector
        rl = sigma * mu - sl * zl - dx * dzl
        ru = sigma * mu - su * zu + dx * dzu
        r1 = np.where(free, -rd + rl / sl - ru / su, 0.0)
        dx, dy = solve(r1)
        dzl = np.where(free, (rl - zl * dx) / sl, 0.0)
        dzu = np.where(free, (ru + zu * dx) / su, 0.0)
        ap = STEP * min(_max_step(sl[free], dx[free]), _max_step(su[free], -dx[free]))
        ad = STEP * min(_max_step(zl[free], dzl[free]), _max_step(zu[free], dzu[free]))
        ap, ad = min(ap, 1.0), min(ad, 1.0)
        x = x + ap * dx
        y = y + ad * dy
        zl = zl + ad * dzl
        zu = zu + ad * dzu
    obj = float(0.5 * x @ Q @ x + c @ x)
    return dict(status=status, obj=obj, x=x, y=y, zl=zl, zu=zu, iters=it)


def kkt_certificate(Q, c, A, b, l, u, x, y, zl, zu):
    """Residuals of the KKT system and the duality gap of a convex QP:
    primal infeasibility, dual infeasibility (free variables), and
    gap = f(x) - dual(y, zl, zu) (>= 0; small = x optimal)."""
    free = l < u
    rp = float(np.max(np.abs(A @ x - b), initial=0.0))
    g = Q @ x + c - A.T @ y - zl + zu
    rd = float(np.max(np.abs(g[free]), initial=0.0))
    box = float(max(np.max(l - x, initial=0.0), np.max(x - u, initial=0.0)))
    # f(x) - L(x, y, z): with x primal feasible and (y, z >= 0) dual
    # feasible this bounds f(x) - f* (weak duality of the convex QP)
    gap = y @ (A @ x - b) + zl[free] @ (x - l)[free] + zu[free] @ (u - x)[free]
    zmin = float(min(np.min(zl[free], initial=0.0), np.min(zu[free], initial=0.0)))
    return dict(rp=rp, rd=rd, box=box, gap=float(gap), zmin=zmin)
