"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the batched branch-and-bound tree step
(minotaur_amd/csrc/bnb.cpp + bnb.hip + the branching part of
node_decide.hip) over the C oracles: same node stack, same round structure,
same decisions (PCBProcessor::shouldPrune_ tolerances, IntVarHandler
integrality, MaxVioBrancher score and direction, IntVarHandler::getBranches
children), same stack order.  ``CpuBnbContext`` exposes the engine's
bnb_* methods so minotaur_amd.bnb's drivers run unchanged on it (gloo
tests of the multi-rank control flow, and tree-parity checks of the GPU
driver).
"""
from __future__ import annotations

import math

import numpy as np

import oracle

ABS_TOL = REL_TOL = INT_TOL = 1e-6


class _Stats:
    def __init__(self):
        self.rounds = self.nodes = 0
        self.ndec = [0, 0, 0, 0, 0]
        self.open = 0
        self.last_batch = 0
        self.incumbent = math.inf


class CpuBnbContext:
    def __init__(self, p, pfi=0):
        self.problem = p
        self.pfi = pfi   # node LPs in K3P's product form (Context.oracle_pfi())

    # -- mgpu_bnb_init ------------------------------------------------------
    def bnb_init(self, capacity, root_lb=None, root_ub=None, incumbent=math.inf):
        p = self.problem
        lb = np.array(p.vlb if root_lb is None else root_lb, dtype=np.float64)
        ub = np.array(p.vub if root_ub is None else root_ub, dtype=np.float64)
        self.cap = capacity
        self.pool = [(lb, ub, -math.inf, 0)]
        st, obj, x, y, it, ws = oracle.dual_simplex_root(p, lb, ub)
        self.ws = ws if st == 0 else None
        self.inc = incumbent
        self.best_x = np.full(p.n, np.nan)
        self.tot = _Stats()
        self.tot.incumbent = incumbent

    # -- mgpu_bnb_round -----------------------------------------------------
    def bnb_round(self, batch, incumbent=math.inf):
        p = self.problem
        if incumbent < self.inc:
            self.inc = incumbent
        count = len(self.pool)
        nb = min(batch, count, self.cap - count)
        if nb <= 0:
            self.tot.open = len(self.pool)
            return self.tot
        base = count - nb
        nodes = self.pool[base:]
        del self.pool[base:]
        LB = np.stack([n[0] for n in nodes])
        UB = np.stack([n[1] for n in nodes])
        f = oracle.linear_fbbt(p, LB, UB, self.inc if math.isfinite(self.inc) else None)
        status = np.full(nb, 12, dtype=np.int32)
        obj = np.full(nb, math.inf)
        x = np.zeros((nb, p.n))
        keep = np.nonzero(f.infeas == 0)[0]
        if keep.size:
            s2, o2, _, x2 = oracle.dual_simplex(p, f.lb[keep], f.ub[keep], self.ws, want_x=True,
                                                 pfi=self.pfi if self.ws is not None else 0)
            status[keep], obj[keep], x[keep] = s2, o2, x2
        ints = np.isin(p.vtype, (0, 1))
        children = []
        best, best_i = math.inf, -1
        for i in range(nb):
            dec = self._decide(f.infeas[i], status[i], obj[i], x[i], ints)
            self.tot.ndec[dec] += 1
            if dec == 3 and (obj[i] < best):
                best, best_i = obj[i], i
            if dec != 0:
                continue
            j, v, up_first = self._branch(x[i], ints)
            down = (f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i][3] + 1)
            down[1][j] = math.floor(v)
            up = (f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i][3] + 1)
            up[0][j] = math.ceil(v)
            children += [down, up] if up_first else [up, down]   # preferred on top
        self.pool += children
        if best_i >= 0 and best < self.inc:
            self.inc = best
            self.best_x = x[best_i].copy()
        self.tot.rounds += 1
        self.tot.nodes += nb
        self.tot.open = len(self.pool)
        self.tot.last_batch = nb
        self.tot.incumbent = self.inc
        return self.tot

    def _decide(self, finf, st, solval, x, ints):
        dec, _ = oracle.node_decide(self.problem.vtype, [st], [solval], x[None], self.inc,
                                    [finf], ABS_TOL, REL_TOL, math.inf, INT_TOL)
        return int(dec[0])

    @staticmethod
    def _branch(x, ints):
        best, bj = -math.inf, -1
        for j in np.nonzero(ints)[0]:
            v = x[j]
            if not abs(math.floor(v + 0.5) - v) > INT_TOL:
                continue
            dd, ud = v - math.floor(v), math.ceil(v) - v
            sc = 0.1 * (0.8 * min(dd, ud) + 0.2 * max(dd, ud))
            if sc > best:
                best, bj = sc, int(j)
        v = x[bj]
        return bj, v, (v - math.floor(v)) > (math.ceil(v) - v)

    # -- mgpu_bnb_shard / mgpu_bnb_best ---------------------------------------
    def bnb_shard(self, rank, world):
        self.pool = self.pool[rank::world]
        self.tot.open = len(self.pool)
        return len(self.pool)

    def bnb_best(self):
        return self.inc, self.best_x.copy()
