"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the batched branch-and-bound tree step
(minotaur_amd/csrc/bnb.cpp + bnb.hip + bnb_select.hip + the branching part of
node_decide.hip) over the C oracles: same node pool, same round structure,
same decisions (PCBProcessor::shouldPrune_ tolerances, IntVarHandler
integrality, MaxVioBrancher score and direction, IntVarHandler::getBranches
children), same pool order:

* order 0 (depth-first): the pool is a stack, the preferred child on top;
* order 1 (best-first): open nodes pruned by TreeManager::shouldPrune_'s rule,
  then the `batch` nodes with the lowest (bound, slot) are taken; children go
  to the free slots in the engine's order (the slots just taken, the older
  holes ascending, then new slots);
* warm 0: node LPs from the root optimum (shared); warm 1: from the parent's
  optimal basis, whose own optimum is handed to both children.

``CpuBnbContext`` exposes the engine's bnb_* methods so minotaur_amd.bnb's
drivers run unchanged on it (gloo tests of the multi-rank control flow, and
tree-parity checks of the GPU driver).
"""
from __future__ import annotations

import math
import struct

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
        self.pruned = 0
        self.lps = self.pivots = 0


def _order_key(v):
    """order_key() of bnb_select.hip: IEEE f64 bits mapped to an unsigned
    integer with the same order (-0.0 before +0.0)."""
    b = struct.unpack('<Q', struct.pack('<d', v))[0]
    return (~b) & 0xFFFFFFFFFFFFFFFF if b >> 63 else b | (1 << 63)


class _Node:
    __slots__ = ('lb', 'ub', 'nlb', 'depth', 'ws')

    def __init__(self, lb, ub, nlb, depth, ws=None):
        self.lb, self.ub, self.nlb, self.depth, self.ws = lb, ub, nlb, depth, ws


class CpuBnbContext:
    def __init__(self, p, pfi=0, order=0, warm=0):
        self.problem = p
        self.pfi = pfi   # node LPs in K3P's product form (Context.oracle_pfi())
        self.order, self.warm = order, warm

    def bnb_config(self, order=0, warm=0):
        self.order, self.warm = int(order), int(warm)

    # -- mgpu_bnb_init ------------------------------------------------------
    def bnb_init(self, capacity, root_lb=None, root_ub=None, incumbent=math.inf):
        p = self.problem
        lb = np.array(p.vlb if root_lb is None else root_lb, dtype=np.float64)
        ub = np.array(p.vub if root_ub is None else root_ub, dtype=np.float64)
        self.cap = capacity
        st, obj, x, y, it, ws = oracle.dual_simplex_root(p, lb, ub, iter_limit=10000)
        self.ws = ws if st == 0 else None
        self.pool = [_Node(lb, ub, -math.inf, 0, self.ws)]   # stack, or slots (None = free)
        self.inc = incumbent
        self.best_x = np.full(p.n, np.nan)
        self.tot = _Stats()
        self.tot.incumbent = incumbent

    # -- mgpu_bnb_round -----------------------------------------------------
    def _select(self, batch):
        """Best-first: prune, sort, take; returns (nodes, free slots, live)."""
        inc = float(self.inc)
        for i, nd in enumerate(self.pool):
            if nd is None:
                continue
            lb = float(nd.nlb)
            if lb > inc - 1e-6 or abs(inc - lb) / (abs(inc) + 1e-6) * 100.0 < 1e-6:
                self.pool[i] = None
                self.tot.pruned += 1
        live = sorted((i for i, nd in enumerate(self.pool) if nd is not None),
                      key=lambda i: (_order_key(self.pool[i].nlb), i))
        holes = [i for i, nd in enumerate(self.pool) if nd is None]
        nb = min(batch, len(live))
        sel = live[:nb]
        nodes = [self.pool[i] for i in sel]
        for i in sel:
            self.pool[i] = None
        return nodes, sel + holes, len(live)

    def bnb_round(self, batch, incumbent=math.inf):
        p = self.problem
        if incumbent < self.inc:
            self.inc = incumbent
        if self.order == 0:
            count = len(self.pool)
            nb = min(batch, count, self.cap - count)
            if nb <= 0:
                self.tot.open = len(self.pool)
                return self.tot
            base = count - nb
            nodes = self.pool[base:]
            del self.pool[base:]
            free = None
        else:
            nodes, free, live = self._select(batch)
            nb = len(nodes)
            self.tot.open = live
            if nb == 0:
                return self.tot
        LB = np.stack([nd.lb for nd in nodes])
        UB = np.stack([nd.ub for nd in nodes])
        f = oracle.linear_fbbt(p, LB, UB, self.inc if math.isfinite(self.inc) else None)
        status = np.full(nb, 12, dtype=np.int32)
        obj = np.full(nb, math.inf)
        x = np.zeros((nb, p.n))
        wo = [None] * nb
        keep = np.nonzero(f.infeas == 0)[0]
        if keep.size:
            if self.warm:
                ws = oracle.WarmStart(*(np.stack([getattr(nodes[i].ws, k) for i in keep])
                                        for k in ('head', 'st', 'binv', 'd')))
                s2, o2, i2, x2, w2 = oracle.dual_simplex_nodes(p, f.lb[keep], f.ub[keep], ws)
                for t, i in enumerate(keep):
                    wo[i] = oracle.WarmStart(w2.head[t].copy(), w2.st[t].copy(),
                                             w2.binv[t].copy(), w2.d[t].copy())
            else:
                s2, o2, i2, x2 = oracle.dual_simplex(p, f.lb[keep], f.ub[keep], self.ws,
                                                      want_x=True,
                                                      pfi=self.pfi if self.ws is not None else 0)
            status[keep], obj[keep], x[keep] = s2, o2, x2
            self.tot.lps += int(keep.size)
            self.tot.pivots += int(np.sum(i2))
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
            w = wo[i] if self.warm else self.ws
            down = _Node(f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i].depth + 1, w)
            down.ub[j] = math.floor(v)
            up = _Node(f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i].depth + 1, w)
            up.lb[j] = math.ceil(v)
            if self.order == 0:
                children += [down, up] if up_first else [up, down]   # preferred on top
            else:
                children += [up, down] if up_first else [down, up]   # preferred: lower index
        if self.order == 0:
            self.pool += children
        else:
            hw = len(self.pool)
            for c, nd in enumerate(children):
                s = free[c] if c < len(free) else hw + (c - len(free))
                while s >= len(self.pool):
                    self.pool.append(None)
                self.pool[s] = nd
        if best_i >= 0 and best < self.inc:
            self.inc = best
            self.best_x = x[best_i].copy()
        self.tot.rounds += 1
        self.tot.nodes += nb
        self.tot.open = sum(nd is not None for nd in self.pool)
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
        if self.order == 0:
            self.pool = self.pool[rank::world]
        else:
            idx = 0
            for i, nd in enumerate(self.pool):
                if nd is None:
                    continue
                if idx % world != rank:
                    self.pool[i] = None
                idx += 1
        self.tot.open = sum(nd is not None for nd in self.pool)
        return self.tot.open

    def bnb_export(self, k):
        """mgpu_bnb_export: the stack's top k, or the first k live slots."""
        n = self.problem.n
        if self.order == 0:
            k = min(k, len(self.pool))
            nodes = self.pool[len(self.pool) - k:]
            del self.pool[len(self.pool) - k:]
        else:
            idx = [i for i, nd in enumerate(self.pool) if nd is not None][:k]
            nodes = [self.pool[i] for i in idx]
            for i in idx:
                self.pool[i] = None
        self.tot.open = sum(nd is not None for nd in self.pool)
        if not nodes:
            return np.empty((0, n)), np.empty((0, n)), np.empty(0), np.empty(0, np.int32)
        return (np.stack([nd.lb for nd in nodes]), np.stack([nd.ub for nd in nodes]),
                np.array([nd.nlb for nd in nodes]), np.array([nd.depth for nd in nodes],
                                                             dtype=np.int32))

    def bnb_import(self, lb, ub, nlb, depth):
        """mgpu_bnb_import: on top of the stack / past the high-water mark;
        with parent warm starts a migrated node starts from the root basis."""
        for t in range(len(nlb)):
            self.pool.append(_Node(np.array(lb[t]), np.array(ub[t]), float(nlb[t]),
                                   int(depth[t]), self.ws))
        self.tot.open = sum(nd is not None for nd in self.pool)

    def bnb_best(self):
        return self.inc, self.best_x.copy()
