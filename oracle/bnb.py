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
  optimal basis, whose own optimum is handed to both children; warm 2: from
  the parent's optimal basis kept as its pivot path from the root basis
  (oracle.dual_simplex_path, K3P's product form), paths of at most
  min(PATH_INHERIT = 32, pfi) basic columns handed on, else the children
  restart from the root;
* brancher 0: MaxVioBrancher; brancher 1: the batched ReliabilityBrancher of
  bnb_rel.hip (pseudocosts frozen at the round's start plus each node's own
  updateAfterSolve observation, strong-branching LPs from each node's optimal
  basis with iteration limit 25, observations folded in node order).

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
        self.sb_lps = self.sb_pivots = self.sb_pruned = self.sb_modified = 0
        self.pfi_pivots = 0


def _order_key(v):
    """order_key() of bnb_select.hip: IEEE f64 bits mapped to an unsigned
    integer with the same order (-0.0 before +0.0)."""
    b = struct.unpack('<Q', struct.pack('<d', v))[0]
    return (~b) & 0xFFFFFFFFFFFFFFFF if b >> 63 else b | (1 << 63)


class _Node:
    __slots__ = ('lb', 'ub', 'nlb', 'depth', 'ws', 'pvar', 'pval', 'path')

    def __init__(self, lb, ub, nlb, depth, ws=None, pvar=-1, pval=0.0, path=None):
        self.lb, self.ub, self.nlb, self.depth, self.ws = lb, ub, nlb, depth, ws
        self.pvar, self.pval = pvar, pval
        self.path = path    # warm 2: (k, pivots, statuses) or None = the root basis


# ReliabilityBrancher defaults (ReliabilityBrancher.cpp:43-58)
REL_MAX_CANDS, REL_ITER, REL_THRESH, REL_MIN_DIST, REL_ETOL = 20, 25, 4, 50, 1e-6
REL_MAX_DEPTH = 1000   # maxDepth_: no strong branching below it (:105)
PATH_MAX = oracle.PATH_MAX   # path slots per node (MGPU_PATH_MAX)
PATH_INHERIT = 32      # warm 2: longest basis difference handed to children (bnb.cpp kPathInherit)


def _rel_score(up, down):
    """ReliabilityBrancher::getScore_ (:368-377)."""
    return down * 0.8 + up * 0.2 if up > down else up * 0.8 + down * 0.2


def _fractional(v):
    return abs(math.floor(v + 0.5) - v) > INT_TOL


class CpuBnbContext:
    def __init__(self, p, pfi=0, order=0, warm=0, brancher=0):
        self.problem = p
        self.pfi = pfi   # node LPs in K3P's product form (Context.oracle_pfi())
        self.order, self.warm = order, warm
        self.brancher = brancher
        self.grow_next = 0

    def bnb_config(self, order=0, warm=0):
        self.order, self.warm = int(order), int(warm)

    def bnb_brancher(self, kind):
        self.brancher = int(kind)

    def bnb_growth(self, div):
        """mgpu_bnb_growth: rounds of at most max(1, nodes so far // div)."""
        self.grow_next = int(div)

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
        self.grow = self.grow_next
        self.rel = self.brancher == 1
        if self.rel:   # ReliabilityBrancher::initialize (:384-398)
            n = p.n
            self.pc_up, self.pc_dn = [0.0] * n, [0.0] * n
            self.cnt_up, self.cnt_dn = [0] * n, [0] * n
            self.last = [20000] * n
            self.calls = 0

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
        if self.grow > 0:     # mgpu_bnb_growth (bnb.cpp mgpu_bnb_round)
            batch = min(batch, max(1, self.tot.nodes // self.grow))
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
            if self.rel and not self.warm:
                # the node's optimal basis is needed: dense solve from the root
                k = keep.size
                ws = oracle.WarmStart(*(np.stack([getattr(self.ws, a)] * k)
                                        for a in ('head', 'st', 'binv', 'd')))
                s2, o2, i2, x2, w2 = oracle.dual_simplex_nodes(p, f.lb[keep], f.ub[keep], ws)
                for t, i in enumerate(keep):
                    wo[i] = oracle.WarmStart(w2.head[t].copy(), w2.st[t].copy(),
                                             w2.binv[t].copy(), w2.d[t].copy())
            elif self.warm == 2:
                N = p.n + p.m
                k_in = np.zeros(keep.size, np.int32)
                path_in = np.zeros((keep.size, oracle.PATH_MAX), np.uint32)
                st_in = np.zeros((keep.size, N), np.int8)
                for t, i in enumerate(keep):
                    if nodes[i].path is not None:
                        k_in[t], path_in[t], st_in[t] = nodes[i].path
                s2, o2, i2, x2, ko, po, so = oracle.dual_simplex_path(
                    p, f.lb[keep], f.ub[keep], self.ws, k_in, path_in, st_in, self.pfi,
                    min(PATH_INHERIT, self.pfi))
                self.tot.pfi_pivots += int(np.minimum(i2, np.maximum(self.pfi - k_in, 0)).sum())
                for t, i in enumerate(keep):
                    wo[i] = (int(ko[t]), po[t].copy(), so[t].copy()) if ko[t] > 0 else None
            elif self.warm:
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
                if self.ws is not None and self.pfi > 0:
                    self.tot.pfi_pivots += int(np.minimum(i2, self.pfi).sum())
            status[keep], obj[keep], x[keep] = s2, o2, x2
            self.tot.lps += int(keep.size)
            self.tot.pivots += int(np.sum(i2))
        ints = np.isin(p.vtype, (0, 1))
        children = []
        best, best_i = math.inf, -1
        decs = [self._decide(f.infeas[i], status[i], obj[i], x[i], ints) for i in range(nb)]
        if self.rel:
            choice = self._rel_round(nodes, decs, obj, x, f, wo)
        for i in range(nb):
            dec = decs[i]
            self.tot.ndec[0 if dec == 5 else dec] += 1
            if dec == 3 and (obj[i] < best):
                best, best_i = obj[i], i
            if dec not in (0, 5):
                continue
            if self.rel:
                j, v, up_first = choice[i]
            else:
                j, v, up_first = self._branch(x[i], ints)
            w = wo[i] if self.warm == 1 else self.ws
            path = wo[i] if self.warm == 2 else None
            if dec == 5:
                # ModifiedByBrancher: the node again with the bound change,
                # from the basis its strong branching left (warm 1)
                wm = self._chain[i] if self.warm == 1 else w
                nd = _Node(f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i].depth, wm)
                if up_first:
                    nd.lb[j] = math.ceil(v)
                else:
                    nd.ub[j] = math.floor(v)
                children.append(nd)
                continue
            down = _Node(f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i].depth + 1, w, j, v,
                         path)
            down.ub[j] = math.floor(v)
            up = _Node(f.lb[i].copy(), f.ub[i].copy(), obj[i], nodes[i].depth + 1, w, j, v, path)
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

    # -- batched reliability branching (bnb_rel.hip) ----------------------------
    def _rel_round(self, nodes, decs, obj, x, f, wo):
        """Restates rel_prepare / the strong-branching LP batch / rel_decide /
        pc_fold over the round; updates ``decs`` in place (1 pruned by the
        brancher, 5 modified) and returns {node: (var, value, up_first)}."""
        p = self.problem
        nb = len(nodes)
        ints = [j for j in range(p.n) if p.vtype[j] in (0, 1)]
        obs, calls, sb = {}, {}, {}
        rank = 0
        for i in range(nb):
            if decs[i] == 0:
                calls[i] = self.calls + rank + 1
                rank += 1
            nd = nodes[i]
            if nd.pvar >= 0 and decs[i] in (0, 3):
                newval, oldval = x[i][nd.pvar], nd.pval
                c = (obj[i] - nd.nlb) / (abs(newval - oldval) + REL_ETOL)
                if c < 0.0 or math.isinf(c) or math.isnan(c):
                    c = 0.0
                obs[i] = (nd.pvar, 0 if newval < oldval else 1, c)

        def view(i, j):
            pu, pd, cu, cd = self.pc_up[j], self.pc_dn[j], self.cnt_up[j], self.cnt_dn[j]
            o = obs.get(i)
            if o is not None and o[0] == j:
                if o[1] == 0:
                    pd = (pd * cd + o[2]) / (cd + 1)
                    cd += 1
                else:
                    pu = (pu * cu + o[2]) / (cu + 1)
                    cu += 1
            return pu, pd, cu, cd

        def reliable(i, j, v):
            d = (calls[i] - self.last[j]) & 0xFFFFFFFF
            return float(REL_MIN_DIST) > abs(float(d)) or (v[2] >= REL_THRESH and
                                                           v[3] >= REL_THRESH)

        def unrel_sorted(i):
            out = []
            for j in ints:
                v = x[i][j]
                if not _fractional(v):
                    continue
                pv = view(i, j)
                if reliable(i, j, pv):
                    continue
                dd, ud = v - math.floor(v), math.ceil(v) - v
                out.append(((pv[2] + pv[3]) - 1e-5 * (pv[0] + pv[1]) - 1e-6 * max(dd, ud), j))
            return [j for _, j in sorted(out)]

        def sb_prune(chcut, change, st):
            if st in (3, 2, 5):
                return True, True
            if st in (1, 0):
                return change > chcut - REL_ETOL, True
            if st == 6:
                return False, True
            return False, False

        # the strong-branching LPs, chained per node as the reference's engine
        # runs them (strongBranch_ through one LPEngine, :469-506): each LP
        # from the basis the previous optimal / iteration-limited one left
        # (the first from the node's optimal basis), a node stopping after the
        # first candidate with a verdict (findBestCandidate_ :111-118); step s
        # is the s-th LP of every node still strong-branching (bnb_rel.hip)
        for i in range(nb):
            if decs[i] == 0:
                maxcnt = 0 if nodes[i].depth > REL_MAX_DEPTH else REL_MAX_CANDS
                sb[i] = unrel_sorted(i)[:maxcnt]
        sbn = [i for i in range(nb) if decs[i] == 0 and sb[i]]
        chain = {i: wo[i] for i in sbn}
        res = {i: [] for i in sbn}
        stopped = set()
        for step in range(2 * max((len(sb[i]) for i in sbn), default=0)):
            act = [i for i in sbn if i not in stopped and step < 2 * len(sb[i])]
            if not act:
                break
            kl, ku = [], []
            for i in act:
                j = sb[i][step >> 1]
                v = x[i][j]
                lb, ub = f.lb[i].copy(), f.ub[i].copy()
                if step & 1:
                    lb[j] = math.ceil(v)
                else:
                    ub[j] = math.floor(v)
                kl.append(lb)
                ku.append(ub)
            ws = oracle.WarmStart(*(np.stack([getattr(chain[i], a) for i in act])
                                    for a in ('head', 'st', 'binv', 'd')))
            cst, cobj, cit, _, w2 = oracle.dual_simplex_nodes(
                p, np.stack(kl), np.stack(ku), ws, iter_limit=REL_ITER)
            for t, i in enumerate(act):
                res[i].append((int(cst[t]), float(cobj[t]), int(cit[t])))
                chain[i] = oracle.WarmStart(w2.head[t].copy(), w2.st[t].copy(),
                                            w2.binv[t].copy(), w2.d[t].copy())
                if step & 1:
                    (sd, od, _), (su, ou, _) = res[i][-2], res[i][-1]
                    mc = self.inc - obj[i]
                    pd_, rd = sb_prune(mc, max(od - obj[i], 0.0), sd)
                    pu_, ru = sb_prune(mc, max(ou - obj[i], 0.0), su)
                    if rd and ru and (pd_ or pu_):
                        stopped.add(i)
        for i in sbn:
            self.tot.sb_lps += len(res[i])
            self.tot.sb_pivots += sum(r[2] for r in res[i])
        self._chain = chain
        choice, events = {}, []
        last_upd = {}

        for i in range(nb):
            if i in obs:
                events.append(obs[i])
            if decs[i] != 0:
                continue
            xi = x[i]
            objval = obj[i]
            best, bj, down_first = -math.inf, -1, False
            for j in ints:
                v = xi[j]
                if not _fractional(v):
                    continue
                pv = view(i, j)
                if not reliable(i, j, pv):
                    continue
                cd, cu = (v - math.floor(v)) * pv[1], (math.ceil(v) - v) * pv[0]
                sc = _rel_score(cu, cd)
                if sc > best:
                    best, bj, down_first = sc, j, cu > cd
            maxchange = self.inc - objval
            status = 0
            mod = None
            for k, j in enumerate(sb[i]):
                v = xi[j]
                dd, ud = v - math.floor(v), math.ceil(v) - v
                (sd, od, _), (su, ou, _) = res[i][2 * k], res[i][2 * k + 1]
                cd = max(od - objval, 0.0)
                cu = max(ou - objval, 0.0)
                pd_, rel_d = sb_prune(maxchange, cd, sd)
                pu_, rel_u = sb_prune(maxchange, cu, su)
                if not (rel_d and rel_u):
                    cu = cd = 0.0
                elif pu_ and pd_:
                    status = 1
                elif pu_:
                    status, mod = 2, (j, v, False)
                elif pd_:
                    status, mod = 2, (j, v, True)
                else:
                    events.append((j, 0, abs(cd) / (abs(dd) + REL_ETOL)))
                    events.append((j, 1, abs(cu) / (abs(ud) + REL_ETOL)))
                sc = _rel_score(cu, cd)
                last_upd[j] = max(last_upd.get(j, -1), calls[i])
                if status != 0:
                    break
                if sc > best:
                    best, bj, down_first = sc, j, cu > cd
            if status == 0:
                for j in unrel_sorted(i)[len(sb[i]):]:
                    v = xi[j]
                    pv = view(i, j)
                    cd, cu = (v - math.floor(v)) * pv[1], (math.ceil(v) - v) * pv[0]
                    sc = _rel_score(cu, cd)
                    if sc > best:
                        best, bj, down_first = sc, j, cu > cd
                choice[i] = (bj, xi[bj], not down_first)
            elif status == 1:
                decs[i] = 1
                self.tot.sb_pruned += 1
            else:
                decs[i] = 5
                choice[i] = mod
                self.tot.sb_modified += 1
        for j, c in last_upd.items():   # the round's last writer (largest call number)
            self.last[j] = c
        for j, side, c in events:      # updatePCost_ in node order
            if side == 0:
                self.pc_dn[j] = (self.pc_dn[j] * self.cnt_dn[j] + c) / (self.cnt_dn[j] + 1)
                self.cnt_dn[j] += 1
            else:
                self.pc_up[j] = (self.pc_up[j] * self.cnt_up[j] + c) / (self.cnt_up[j] + 1)
                self.cnt_up[j] += 1
        self.calls += rank
        return choice

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
        self.pick = []
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

    def _place(self, nodes):
        """mgpu_bnb_import[_dev]'s placement: on top of the stack, or the
        lowest free slots first, then past the high-water mark."""
        if self.order == 0:
            self.pool.extend(nodes)
        else:
            free = [i for i, nd in enumerate(self.pool) if nd is None]
            for t, nd in enumerate(nodes):
                if t < len(free):
                    self.pool[free[t]] = nd
                else:
                    self.pool.append(nd)
        self.tot.open = sum(nd is not None for nd in self.pool)

    def _migrant(self, lb, ub, nlb, depth):
        # a migrated node starts from the root basis, without parent
        # branching data
        return _Node(np.array(lb, dtype=np.float64), np.array(ub, dtype=np.float64),
                     float(nlb), int(depth), self.ws)

    def bnb_import(self, lb, ub, nlb, depth):
        """mgpu_bnb_import."""
        self._place([self._migrant(lb[t], ub[t], nlb[t], depth[t]) for t in range(len(nlb))])

    # -- mgpu_bnb_pick / export_dev / import_dev (LoadBalance_) ----------------
    def bnb_pick(self, S):
        """The next S candidates: the stack's top (topmost first), or the
        live nodes pruned by the incumbent and sorted by (bound, slot)."""
        if self.order == 0:
            k = min(int(S), len(self.pool))
            self.pick = [len(self.pool) - 1 - t for t in range(k)]
        else:
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
            self.tot.open = len(live)
            self.pick = live[:int(S)]
        return np.array([self.pool[i].nlb for i in self.pick], dtype=np.float64)

    def bnb_row_width(self):
        n, N = self.problem.n, self.problem.n + self.problem.m
        return 2 * n + 2 + (1 + PATH_MAX + (N + 15) // 16 if self.warm == 2 else 0)

    def bnb_export_rows(self, idx):
        """Rows [k, W] = [lb | ub | bound | depth] of picked nodes idx, in
        warm mode 2 followed by [k | path (PATH_MAX, zeros past k) | column
        statuses, 16 two-bit codes per f64 (zeros for k = 0)]
        (bnb_migrate.hip), removed from the pool (the stack keeps the
        others' order)."""
        import torch
        n, N = self.problem.n, self.problem.n + self.problem.m
        slots = [self.pick[int(i)] for i in idx]
        assert len(set(slots)) == len(slots)
        rows = torch.zeros((len(slots), self.bnb_row_width()), dtype=torch.float64)
        for t, sl in enumerate(slots):
            nd = self.pool[sl]
            rows[t, :n] = torch.from_numpy(np.asarray(nd.lb, dtype=np.float64))
            rows[t, n:2 * n] = torch.from_numpy(np.asarray(nd.ub, dtype=np.float64))
            rows[t, 2 * n] = float(nd.nlb)
            rows[t, 2 * n + 1] = float(nd.depth)
            if self.warm == 2 and nd.path is not None and int(nd.path[0]) > 0:
                k, pv, sv = nd.path
                w = 2 * n + 2
                rows[t, w] = float(k)
                for i in range(int(k)):
                    rows[t, w + 1 + i] = float(int(pv[i]))
                sv = np.asarray(sv, dtype=np.int64) & 3
                for q in range((N + 15) // 16):
                    bits = 0
                    for i in range(16):
                        if q * 16 + i < N:
                            bits |= int(sv[q * 16 + i]) << (2 * i)
                    rows[t, w + 1 + PATH_MAX + q] = float(bits)
        if self.order == 0:
            gone = set(slots)
            self.pool = [nd for i, nd in enumerate(self.pool) if i not in gone]
        else:
            for sl in slots:
                self.pool[sl] = None
        self.pick = []
        self.tot.open = sum(nd is not None for nd in self.pool)
        return rows

    def bnb_import_rows(self, rows):
        n, N = self.problem.n, self.problem.n + self.problem.m
        v = rows.detach().cpu().numpy()
        nodes = []
        for r in v:
            nd = self._migrant(r[:n], r[n:2 * n], r[2 * n], int(r[2 * n + 1]))
            w = 2 * n + 2
            if self.warm == 2 and int(r[w]) > 0:   # the basis the row carries
                k = int(r[w])
                pv = np.zeros(PATH_MAX, dtype=np.uint32)
                pv[:] = r[w + 1:w + 1 + PATH_MAX].astype(np.uint64).astype(np.uint32)
                sv = np.zeros(N, dtype=np.int8)
                for j in range(N):
                    sv[j] = (int(r[w + 1 + PATH_MAX + j // 16]) >> (2 * (j % 16))) & 3
                nd.path = (k, pv, sv)
            nodes.append(nd)
        self._place(nodes)

    def bnb_count(self):
        live = sum(nd is not None for nd in self.pool)
        return live, self.cap - live

    def bnb_best(self):
        return self.inc, self.best_x.copy()
