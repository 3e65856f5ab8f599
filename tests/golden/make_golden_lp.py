"""LP golden vectors: HiGHS (scipy 1.15.3 linprog method='highs') objective
and status for seeded node boxes, plus the AMPLOsiUT known answers
(src/testing/AMPLOsiUT.cpp:46-120: lp0 -> -8.42857 ProvenOptimal, lp_eg0 ->
ProvenInfeasible), re-encoded by hand from src/testing/instances/*.mod.

  lp_<case>.npz : lb, ub [B,n]; status [B] (EngineStatus numerics);
                  obj [B] (incl. constant; inf when infeasible); the problem.
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402
from minotaur_amd.problem import (LinProblem, from_rows, knapsack_oa,  # noqa: E402
                                  random_boxes, random_problem)

OUT = os.path.dirname(os.path.abspath(__file__))
# optional: regenerate only the named cases (argv), e.g. nvs08_oa
ONLY = set(sys.argv[1:])
INF = math.inf


def known_problems():
    # lp0.mod: max 4x1 - x2 s.t. 7x1-2x2<=14, x2<=3, 2x1-2x2<=3 (x free)
    lp0 = from_rows('lp0', 2, [[(0, 7), (1, -2)], [(1, 1)], [(0, 2), (1, -2)]],
                    [-INF] * 3, [14, 3, 3], [-INF] * 2, [INF] * 2, [4, 4], [-4, 1])
    # lp_eg0.mod: min x0+x1+x2, x0+x1<=3, x0+x2<=0, x0,x1>=0, x2>=1
    lpeg0 = from_rows('lp_eg0', 3, [[(0, 1), (1, 1)], [(0, 1), (2, 1)]], [-INF] * 2, [3, 0],
                      [0, 0, 1], [INF] * 3, [4, 4, 4], [1, 1, 1])
    # milp.mod relaxation: min x4, 2x0+2x1+2x2+2x3+x4 = 1, x binary
    milp = from_rows('milp', 5, [[(0, 2), (1, 2), (2, 2), (3, 2), (4, 1)]], [1], [1],
                     [0] * 5, [1] * 5, [0] * 5, [0, 0, 0, 0, 1])
    return [lp0, lpeg0, milp]


def dump(name, p, LB, UB):
    if ONLY and name not in ONLY:
        return
    st = np.zeros(LB.shape[0], dtype=np.int32)
    obj = np.zeros(LB.shape[0])
    for b in range(LB.shape[0]):
        st[b], obj[b] = oracle.highs(p, LB[b], UB[b])
    np.savez_compressed(os.path.join(OUT, f'lp_{name}.npz'), lb=LB, ub=UB, status=st, obj=obj,
                        name=p.name, n=p.n, m=p.m, rowptr=p.rowptr, colidx=p.colidx,
                        val=p.val, rlo=p.rlo, rhi=p.rhi, vlb=p.vlb, vub=p.vub,
                        vtype=p.vtype, obj_c=p.obj, obj_const=p.obj_const)
    print(f'{name:16s} B={LB.shape[0]:4d} status counts {np.bincount(st, minlength=5)}')


def main():
    for p in known_problems():
        dump(p.name, p, p.vlb[None], p.vub[None])
    inst = os.path.join(ROOT, 'minotaur_amd', 'instances')
    tls4 = LinProblem.load(os.path.join(inst, 'tls4_lin.npz'))
    LB, UB = random_boxes(tls4, 200, 20261015)
    dump('tls4', tls4, np.vstack([tls4.vlb[None], LB]), np.vstack([tls4.vub[None], UB]))
    oa = LinProblem.load(os.path.join(inst, 'tls4_oa.npz'))
    LB, UB = random_boxes(oa, 200, 20261017)
    dump('tls4_oa', oa, np.vstack([oa.vlb[None], LB]), np.vstack([oa.vub[None], UB]))
    nv = LinProblem.load(os.path.join(inst, 'nvs08_oa.npz'))
    LB, UB = random_boxes(nv, 200, 808)
    dump('nvs08_oa', nv, np.vstack([nv.vlb[None], LB]), np.vstack([nv.vub[None], UB]))
    ks = knapsack_oa()
    LB, UB = random_boxes(ks, 300, 7)
    dump('knapsack', ks, np.vstack([ks.vlb[None], LB]), np.vstack([ks.vub[None], UB]))
    for s in range(6):
        p = random_problem(s)
        LB, UB = random_boxes(p, 40, 100 + s, max_depth=4)
        dump(f'random{s}', p, np.vstack([p.vlb[None], LB]), np.vstack([p.vub[None], UB]))


if __name__ == '__main__':
    main()
