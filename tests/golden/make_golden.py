"""Generate the committed golden vectors from the REFERENCE itself.

Runs Minotaur's own LinearHandler::presolveNode (compiled from
/root/reference/src/base into oracle/_ref/libref_fbbt.so by oracle/Makefile)
on seeded node boxes and stores inputs + outputs as small .npz fixtures:

  fbbt_<case>.npz : lb_in, ub_in [B,n]; lb_out, ub_out [B,n]; infeas, nmods
                    [B]; mod_var/mod_lu/mod_val [B,cap] (push order);
                    incumbent (nan = none); the problem (LinProblem fields).

Run in the container that has /root/reference:
    make -C oracle ref && python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402
from minotaur_amd.problem import (LinProblem, knapsack_oa, random_boxes,  # noqa: E402
                                  random_problem)

OUT = os.path.dirname(os.path.abspath(__file__))
# optional: regenerate only the named cases (argv), e.g. nvs08_oa
ONLY = set(sys.argv[1:])
CAP = 256


def dump(name, p, LB, UB, incumbent):
    if ONLY and name not in ONLY:
        return
    r = oracle.ref_linear_fbbt(p, LB, UB, incumbent, CAP)
    np.savez_compressed(
        os.path.join(OUT, f'fbbt_{name}.npz'),
        lb_in=LB, ub_in=UB, lb_out=r.lb, ub_out=r.ub, infeas=r.infeas,
        nmods=r.nmods, mod_var=r.mod_var.astype(np.int16),
        mod_lu=r.mod_lu.astype(np.int8), mod_val=r.mod_val,
        incumbent=np.float64(math.nan if incumbent is None else incumbent),
        ref_us_per_node=np.float64(1e6 * r.seconds / LB.shape[0]),
        name=p.name, n=p.n, m=p.m, rowptr=p.rowptr, colidx=p.colidx, val=p.val,
        rlo=p.rlo, rhi=p.rhi, vlb=p.vlb, vub=p.vub, vtype=p.vtype, obj=p.obj,
        obj_const=p.obj_const)
    print(f'{name:24s} B={LB.shape[0]:5d} infeas={int(r.infeas.sum()):4d} '
          f'mean nmods={r.nmods.mean():6.2f} max nmods={r.nmods.max():4d} '
          f'ref {1e6 * r.seconds / LB.shape[0]:.2f} us/node')


def main():
    inst = os.path.join(ROOT, 'minotaur_amd', 'instances')
    tls4 = LinProblem.load(os.path.join(inst, 'tls4_lin.npz'))
    LB, UB = random_boxes(tls4, 256, 20261015)
    dump('tls4_noinc', tls4, LB, UB, None)
    dump('tls4_inc20', tls4, LB, UB, 20.0)
    # root box (the node every tree starts from) and a tight incumbent
    dump('tls4_root', tls4, tls4.vlb[None, :].copy(), tls4.vub[None, :].copy(), None)
    dump('tls4_inc8', tls4, LB[:64], UB[:64], 8.0)
    # config 2 as a MINLP: tls4's outer-approximation LP (tangent rows for
    # its four convex sqrt rows); OA-MILP optimum 3.2, so incumbent 3.5 drives
    # varBndsFromObj_ and the root box is the tree's first node
    oa = LinProblem.load(os.path.join(inst, 'tls4_oa.npz'))
    LB, UB = random_boxes(oa, 256, 20261017)
    LB, UB = np.vstack([oa.vlb[None], LB]), np.vstack([oa.vub[None], UB])
    dump('tls4_oa_noinc', oa, LB, UB, None)
    dump('tls4_oa_inc3p5', oa, LB, UB, 3.5)
    # config 1: the nvs08 outer-approximation LP (root + seeded boxes)
    nv = LinProblem.load(os.path.join(inst, 'nvs08_oa.npz'))
    LB, UB = random_boxes(nv, 255, 808)
    LB, UB = np.vstack([nv.vlb[None], LB]), np.vstack([nv.vub[None], UB])
    dump('nvs08_oa', nv, LB, UB, None)
    dump('nvs08_oa_inc20', nv, LB, UB, 20.0)
    ks = knapsack_oa()
    LB, UB = random_boxes(ks, 1000, 7)
    dump('knapsack_noinc', ks, LB, UB, None)
    dump('knapsack_inc3', ks, LB[:256], UB[:256], 3.0)
    for s in range(8):
        p = random_problem(s)
        LB, UB = random_boxes(p, 96, 100 + s)
        dump(f'random{s}', p, LB, UB, None if s % 2 == 0 else 0.0)
    # edge cases: empty batch rows, a fully fixed box, crossing bounds
    p = random_problem(99, n=30, m=20)
    LB, UB = random_boxes(p, 32, 5)
    LB[0] = UB[0] = np.where(np.isfinite(p.vlb), p.vlb, 0.0)   # fixed box
    LB[1, 3], UB[1, 3] = 2.0, 1.0                               # crossing
    LB[2, :] = -math.inf
    UB[2, :] = math.inf                                         # free box
    dump('edge', p, LB, UB, None)


if __name__ == '__main__':
    main()
