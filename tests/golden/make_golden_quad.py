"""Generate the committed quadratic-FBBT golden vectors from the REFERENCE.

Runs Minotaur's own QuadHandler::presolveNode (src/base/QuadHandler.cpp:
1204-1269, compiled from /root/reference/src/base with the driver
oracle/ref/ref_quad.cpp into oracle/_ref/libref_fbbt.so) on seeded QCQPs and
node boxes, and stores inputs + outputs as small .npz fixtures:

  quad_<case>.npz : the QuadProblem fields; lb_in, ub_in [B,nv]; rows_in [R]
                    (the reference's relax_ rows at the root); qt; incumbent
                    (nan = none); lb_out, ub_out [B,nv]; rows_out [B,R];
                    infeas, nmods [B]; mod_kind/mod_idx/mod_v1/mod_v2
                    [B,cap] in r_mods order.

Run in the container that has /root/reference:
    make -C oracle ref && python tests/golden/make_golden_quad.py
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402
from minotaur_amd.quad import (_ARRAYS, from_functions, objective_at,  # noqa: E402
                               random_qcqp, random_quad_boxes)
from minotaur_amd.problem import BINARY, CONTINUOUS, INTEGER  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
CAP = 128


def dump(name, qp, LB, UB, incumbent, qt):
    rows = oracle.ref_quad_root_rows(qp)
    r = oracle.ref_quad_fbbt(qp, LB, UB, incumbent, qt, rows, CAP)
    assert int(r.nmods.max(initial=0)) <= CAP, name
    np.savez_compressed(
        os.path.join(OUT, f'quad_{name}.npz'),
        **{k: getattr(qp, k) for k in _ARRAYS}, nv0=qp.nv0, has_obj=int(qp.has_obj),
        obj_const=qp.obj_const, name=qp.name,
        lb_in=LB, ub_in=UB, rows_in=rows, qt=int(qt),
        incumbent=np.float64(math.nan if incumbent is None else incumbent),
        lb_out=r.lb, ub_out=r.ub, rows_out=r.rows, infeas=r.infeas, nmods=r.nmods,
        mod_kind=r.kind.astype(np.int8), mod_idx=r.idx.astype(np.int16), mod_v1=r.v1,
        mod_v2=r.v2)
    print(f'{name:22s} nv={qp.nv:3d} B={LB.shape[0]:4d} qt={qt} infeas={int(r.infeas.sum()):4d} '
          f'mean nmods={r.nmods.mean():6.2f} max={int(r.nmods.max(initial=0)):3d} '
          f'ref {1e6 * r.seconds / max(1, LB.shape[0]):.1f} us/node')


def micro():
    """Hand-built cases: one square, one bilinear, a univariate row
    a x^2 + b x, a pure-square row (the :1852 branch), zero-width and
    sign-changing boxes."""
    C = CONTINUOUS
    vtype = [C, C, C, INTEGER]
    vlb = [-2.0, 1.0, -3.0, -2.0]
    vub = [3.0, 4.0, 2.0, 5.0]
    funcs = [
        ({0: 1.0}, {(0, 1): 1.0}),                  # x0*x1 + x0 (Bilinear: no QT)
        ({2: -1.5, 1: 0.5}, {(2, 2): 2.0}),         # 2 x2^2 - 1.5 x2 + 0.5 x1
        ({3: 1.0}, {(0, 0): -1.0, (3, 3): 0.5}),    # -x0^2 + 0.5 x3^2 + x3
        ({1: 2.0}, {(1, 1): 1.0, (0, 2): -1.0}),    # x1^2 + 2 x1 - x0 x2
    ]
    clb = [-math.inf, -1.0, -4.0, 2.0]
    cub = [6.0, 3.0, math.inf, 12.0]
    obj = ({0: 1.0, 2: -2.0}, {(0, 0): 1.0, (2, 2): 0.5})
    return from_functions('micro', vtype, vlb, vub, funcs, clb, cub, obj=obj, obj_const=0.5)


def main():
    qp = micro()
    LB, UB = random_quad_boxes(qp, 96, 11, edge=True)
    LB[0], UB[0] = qp.vlb, qp.vub                      # root box
    for qt in (1, 0):
        dump(f'micro_qt{qt}', qp, LB, UB, None, qt)
    dump('micro_inc', qp, LB, UB, 1.0, 1)
    for s in range(6):
        qp = random_qcqp(s, nv0=10 + 2 * s, ncon=4 + s)
        LB, UB = random_quad_boxes(qp, 128, 100 + s, edge=(s % 2 == 1))
        x = 0.5 * (qp.vlb[:qp.nv0] + qp.vub[:qp.nv0])
        inc = objective_at(qp, x) if s % 3 == 2 else None
        dump(f'qcqp{s}', qp, LB, UB, inc, 1 if s % 3 != 1 else 0)
    qp = random_qcqp(42, nv0=14, ncon=8, aux_bounds='free')
    LB, UB = random_quad_boxes(qp, 128, 7, edge=True)
    dump('qcqp_freeaux', qp, LB, UB, None, 1)
    dump('qcqp_freeaux_qt0', qp, LB, UB, None, 0)


if __name__ == '__main__':
    main()
