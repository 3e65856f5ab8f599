"""Config 1 (BASELINE configs[0]: simple-bnb on test_instances/nvs08.nl) on the
GPU, end to end, on its outer-approximation LP (minotaur_amd/instances/
nvs08_oa.npz, built from the file by the .nl reader; see
minotaur_amd.problem.nvs08_oa):

* K1 node FBBT equals the reference's LinearHandler::presolveNode bit for
  bit (tests/golden/fbbt_nvs08_oa*.npz also run in test_fbbt_gpu.py);
* the K3P / K3 node LPs equal HiGHS within 1e-6 and the oracle pivot for
  pivot;
* the batched tree proves the HiGHS MILP optimum of the OA-LP (a lower
  bound on nvs08's MINLP optimum 23.4497) and evaluates the same tree as
  the CPU restatement oracle/bnb.py (rounds, nodes, decisions).
"""
import math
import os

import numpy as np
import pytest

import oracle
from golden_io import assert_lp_matches, bits_equal, load_fbbt, load_lp
from minotaur_amd import bnb
from minotaur_amd.problem import LinProblem

pytestmark = pytest.mark.gpu

INST = os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd', 'instances')


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize('name', ['nvs08_oa', 'nvs08_oa_inc20'])
def test_nvs08_fbbt_bit_exact_vs_reference(ctx, name):
    p, g = load_fbbt(name)
    ctx.load(p)
    r = ctx.fbbt(g['lb_in'], g['ub_in'],
                 math.inf if g['incumbent'] is None else g['incumbent'], mod_cap=g['mod_cap'])
    assert bits_equal(r.lb, g['lb_out']) and bits_equal(r.ub, g['ub_out'])
    assert np.array_equal(r.infeasible, g['infeas']) and np.array_equal(r.nmods, g['nmods'])


def test_nvs08_lp_vs_highs_and_oracle(ctx):
    p, g = load_lp('nvs08_oa')
    ctx.load(p)
    r = ctx.lp_solve(g['lb'], g['ub'])                     # slack basis: K3
    assert_lp_matches(r.status, r.obj, g)
    so, oo, io, _ = oracle.dual_simplex(p, g['lb'], g['ub'])
    assert np.array_equal(r.status, so) and np.array_equal(r.iters, io)
    st0, _, _, _, _, ows = oracle.dual_simplex_root(p)
    from minotaur_amd.runtime import WarmStart
    ws = WarmStart(ows.head, ows.st, ows.d, np.ascontiguousarray(ows.binv.T))
    w = ctx.lp_solve(g['lb'], g['ub'], ws)                 # shared root basis: K3P
    assert_lp_matches(w.status, w.obj, g)
    so, oo, io, _ = oracle.dual_simplex(p, g['lb'], g['ub'], ows, pfi=ctx.oracle_pfi())
    assert np.array_equal(w.status, so) and np.array_equal(w.iters, io)


@pytest.mark.parametrize('batch', [1, 16, 1024])
def test_nvs08_tree_proves_highs_optimum(ctx, batch):
    from bnb import CpuBnbContext
    p = LinProblem.load(os.path.join(INST, 'nvs08_oa.npz'))
    hs, hobj = oracle.highs_milp(p)
    assert hs == 0 and hobj <= 23.4497 + 1e-4
    ctx.load(p)
    og, xg, sg, _ = bnb.solve(ctx, batch=batch, capacity=1 << 16)
    assert sg.open == 0 and sg.ndec[4] == 0
    assert abs(og - hobj) <= 1e-6 * max(1.0, abs(hobj))
    assert abs(xg[1] - round(xg[1])) <= 1e-6 and abs(xg[2] - round(xg[2])) <= 1e-6
    oc, _, sc, _ = bnb.solve(CpuBnbContext(p, ctx.oracle_pfi()), batch=batch, capacity=1 << 16)
    assert (sg.rounds, sg.nodes, list(sg.ndec)) == (sc.rounds, sc.nodes, list(sc.ndec))
    assert abs(og - oc) <= 1e-9 * max(1.0, abs(oc))
