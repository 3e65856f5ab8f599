"""CPU: the plain-C oracle reproduces the reference's own FBBT outputs
(golden vectors generated from oracle/_ref, i.e. Minotaur's LinearHandler
compiled from /root/reference) bit for bit, mod log included."""
import numpy as np
import pytest

import oracle
from golden_io import assert_mods_equal, bits_equal, cases, load_fbbt


@pytest.mark.parametrize('name', cases())
def test_oracle_matches_reference_golden(name):
    p, g = load_fbbt(name)
    r = oracle.linear_fbbt(p, g['lb_in'], g['ub_in'], g['incumbent'], g['mod_cap'])
    assert bits_equal(r.lb, g['lb_out'])
    assert bits_equal(r.ub, g['ub_out'])
    assert np.array_equal(r.infeas, g['infeas'])
    assert np.array_equal(r.nmods, g['nmods'])
    assert_mods_equal(r.nmods, r.mod_var, r.mod_lu, r.mod_val, g, g['mod_cap'])


def test_oracle_threads_agree():
    p, g = load_fbbt('tls4_noinc')
    a = oracle.linear_fbbt(p, g['lb_in'], g['ub_in'], None, 0, nthreads=1)
    b = oracle.linear_fbbt(p, g['lb_in'], g['ub_in'], None, 0, nthreads=4)
    assert bits_equal(a.lb, b.lb) and bits_equal(a.ub, b.ub)


@pytest.mark.skipif(not oracle.have_ref(), reason="reference build not present")
def test_oracle_matches_reference_live():
    """When the reference library is built here, compare on fresh seeds."""
    from minotaur_amd.problem import random_boxes, random_problem
    for s in (11, 12, 13):
        p = random_problem(s, n=50, m=35)
        LB, UB = random_boxes(p, 64, 1000 + s)
        for inc in (None, 1.0):
            r = oracle.ref_linear_fbbt(p, LB, UB, inc, 256)
            o = oracle.linear_fbbt(p, LB, UB, inc, 256)
            assert bits_equal(r.lb, o.lb) and bits_equal(r.ub, o.ub)
            assert np.array_equal(r.infeas, o.infeas)
            assert np.array_equal(r.nmods, o.nmods)
