"""GPU: checkpoint / resume of the batched tree's open pool in Minotaur's
Serializer format (bnb.checkpoint / bnb.restore over mgpu_bnb_export /
mgpu_bnb_import and mgpu_node_serialize / mgpu_node_deserialize, whose bytes
equal the reference's own Serializer::writeNode: tests/test_serial_cpu.py).
SURVEY §5 names the node wire format as the checkpoint-able open-node list.
Config 2's tls4-OA tree is interrupted after a few rounds, its open nodes are
written as writeNode records, and both the interrupted pool and a fresh tree
restored from the bytes prove the optimum 3.2 (HiGHS's), depth-first and
best-first."""
import math
import os

import pytest

from minotaur_amd import bnb, runtime
from minotaur_amd.problem import LinProblem

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


@pytest.fixture(scope='module')
def ctx():
    from minotaur_amd.runtime import Context
    c = Context(0)
    yield c
    c.close()


def _finish(ctx, batch):
    for _ in range(100000):
        st = ctx.bnb_round(batch)
        if st.open == 0:
            break
    assert st.open == 0
    return ctx.bnb_best()[0]


@pytest.mark.parametrize('order', [0, 1])
def test_checkpoint_resume_in_the_reference_format(ctx, order):
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx.load(p)
    cap = 1 << 18
    ctx.bnb_config(order, 1)
    ctx.bnb_brancher(0)
    ctx.bnb_growth(0)
    ctx.bnb_init(cap)
    for _ in range(4):
        st = ctx.bnb_round(512)
    open0, _ = ctx.bnb_count()
    assert open0 > 0
    inc, _ = ctx.bnb_best()
    data = bnb.checkpoint(ctx)
    ids, nlb, L, U = runtime.deserialize_nodes(data, p.vlb, p.vub)
    assert len(ids) == open0 and ctx.bnb_count()[0] == open0   # the pool put back
    assert all(math.isfinite(v) for v in nlb)
    obj_a = _finish(ctx, 4096)                                  # the interrupted pool
    bnb.restore(ctx, data, cap, incumbent=inc)                  # a fresh tree from the bytes
    assert ctx.bnb_count()[0] == open0
    obj_b = _finish(ctx, 4096)
    for obj in (obj_a, obj_b):
        assert abs(obj - 3.2) <= 1e-6 * 3.2
