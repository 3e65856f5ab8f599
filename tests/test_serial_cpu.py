"""CPU: open nodes in Minotaur's Serializer wire format (mgpu_node_serialize /
mgpu_node_deserialize, minotaur_amd/csrc/serial.cpp) against the reference's
own Serializer::writeNode and DeSerializer::readNode (src/base/Serializer.cpp:
26-191, compiled into oracle/_ref/libminotaur_hip_integ.so; integ_driver.cpp
integ_serialize_path / integ_deserialize_node).

The reference serializes a node from its path: the relaxation mods of every
ancestor's Branch and of every ancestor node, merged per (variable, bound
side) keeping the first old and the last new value.  The batched pool keeps
the node's box; the box against the root box gives the same merged entries.
Paths are random (seeded): branchings and node-level (presolve) mods, the same
bound tightened several times, both bound sides.  Bar: identical bytes, and
both deserializers give back the node's box, id and lower bound."""
import ctypes
import os

import numpy as np
import pytest

from minotaur_amd import runtime


@pytest.fixture(scope='module')
def integ():
    from test_simplex_cuts_cpu import LIB, load_integ
    if not os.path.exists(LIB):
        pytest.skip("integration library not built (needs /root/reference at build time)")
    lib = load_integ()
    P = ctypes.c_void_p
    lib.integ_serialize_path.restype = ctypes.c_long
    lib.integ_serialize_path.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, P, P, P,
                                         ctypes.c_uint, ctypes.c_double, P, ctypes.c_long]
    lib.integ_deserialize_node.restype = ctypes.c_int
    lib.integ_deserialize_node.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, P, P, P]
    return lib


def random_path(seed, n=12, steps=20, root=None):
    """Root box (or the given one), a path of strict tightenings (kind 0
    branch / 1 node mod), the node's final box."""
    rng = np.random.default_rng(seed)
    rl = np.where(rng.random(n) < 0.5, 0.0, -5.0)
    ru = rl + 10.0
    if root is not None:
        rl, ru = root
    lb, ub = rl.copy(), ru.copy()
    kind, var, lu, val = [], [], [], []
    for _ in range(steps):
        j = int(rng.integers(n))
        side = int(rng.integers(2))
        lo, hi = lb[j], ub[j]
        v = lo + (hi - lo) * rng.uniform(0.1, 0.9)
        if side == 0:
            lb[j] = v
        else:
            ub[j] = v
        kind.append(int(rng.integers(2)))
        var.append(j)
        lu.append(side)
        val.append(v)
    arr = lambda a, t: np.ascontiguousarray(a, dtype=t)
    return (rl, ru, lb, ub, arr(kind, np.int32), arr(var, np.int32), arr(lu, np.int32),
            arr(val, np.float64))


def ref_bytes(integ, rl, ru, kind, var, lu, val, node_id, nlb):
    n = ctypes.c_int(rl.size)
    k = integ.integ_serialize_path(n, rl.ctypes.data, ru.ctypes.data, len(kind),
                                   kind.ctypes.data, var.ctypes.data, lu.ctypes.data,
                                   val.ctypes.data, node_id, nlb, None, 0)
    out = ctypes.create_string_buffer(k)
    k2 = integ.integ_serialize_path(n, rl.ctypes.data, ru.ctypes.data, len(kind),
                                    kind.ctypes.data, var.ctypes.data, lu.ctypes.data,
                                    val.ctypes.data, node_id, nlb, out, k)
    assert k2 == k
    return out.raw[:k]


@pytest.mark.parametrize('seed', range(12))
def test_bytes_equal_the_reference_serializer(integ, seed):
    rl, ru, lb, ub, kind, var, lu, val = random_path(seed, steps=4 + 3 * seed)
    node_id, nlb = 1000 + seed, -3.25 * seed
    ref = ref_bytes(integ, rl, ru, kind, var, lu, val, node_id, nlb)
    ours = runtime.serialize_nodes(rl, ru, lb[None], ub[None], [nlb], ids=[node_id])
    assert ours == ref
    # both deserializers give the node back
    ids, nb, L, U = runtime.deserialize_nodes(ref, rl, ru)
    assert ids.tolist() == [node_id] and nb.tolist() == [nlb]
    assert np.array_equal(L[0], lb) and np.array_equal(U[0], ub)
    i, v = ctypes.c_uint(0), ctypes.c_double(0.0)
    L2, U2 = np.empty(rl.size), np.empty(rl.size)
    buf = ctypes.create_string_buffer(ours, len(ours))
    cnt = integ.integ_deserialize_node(buf, len(ours), rl.size, rl.ctypes.data, ru.ctypes.data,
                                       ctypes.byref(i), ctypes.byref(v), L2.ctypes.data,
                                       U2.ctypes.data)
    assert cnt == int(np.count_nonzero(lb != rl) + np.count_nonzero(ub != ru))
    assert (i.value, v.value) == (node_id, nlb)
    assert np.array_equal(L2, lb) and np.array_equal(U2, ub)


def test_root_node_and_node_streams(integ):
    """A node without mods (the root: k = 0) and several nodes in one stream,
    read back in order."""
    rl, ru = np.zeros(5), np.full(5, 3.0)
    ref = ref_bytes(integ, rl, ru, *(np.zeros(0, t) for t in (np.int32,) * 3 + (np.float64,)),
                    7, 0.5)
    assert ref == runtime.serialize_nodes(rl, ru, rl[None], ru[None], [0.5], ids=[7])
    assert len(ref) == 4 + 8 + 8
    paths = [random_path(s, n=5, steps=2 + s, root=(rl, ru)) for s in range(5)]
    L = np.array([q[2] for q in paths])
    U = np.array([q[3] for q in paths])
    ref = b''.join(ref_bytes(integ, rl, ru, *q[4:], s, float(s)) for s, q in enumerate(paths))
    ours = runtime.serialize_nodes(rl, ru, L, U, np.arange(5, dtype=float))
    assert ours == ref
    ids, nb, L2, U2 = runtime.deserialize_nodes(ref, rl, ru)
    assert ids.tolist() == list(range(5)) and nb.tolist() == [0.0, 1.0, 2.0, 3.0, 4.0]
    assert np.array_equal(L2, L) and np.array_equal(U2, U)


def test_malformed_input_is_refused():
    rl, ru = np.zeros(4), np.ones(4)
    lb, ub = rl.copy(), ru.copy()
    lb[2] = 0.5
    good = runtime.serialize_nodes(rl, ru, lb[None], ub[None], [0.0])
    with pytest.raises(runtime.MgpuError):
        runtime.deserialize_nodes(good[:-3], rl, ru)           # truncated entry
    bad = bytearray(good)
    bad[20:24] = (9).to_bytes(4, 'little')                     # variable 9 of 4
    with pytest.raises(runtime.MgpuError):
        runtime.deserialize_nodes(bytes(bad), rl, ru)
    bad = bytearray(good)
    bad[24:26] = (2).to_bytes(2, 'little')                     # bound side 2
    with pytest.raises(runtime.MgpuError):
        runtime.deserialize_nodes(bytes(bad), rl, ru)
