"""ctypes binding of the C ABI in include/mgpu.h (libmgpu.so, built in-tree).

The product path has no CPU fallback: if ``libmgpu.so`` is missing or no HIP
device is visible, every call raises ``MgpuError``.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MGPU_LIB overrides the library (diagnostic builds in tools/ only)
LIB_PATH = os.environ.get('MGPU_LIB', os.path.join(HERE, 'libmgpu.so'))

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double

LP_PFI_MAX = 32  # MGPU_LP_PFI_MAX (include/mgpu.h): K3P's default eta-file cap
LP_PFI_BIG = 48  # MGPU_LP_PFI_BIG: the largest cap (the 48-eta build)
LP_PFI_WIDE_MAX = 32  # MGPU_LP_PFI_WIDE_MAX: K3PW eta-file cap
PATH_MAX = 32  # MGPU_PATH_MAX: columns per basis warm start
PATH_INHERIT = 32  # the batched tree's largest basis difference handed to children (warm mode 2)

# Every entry point declared in include/mgpu.h (checked by the CPU tests).
EXPORTS = [
    'mgpu_create', 'mgpu_destroy', 'mgpu_last_error', 'mgpu_set_stream',
    'mgpu_get_stream', 'mgpu_sync', 'mgpu_load_lp', 'mgpu_fbbt', 'mgpu_fbbt_dev',
    'mgpu_set_fbbt_variant', 'mgpu_set_lp_variant', 'mgpu_set_lp_pfi', 'mgpu_last_kernel_ms',
    'mgpu_set_qp_ktime',
    'mgpu_lp_solve', 'mgpu_lp_solve_dev',
    'mgpu_node_decide_dev', 'mgpu_load_quad', 'mgpu_quad_rows', 'mgpu_quad_fbbt',
    'mgpu_quad_fbbt_dev', 'mgpu_lp_bound', 'mgpu_lp_bound_dev', 'mgpu_bnb_init',
    'mgpu_bnb_round', 'mgpu_bnb_best', 'mgpu_bnb_shard', 'mgpu_bnb_config', 'mgpu_bnb_export',
    'mgpu_bnb_import', 'mgpu_strong_branch',
    'mgpu_strong_branch_dev', 'mgpu_load_qp', 'mgpu_qp_solve', 'mgpu_qp_solve_dev',
    'mgpu_set_node_rows', 'mgpu_lp_solve_rows', 'mgpu_lp_solve_rows_dev', 'mgpu_bnb_brancher',
    'mgpu_bnb_relaxation',
    'mgpu_lp_refactor', 'mgpu_set_lp_pfi_wide', 'mgpu_lp_pfi_cap', 'mgpu_lp_solve_path',
    'mgpu_lp_solve_path_dev', 'mgpu_bnb_guided_dive', 'mgpu_ws_alloc', 'mgpu_ws_free',
    'mgpu_ws_read', 'mgpu_ws_write', 'mgpu_lp_solve1', 'mgpu_bnb_pick', 'mgpu_bnb_export_dev',
    'mgpu_bnb_import_dev', 'mgpu_bnb_row_width', 'mgpu_bnb_count', 'mgpu_glob_config', 'mgpu_glob_init', 'mgpu_glob_round', 'mgpu_glob_best',
    'mgpu_comm_unique_id', 'mgpu_comm_init', 'mgpu_comm_init_host', 'mgpu_comm_info',
    'mgpu_allreduce_f64', 'mgpu_allreduce_min', 'mgpu_round_reduce', 'mgpu_allgather_f64',
    'mgpu_alltoall_rows_dev', 'mgpu_lb_deal', 'mgpu_bnb_rebalance', 'mgpu_alloc_stats',
    'mgpu_bnb_growth', 'mgpu_set_sb_chain', 'mgpu_glob_brancher', 'mgpu_glob_lp_log',
    'mgpu_node_serialize', 'mgpu_node_deserialize',
]

COMM_ID_BYTES = 128            # MGPU_COMM_ID_BYTES
OP_SUM, OP_MIN, OP_MAX = 0, 1, 2   # MGPU_OP_*

# mgpu_host_transport's callbacks (include/mgpu.h)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.c_int, ctypes.c_int)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.c_int, ctypes.POINTER(ctypes.c_double))
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_int32), ctypes.c_int)


class HostTransport(ctypes.Structure):
    """mgpu_host_transport (include/mgpu.h)."""
    _fields_ = [('user', ctypes.c_void_p), ('allreduce', ALLREDUCE_FN),
                ('allgather', ALLGATHER_FN), ('alltoallv', ALLTOALLV_FN)]


class BnbStats(ctypes.Structure):
    """mgpu_bnb_stats (include/mgpu.h)."""
    _fields_ = [('rounds', ctypes.c_longlong), ('nodes', ctypes.c_longlong),
                ('ndec', ctypes.c_longlong * 5), ('open', ctypes.c_int),
                ('last_batch', ctypes.c_int), ('incumbent', ctypes.c_double),
                ('pruned', ctypes.c_longlong), ('lps', ctypes.c_longlong),
                ('pivots', ctypes.c_longlong), ('sb_lps', ctypes.c_longlong),
                ('sb_pivots', ctypes.c_longlong), ('sb_pruned', ctypes.c_longlong),
                ('sb_modified', ctypes.c_longlong), ('pfi_pivots', ctypes.c_longlong)]

class GlobStats(ctypes.Structure):
    """mgpu_glob_stats (include/mgpu.h)."""
    _fields_ = [('rounds', ctypes.c_longlong), ('nodes', ctypes.c_longlong),
                ('ndec', ctypes.c_longlong * 6), ('lps', ctypes.c_longlong),
                ('pivots', ctypes.c_longlong), ('br_int', ctypes.c_longlong),
                ('br_cont', ctypes.c_longlong), ('open', ctypes.c_int),
                ('last_batch', ctypes.c_int), ('incumbent', ctypes.c_double),
                ('cuts', ctypes.c_longlong), ('resolves', ctypes.c_longlong),
                ('obbt_lps', ctypes.c_longlong), ('sb_lps', ctypes.c_longlong)]


_lib = None


class MgpuError(RuntimeError):
    pass


def load_library():
    """Load libmgpu.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MgpuError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                        "(there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If
    # torch is importable, load it first so libmgpu.so binds to that same
    # runtime (same soname) and device pointers / streams are shared.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    lib.mgpu_create.argtypes = [_I, ctypes.POINTER(_P)]
    lib.mgpu_destroy.argtypes = [_P]
    lib.mgpu_last_error.argtypes = [_P]
    lib.mgpu_last_error.restype = ctypes.c_char_p
    lib.mgpu_set_stream.argtypes = [_P, _P]
    lib.mgpu_get_stream.argtypes = [_P]
    lib.mgpu_get_stream.restype = _P
    lib.mgpu_sync.argtypes = [_P]
    lib.mgpu_load_lp.argtypes = [_P, _I, _I] + [_P] * 9 + [_D]
    lib.mgpu_fbbt.argtypes = [_P, _I, _P, _P, _D, _P, _P, _P, _P, _I, _P, _P, _P]
    lib.mgpu_fbbt_dev.argtypes = [_P, _I, _P, _P, _D, _P, _P, _P, _P, _I, _P, _P, _P]
    lib.mgpu_set_fbbt_variant.argtypes = [_P, _I]
    lib.mgpu_set_lp_variant.argtypes = [_P, _I]
    lib.mgpu_set_lp_pfi.argtypes = [_P, _I]
    lib.mgpu_set_lp_pfi_wide.argtypes = [_P, _I]
    lib.mgpu_lp_pfi_cap.argtypes = [_P]
    lib.mgpu_lp_solve.argtypes = [_P, _I] + [_P] * 7 + [_I, _I] + [_P] * 8
    lib.mgpu_lp_solve_dev.argtypes = [_P, _I] + [_P] * 7 + [_I, _I] + [_P] * 8
    lib.mgpu_node_decide_dev.argtypes = [_P, _I] + [_P] * 4 + [_D] * 5 + [_P] * 3
    lib.mgpu_load_quad.argtypes = ([_P, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _I]
                                   + [_P] * 9 + [_I, _D])
    lib.mgpu_quad_rows.argtypes = [_P, _P, _P, _P, _P]
    lib.mgpu_quad_fbbt.argtypes = [_P, _I, _P, _P, _D, _I, _P, _I] + [_P] * 5 + [_I] + [_P] * 4
    lib.mgpu_quad_fbbt_dev.argtypes = ([_P, _I, _P, _P, _D, _I, _P, _I] + [_P] * 5 + [_I]
                                       + [_P] * 4)
    lib.mgpu_lp_bound.argtypes = [_P, _I] + [_P] * 7 + [_I] + [_P] * 4
    lib.mgpu_lp_bound_dev.argtypes = [_P, _I] + [_P] * 7 + [_I] + [_P] * 4
    lib.mgpu_bnb_init.argtypes = [_P, _I, _P, _P, _D]
    lib.mgpu_bnb_config.argtypes = [_P, _I, _I]
    lib.mgpu_bnb_brancher.argtypes = [_P, _I]
    lib.mgpu_bnb_growth.argtypes = [_P, _I]
    lib.mgpu_set_sb_chain.argtypes = [_P, _I]
    lib.mgpu_glob_brancher.argtypes = [_P, _I]
    lib.mgpu_glob_lp_log.argtypes = [_P, _I, _P, _P, _P]
    lib.mgpu_node_serialize.argtypes = [ctypes.c_uint32, _D, _I, _P, _P, _P, _P, _P,
                                        ctypes.c_size_t, _P]
    lib.mgpu_node_deserialize.argtypes = [_P, ctypes.c_size_t, _I, _P, _P, _P, _P, _P, _P, _P]
    lib.mgpu_bnb_relaxation.argtypes = [_P, _I]
    lib.mgpu_bnb_guided_dive.argtypes = [_P, _I]
    lib.mgpu_bnb_export.argtypes = [_P, _I, _P, _P, _P, _P, _P]
    lib.mgpu_bnb_import.argtypes = [_P, _I, _P, _P, _P, _P]
    lib.mgpu_bnb_pick.argtypes = [_P, _I, _P, _P]
    lib.mgpu_bnb_export_dev.argtypes = [_P, _I, _P, _P]
    lib.mgpu_bnb_import_dev.argtypes = [_P, _I, _P]
    lib.mgpu_bnb_row_width.argtypes = [_P]
    lib.mgpu_bnb_count.argtypes = [_P, _P, _P]
    lib.mgpu_alloc_stats.argtypes = [_P, _P]
    lib.mgpu_comm_unique_id.argtypes = [_P]
    lib.mgpu_comm_init.argtypes = [_P, _I, _I, _P]
    lib.mgpu_comm_init_host.argtypes = [_P, _I, _I, ctypes.POINTER(HostTransport)]
    lib.mgpu_comm_info.argtypes = [_P, _P, _P]
    lib.mgpu_allreduce_f64.argtypes = [_P, _P, _I, _I]
    lib.mgpu_allreduce_min.argtypes = [_P, _P]
    lib.mgpu_round_reduce.argtypes = [_P, _D, _D, _I, _P]
    lib.mgpu_allgather_f64.argtypes = [_P, _P, _I, _P]
    lib.mgpu_alltoall_rows_dev.argtypes = [_P, _I, _P, _P, _P, _P]
    lib.mgpu_lb_deal.argtypes = [_I, _I, _P, _P, _P, _P]
    lib.mgpu_bnb_rebalance.argtypes = [_P, _I, _P, _P, _P, _P, _P, _P]
    lib.mgpu_glob_config.argtypes = [_P, _I, _I, _I, _I, _I]
    lib.mgpu_glob_init.argtypes = [_P, _I, _D]
    lib.mgpu_glob_round.argtypes = [_P, _I, _D, ctypes.POINTER(GlobStats)]
    lib.mgpu_glob_best.argtypes = [_P, _P, _P]
    lib.mgpu_bnb_round.argtypes = [_P, _I, _D, ctypes.POINTER(BnbStats)]
    lib.mgpu_bnb_best.argtypes = [_P, _P, _P]
    lib.mgpu_bnb_shard.argtypes = [_P, _I, _I, _P]
    lib.mgpu_strong_branch.argtypes = [_P, _P, _P, _I] + [_P] * 6 + [_I] + [_P] * 3
    lib.mgpu_strong_branch_dev.argtypes = [_P, _P, _P, _I] + [_P] * 6 + [_I] + [_P] * 5
    lib.mgpu_load_qp.argtypes = [_P, _I, _I, _P, _P, _D, _P, _P]
    lib.mgpu_qp_solve.argtypes = [_P, _I, _P, _P, _I, _P, _P, _P, _P]
    lib.mgpu_qp_solve_dev.argtypes = [_P, _I, _P, _P, _I, _P, _P, _P, _P]
    lib.mgpu_set_node_rows.argtypes = [_P, _I, _I, _P, _P, _I, _P, _P, _P]
    lib.mgpu_lp_refactor.argtypes = [_P] + [_P] * 7
    lib.mgpu_lp_solve_rows.argtypes = [_P, _I] + [_P] * 6 + [_I, _I] + [_P] * 5
    lib.mgpu_lp_solve_rows_dev.argtypes = [_P, _I] + [_P] * 6 + [_I, _I] + [_P] * 5
    lib.mgpu_lp_solve_path.argtypes = [_P, _I] + [_P] * 9 + [_I, _I] + [_P] * 7
    lib.mgpu_lp_solve_path_dev.argtypes = [_P, _I] + [_P] * 10 + [_I, _I] + [_P] * 7
    lib.mgpu_ws_alloc.argtypes = [_P, ctypes.POINTER(_I)]
    lib.mgpu_ws_free.argtypes = [_P, _I]
    lib.mgpu_ws_read.argtypes = [_P, _I, _P, _P, _P, _P]
    lib.mgpu_ws_write.argtypes = [_P, _I, _P, _P, _P, _P]
    lib.mgpu_lp_solve1.argtypes = [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P]
    lib.mgpu_set_qp_ktime.argtypes = [_P, _I]
    lib.mgpu_last_kernel_ms.argtypes = [_P, ctypes.c_char_p]
    lib.mgpu_last_kernel_ms.restype = _D
    for name in EXPORTS:
        getattr(lib, name).restype = getattr(lib, name).restype or _I
    _lib = lib
    return lib


def _np(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _hp(a):
    return None if a is None else a.ctypes.data_as(_P)


def _dp(t):
    """Device pointer of a torch CUDA tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def comm_unique_id() -> bytes:
    """mgpu_comm_unique_id: an RCCL unique id for mgpu_comm_init (one rank
    makes it, the launcher hands it to the others)."""
    lib = load_library()
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    rc = lib.mgpu_comm_unique_id(buf)
    if rc != 0:
        raise MgpuError(f"mgpu_comm_unique_id failed rc={rc}")
    return buf.raw


def alloc_stats():
    """mgpu_alloc_stats: (device allocations, bytes) the engine made so far
    in this process."""
    lib = load_library()
    n, b = ctypes.c_longlong(0), ctypes.c_longlong(0)
    lib.mgpu_alloc_stats(ctypes.byref(n), ctypes.byref(b))
    return n.value, b.value


def lb_deal(world, S, lbs):
    """mgpu_lb_deal (host only, no device): LoadBalance_'s deal of the
    rank-major bounds lbs [world * S] -> (owner, local, receiver) arrays."""
    lib = load_library()
    v = np.ascontiguousarray(lbs, dtype=np.float64).reshape(-1)
    if v.size != world * S:
        raise MgpuError(f"lb_deal: {v.size} bounds for world {world} x S {S}")
    o, loc, r = (np.empty(max(v.size, 1), dtype=np.int32) for _ in range(3))
    nd = lib.mgpu_lb_deal(int(world), int(S), _hp(v), _hp(o), _hp(loc), _hp(r))
    if nd < 0:
        raise MgpuError(f"mgpu_lb_deal failed rc={nd}")
    return o[:nd].copy(), loc[:nd].copy(), r[:nd].copy()


def serialize_nodes(root_lb, root_ub, lb, ub, nlb, ids=None) -> bytes:
    """mgpu_node_serialize over k nodes (boxes lb / ub [k][n], lower bounds
    nlb [k], ids default 0..k-1): the concatenated Serializer::writeNode
    records (src/base/Serializer.cpp:26-112), in node order."""
    lib = load_library()
    rl, ru = _np(root_lb, np.float64), _np(root_ub, np.float64)
    L = _np(lb, np.float64).reshape(-1, rl.size)
    U = _np(ub, np.float64).reshape(-1, rl.size)
    nb = _np(nlb, np.float64).reshape(-1)
    k, n = L.shape
    ids = np.arange(k, dtype=np.uint32) if ids is None else _np(ids, np.uint32)
    out = []
    ln = ctypes.c_size_t(0)
    for b in range(k):
        args = (int(ids[b]), float(nb[b]), n, _hp(rl), _hp(ru), _hp(L[b]), _hp(U[b]))
        if lib.mgpu_node_serialize(*args, None, 0, ctypes.byref(ln)) != 0:
            raise MgpuError(f"mgpu_node_serialize failed on node {b}")
        buf = ctypes.create_string_buffer(ln.value)
        if lib.mgpu_node_serialize(*args, buf, ln.value, ctypes.byref(ln)) != 0:
            raise MgpuError(f"mgpu_node_serialize failed on node {b}")
        out.append(buf.raw[:ln.value])
    return b''.join(out)


def deserialize_nodes(data: bytes, root_lb, root_ub):
    """mgpu_node_deserialize until data is used up (DeSerializer::readNode,
    src/base/Serializer.cpp:130-191) -> (ids, lower bounds, lb, ub)."""
    lib = load_library()
    rl, ru = _np(root_lb, np.float64), _np(root_ub, np.float64)
    n = rl.size
    buf = ctypes.create_string_buffer(data, len(data))
    base = ctypes.addressof(buf)
    ids, nlb, L, U = [], [], [], []
    at = 0
    while at < len(data):
        i, v = ctypes.c_uint32(0), ctypes.c_double(0.0)
        lo, hi = np.empty(n), np.empty(n)
        used = ctypes.c_size_t(0)
        if lib.mgpu_node_deserialize(ctypes.c_void_p(base + at), len(data) - at, n, _hp(rl),
                                     _hp(ru), ctypes.byref(i), ctypes.byref(v), _hp(lo), _hp(hi),
                                     ctypes.byref(used)) != 0:
            raise MgpuError(f"mgpu_node_deserialize failed at byte {at}")
        ids.append(i.value)
        nlb.append(v.value)
        L.append(lo)
        U.append(hi)
        at += used.value
    return (np.array(ids, dtype=np.uint32), np.array(nlb), np.array(L).reshape(-1, n),
            np.array(U).reshape(-1, n))


class FbbtOut:
    def __init__(self, lb, ub, infeasible, nmods, mod_var=None, mod_lu=None,
                 mod_val=None):
        self.lb, self.ub, self.infeasible, self.nmods = lb, ub, infeasible, nmods
        self.mod_var, self.mod_lu, self.mod_val = mod_var, mod_lu, mod_val


class QuadOut:
    def __init__(self, lb, ub, rows, infeasible, nmods, kind=None, idx=None, v1=None,
                 v2=None):
        self.lb, self.ub, self.rows, self.infeasible, self.nmods = lb, ub, rows, infeasible, nmods
        self.kind, self.idx, self.v1, self.v2 = kind, idx, v1, v2


class WarmStart:
    """LP basis (getWarmStartCopy equivalent): basic column per row [m],
    column status [n+m] (0 lb, 1 ub, 2 free, 3 basic), reduced costs [n+m]
    and the dense basis inverse stored COLUMN-major: binv[k, i] = (B^-1)[i, k]
    (the ABI layout; ``binv_rows()`` gives (B^-1) itself).  Leading batch
    axis when per node."""

    def binv_rows(self):
        return np.swapaxes(np.asarray(self.binv), -1, -2)

    def __init__(self, head, st, d, binv):
        self.head, self.st, self.d, self.binv = head, st, d, binv

    def node(self, b):
        return WarmStart(self.head[b], self.st[b], self.d[b], self.binv[b])


class LpOut:
    def __init__(self, status, obj, iters, x=None, ws=None):
        self.status, self.obj, self.iters, self.x, self.ws = status, obj, iters, x, ws


class Context:
    """One engine context on one device (one per host thread)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _P()
        rc = self.lib.mgpu_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise MgpuError(f"mgpu_create(device={device}) failed rc={rc} "
                            "(no HIP device visible?)")
        self.h = h
        self.device = device
        self.problem = None

    def close(self):
        if getattr(self, 'h', None):
            self.lib.mgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.mgpu_last_error(self.h)
            raise MgpuError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")

    def set_stream(self, stream_ptr):
        """Run on an existing hipStream_t (e.g. torch.cuda.Stream().cuda_stream).
        0 is refused: the legacy null stream would not be ordered against
        work the engine queues on its own non-blocking stream."""
        if not stream_ptr:
            raise MgpuError("set_stream(0): pass a real stream (torch.cuda.Stream())")
        self._chk(self.lib.mgpu_set_stream(self.h, _P(stream_ptr)), 'mgpu_set_stream')

    def reset_stream(self):
        """Back to the context's own non-blocking stream."""
        self._chk(self.lib.mgpu_set_stream(self.h, None), 'mgpu_set_stream')

    def sync(self):
        self._chk(self.lib.mgpu_sync(self.h), 'mgpu_sync')

    def set_lp_variant(self, v: int):
        """0 auto, 1 K3 (m <= 64), 2 K3L (any m; one node per workgroup),
        3 K3P (product form; shared warm start only)."""
        self._chk(self.lib.mgpu_set_lp_variant(self.h, int(v)), 'mgpu_set_lp_variant')
        self.lp_variant = int(v)

    def set_lp_pfi(self, kmax: int):
        """K3P eta-file cap (0: auto mode never picks K3P)."""
        self._chk(self.lib.mgpu_set_lp_pfi(self.h, int(kmax)), 'mgpu_set_lp_pfi')
        self.lp_pfi = int(kmax)

    def set_lp_pfi_wide(self, kmax: int):
        """K3PW eta-file cap (64 < m <= 128; 0: auto mode never picks K3PW)."""
        self._chk(self.lib.mgpu_set_lp_pfi_wide(self.h, int(kmax)), 'mgpu_set_lp_pfi_wide')

    def oracle_pfi(self, shared_ws=True, want_ws=False):
        """The ``pfi`` argument under which oracle.dual_simplex / lp_bound
        restate what this context runs for such a batch (0 = dense K3/K3L):
        the eta-file cap of K3P / K3PW for the loaded problem
        (mgpu_lp_pfi_cap)."""
        if not shared_ws or want_ws:
            return 0
        k = self.lib.mgpu_lp_pfi_cap(self.h)
        if k < 0:
            raise MgpuError(f"mgpu_lp_pfi_cap failed ({k})")
        return int(k)

    def set_qp_ktime(self, on):
        """Per-kernel event timing of K5's iteration kernels (last_kernel_ms
        'qp_potrf' / 'qp_trsm' / 'qp_step')."""
        self._chk(self.lib.mgpu_set_qp_ktime(self.h, 1 if on else 0), 'mgpu_set_qp_ktime')

    def set_fbbt_variant(self, v: int):
        self._chk(self.lib.mgpu_set_fbbt_variant(self.h, int(v)), 'mgpu_set_fbbt_variant')

    def last_kernel_ms(self, which: str) -> float:
        return float(self.lib.mgpu_last_kernel_ms(self.h, which.encode()))

    # -- problem -----------------------------------------------------------
    def load(self, p):
        """mgpu_load_lp: OsiLPEngine::load equivalent for a LinProblem."""
        self._keep = [_np(p.rowptr, np.int32), _np(p.colidx, np.int32),
                      _np(p.val, np.float64), _np(p.rlo, np.float64),
                      _np(p.rhi, np.float64), _np(p.vlb, np.float64),
                      _np(p.vub, np.float64), _np(p.vtype, np.int32),
                      _np(p.obj, np.float64)]
        k = self._keep
        self._chk(self.lib.mgpu_load_lp(self.h, p.n, p.m, *[_hp(a) for a in k],
                                        float(p.obj_const)), 'mgpu_load_lp')
        self.problem = p

    def load_quad(self, qp):
        """mgpu_load_quad: QuadHandler registries + original quadratic
        functions of a minotaur_amd.quad.QuadProblem."""
        i32 = lambda a: _np(a, np.int32)
        f64 = lambda a: _np(a, np.float64)
        self._qkeep = k = dict(vtype=i32(qp.vtype), sq_x=i32(qp.sq_x), sq_y=i32(qp.sq_y),
                               bx0=i32(qp.bil_x0), bx1=i32(qp.bil_x1), by=i32(qp.bil_y),
                               lptr=i32(qp.lptr), lvar=i32(qp.lvar), lval=f64(qp.lval),
                               qptr=i32(qp.qptr), qv1=i32(qp.qv1), qv2=i32(qp.qv2),
                               qval=f64(qp.qval), clb=f64(qp.clb), cub=f64(qp.cub))
        self._chk(self.lib.mgpu_load_quad(
            self.h, qp.nv0, qp.nv, _hp(k['vtype']), qp.nsq, _hp(k['sq_x']), _hp(k['sq_y']),
            qp.nbil, _hp(k['bx0']), _hp(k['bx1']), _hp(k['by']), qp.ncon, _hp(k['lptr']),
            _hp(k['lvar']), _hp(k['lval']), _hp(k['qptr']), _hp(k['qv1']), _hp(k['qv2']),
            _hp(k['qval']), _hp(k['clb']), _hp(k['cub']), int(qp.has_obj),
            float(qp.obj_const)), 'mgpu_load_quad')
        self.quad = qp

    def quad_rows(self, lb=None, ub=None):
        """Secant/McCormick row state of QuadHandler::relax_ at a box."""
        qp = self.quad
        lb = _np(qp.vlb if lb is None else lb, np.float64)
        ub = _np(qp.vub if ub is None else ub, np.float64)
        R = ctypes.c_int(0)
        self._chk(self.lib.mgpu_quad_rows(self.h, None, None, None, ctypes.byref(R)),
                  'mgpu_quad_rows')
        rows = np.empty(R.value)
        self._chk(self.lib.mgpu_quad_rows(self.h, _hp(lb), _hp(ub), _hp(rows), None),
                  'mgpu_quad_rows')
        return rows

    def quad_fbbt(self, lb, ub, rows=None, incumbent=math.inf, qt=1, mod_cap=0):
        """QuadHandler::presolveNode over host boxes [B,nv] (synchronous).
        rows: [R] shared or [B,R] per node (default: root rows)."""
        qp = self.quad
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        B = lb.shape[0]
        rows = self.quad_rows() if rows is None else _np(rows, np.float64)
        shared = 1 if rows.ndim == 1 else 0
        olb = np.empty_like(lb)
        oub = np.empty_like(ub)
        orows = np.empty((B, qp.nrow_state))
        inf = np.zeros(B, dtype=np.int32)
        nm = np.zeros(B, dtype=np.int32)
        kind = idx = v1 = v2 = None
        if mod_cap > 0:
            kind = np.full((B, mod_cap), -1, dtype=np.int32)
            idx = np.full((B, mod_cap), -1, dtype=np.int32)
            v1 = np.zeros((B, mod_cap))
            v2 = np.zeros((B, mod_cap))
        self._chk(self.lib.mgpu_quad_fbbt(self.h, B, _hp(lb), _hp(ub), float(incumbent),
                                          int(qt), _hp(rows), shared, _hp(olb), _hp(oub),
                                          _hp(orows), _hp(inf), _hp(nm), int(mod_cap),
                                          _hp(kind), _hp(idx), _hp(v1), _hp(v2)),
                  'mgpu_quad_fbbt')
        return QuadOut(olb, oub, orows, inf, nm, kind, idx, v1, v2)

    def quad_fbbt_dev(self, lb, ub, rows, lb_out, ub_out, rows_out, infeasible, nmods,
                      incumbent=math.inf, qt=1, mod_kind=None, mod_idx=None, mod_v1=None,
                      mod_v2=None):
        """Torch CUDA tensors in/out, asynchronous on the context stream;
        rows 1-D = shared row state."""
        B = int(lb.shape[0])
        cap = int(mod_kind.shape[1]) if mod_kind is not None else 0
        shared = 1 if rows.dim() == 1 else 0
        self._chk(self.lib.mgpu_quad_fbbt_dev(
            self.h, B, _dp(lb), _dp(ub), float(incumbent), int(qt), _dp(rows), shared,
            _dp(lb_out), _dp(ub_out), _dp(rows_out), _dp(infeasible), _dp(nmods), cap,
            _dp(mod_kind), _dp(mod_idx), _dp(mod_v1), _dp(mod_v2)), 'mgpu_quad_fbbt_dev')

    # -- FBBT --------------------------------------------------------------
    def fbbt(self, lb, ub, incumbent=math.inf, mod_cap=0) -> FbbtOut:
        """Host arrays [B,n] in, tightened boxes out (synchronous)."""
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        B = lb.shape[0]
        olb = np.empty_like(lb)
        oub = np.empty_like(ub)
        inf = np.zeros(B, dtype=np.int32)
        nm = np.zeros(B, dtype=np.int32)
        mv = ml = mval = None
        if mod_cap > 0:
            mv = np.full((B, mod_cap), -1, dtype=np.int32)
            ml = np.full((B, mod_cap), -1, dtype=np.int32)
            mval = np.zeros((B, mod_cap))
        self._chk(self.lib.mgpu_fbbt(self.h, B, _hp(lb), _hp(ub), float(incumbent),
                                     _hp(olb), _hp(oub), _hp(inf), _hp(nm), int(mod_cap),
                                     _hp(mv), _hp(ml), _hp(mval)), 'mgpu_fbbt')
        return FbbtOut(olb, oub, inf, nm, mv, ml, mval)

    def fbbt_dev(self, lb, ub, lb_out, ub_out, infeasible, nmods,
                 incumbent=math.inf, mod_var=None, mod_lu=None, mod_val=None):
        """Torch CUDA tensors in/out, asynchronous on the context stream."""
        B = int(lb.shape[0])
        cap = int(mod_var.shape[1]) if mod_var is not None else 0
        self._chk(self.lib.mgpu_fbbt_dev(self.h, B, _dp(lb), _dp(ub), float(incumbent),
                                         _dp(lb_out), _dp(ub_out), _dp(infeasible),
                                         _dp(nmods), cap, _dp(mod_var), _dp(mod_lu),
                                         _dp(mod_val)), 'mgpu_fbbt_dev')

    # -- LP ------------------------------------------------------------------
    def lp_solve(self, lb, ub, ws=None, skip=None, iter_limit=0, want_x=False,
                 want_ws=False) -> LpOut:
        """Host arrays [B,n] in; per-node status/objective/iterations out.
        ``ws``: a WarmStart shared by all nodes (1-D arrays) or per node
        (leading batch axis); None = slack basis."""
        p = self.problem
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        B = lb.shape[0]
        n, m = p.n, p.m
        st = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros((B, n)) if want_x else None
        wo = None
        if want_ws:
            wo = WarmStart(np.zeros((B, m), np.int32), np.zeros((B, n + m), np.int8),
                           np.zeros((B, n + m)), np.zeros((B, m, m)))
        wh = wst = wd = wb = None
        shared = 1
        if ws is not None:
            wh = _np(ws.head, np.int32)
            wst = _np(ws.st, np.int8)
            wd = None if ws.d is None else _np(ws.d, np.float64)  # None: rebuilt
            wb = _np(ws.binv, np.float64)
            shared = 1 if wh.ndim == 1 else 0
        sk = None if skip is None else _np(skip, np.int32)
        self._chk(self.lib.mgpu_lp_solve(
            self.h, B, _hp(lb), _hp(ub), _hp(sk), _hp(wh), _hp(wst), _hp(wd), _hp(wb), shared,
            int(iter_limit), _hp(st), _hp(obj), _hp(it), _hp(x),
            _hp(wo.head) if wo else None, _hp(wo.st) if wo else None,
            _hp(wo.d) if wo else None, _hp(wo.binv) if wo else None), 'mgpu_lp_solve')
        return LpOut(st, obj, it, x, wo)

    # -- the single-LP route: device warm-start slots ------------------------
    def ws_alloc(self) -> int:
        s = _I(0)
        self._chk(self.lib.mgpu_ws_alloc(self.h, ctypes.byref(s)), 'mgpu_ws_alloc')
        return s.value

    def ws_free(self, slot):
        self._chk(self.lib.mgpu_ws_free(self.h, int(slot)), 'mgpu_ws_free')

    def ws_read(self, slot) -> WarmStart:
        p = self.problem
        n, m = p.n, p.m
        w = WarmStart(np.zeros(m, np.int32), np.zeros(n + m, np.int8), np.zeros(n + m),
                      np.zeros((m, m)))
        self._chk(self.lib.mgpu_ws_read(self.h, int(slot), _hp(w.head), _hp(w.st), _hp(w.d),
                                        _hp(w.binv)), 'mgpu_ws_read')
        return w

    def ws_write(self, slot, ws):
        d = None if ws.d is None else _np(ws.d, np.float64)
        self._chk(self.lib.mgpu_ws_write(self.h, int(slot), _hp(_np(ws.head, np.int32)),
                                         _hp(_np(ws.st, np.int8)), _hp(d),
                                         _hp(_np(ws.binv, np.float64))), 'mgpu_ws_write')

    def lp_solve1(self, lb, ub, ws_in=-1, ws_d=True, ws_out=-1, iter_limit=0):
        """mgpu_lp_solve1: one LP from device slot ws_in (-1 slack), final
        basis into slot ws_out; returns (status, obj, iters, x, rc)."""
        p = self.problem
        st, it = _I(0), _I(0)
        obj = ctypes.c_double(0.0)
        x = np.zeros(p.n)
        rc = np.zeros(p.n + p.m)
        self._chk(self.lib.mgpu_lp_solve1(
            self.h, _hp(_np(lb, np.float64)), _hp(_np(ub, np.float64)), int(ws_in),
            1 if ws_d else 0, int(ws_out), int(iter_limit), ctypes.byref(st), ctypes.byref(obj),
            ctypes.byref(it), _hp(x), _hp(rc)), 'mgpu_lp_solve1')
        return st.value, obj.value, it.value, x, rc

    def lp_solve_path(self, lb, ub, ws, k_in, path_in, st_in, inherit=PATH_INHERIT,
                      iter_limit=0, want_x=True):
        """Basis warm starts (mgpu_lp_solve_path): node b starts from its
        parent's basis: statuses st_in[b] and the k_in[b] basic columns
        path_in[b] outside the shared root basis ``ws``, rebuilt by column
        replacement.  Returns (LpOut, k_out, path_out, st_out)."""
        p = self.problem
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        B, N = lb.shape[0], p.n + p.m
        st = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros((B, p.n)) if want_x else None
        k_out = np.zeros(B, dtype=np.int32)
        path_out = np.zeros((B, PATH_MAX), dtype=np.uint32)
        st_out = np.zeros((B, N), dtype=np.int8)
        k_in = _np(k_in, np.int32)
        path_in = _np(path_in, np.uint32).reshape(B, PATH_MAX)
        st_in = _np(st_in, np.int8).reshape(B, N)
        self._chk(self.lib.mgpu_lp_solve_path(
            self.h, B, _hp(lb), _hp(ub), _hp(_np(ws.head, np.int32)), _hp(_np(ws.st, np.int8)),
            _hp(_np(ws.d, np.float64)), _hp(_np(ws.binv, np.float64)), _hp(k_in), _hp(path_in),
            _hp(st_in), int(inherit), int(iter_limit), _hp(st), _hp(obj), _hp(it), _hp(x),
            _hp(k_out), _hp(path_out), _hp(st_out)), 'mgpu_lp_solve_path')
        return LpOut(st, obj, it, x, None), k_out, path_out, st_out

    def lp_solve_dev(self, lb, ub, status, obj, iters, ws=None, skip=None, iter_limit=0,
                     x=None, wo=None):
        """Torch CUDA tensors; ``ws``/``wo`` are WarmStart of CUDA tensors."""
        B = int(lb.shape[0])
        shared = 1 if (ws is None or ws.head.dim() == 1) else 0
        self._chk(self.lib.mgpu_lp_solve_dev(
            self.h, B, _dp(lb), _dp(ub), _dp(skip),
            _dp(ws.head) if ws else None, _dp(ws.st) if ws else None,
            _dp(ws.d) if ws else None, _dp(ws.binv) if ws else None, shared, int(iter_limit),
            _dp(status), _dp(obj), _dp(iters), _dp(x),
            _dp(wo.head) if wo else None, _dp(wo.st) if wo else None,
            _dp(wo.d) if wo else None, _dp(wo.binv) if wo else None), 'mgpu_lp_solve_dev')

    def lp_refactor(self, head, st):
        """The basis (head [m], st [n+m]) refactored for the loaded matrix:
        (WarmStart with binv column-major, singular flag)."""
        p = self.problem
        h = _np(head, np.int32)
        s = _np(st, np.int8)
        oh = np.zeros(p.m, np.int32)
        ost = np.zeros(p.n + p.m, np.int8)
        od = np.zeros(p.n + p.m)
        ob = np.zeros((p.m, p.m))
        sing = ctypes.c_int(0)
        self._chk(self.lib.mgpu_lp_refactor(self.h, _hp(h), _hp(s), _hp(oh), _hp(ost), _hp(od),
                                            _hp(ob), ctypes.byref(sing)), 'mgpu_lp_refactor')
        return WarmStart(oh, ost, od, ob), int(sing.value)

    # -- per-node rows (glob path) ---------------------------------------------
    def set_node_rows(self, nr):
        """``nr``: a ``quad.NodeRows`` map (or None to clear)."""
        if nr is None:
            self._chk(self.lib.mgpu_set_node_rows(self.h, 0, 0, None, None, 0, None, None, None),
                      'mgpu_set_node_rows')
            return
        cp, cs = _np(nr.coef_pos, np.int32), _np(nr.coef_src, np.int32)
        ri, lo, hi = (_np(nr.row_idx, np.int32), _np(nr.lo_src, np.int32),
                      _np(nr.hi_src, np.int32))
        self._keep_rows = (cp, cs, ri, lo, hi)
        self._chk(self.lib.mgpu_set_node_rows(self.h, int(nr.stride), int(cp.size), _hp(cp),
                                              _hp(cs), int(ri.size), _hp(ri), _hp(lo), _hp(hi)),
                  'mgpu_set_node_rows')

    def lp_solve_rows(self, lb, ub, vals, ws=None, skip=None, iter_limit=0, want_x=False):
        """Every node's own LP (node rows from ``vals`` [B, stride]); ``ws``:
        a WarmStart whose head/st (1-D shared or per node) are refactored for
        each node's matrix -- with ws.binv (shared, column-major, the warm
        basis' inverse for the loaded matrix) by column replacement, else
        from scratch; None = slack basis."""
        p = self.problem
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        vals = _np(vals, np.float64)
        B = lb.shape[0]
        st = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros((B, p.n)) if want_x else None
        wh = wst = wb = None
        shared = 1
        if ws is not None:
            wh = _np(ws.head, np.int32)
            wst = _np(ws.st, np.int8)
            shared = 1 if wh.ndim == 1 else 0
            if ws.binv is not None:
                wb = _np(ws.binv, np.float64)
        sk = None if skip is None else _np(skip, np.int32)
        self._chk(self.lib.mgpu_lp_solve_rows(
            self.h, B, _hp(lb), _hp(ub), _hp(sk), _hp(vals), _hp(wh), _hp(wst), shared,
            int(iter_limit), _hp(st), _hp(obj), _hp(it), _hp(x), _hp(wb)), 'mgpu_lp_solve_rows')
        return LpOut(st, obj, it, x, None)

    def lp_solve_rows_dev(self, lb, ub, vals, status, obj, iters, ws=None, skip=None,
                          iter_limit=0, x=None):
        """Torch CUDA tensors (``vals`` e.g. quad_fbbt_dev's rows_out)."""
        B = int(lb.shape[0])
        shared = 1 if (ws is None or ws.head.dim() == 1) else 0
        self._chk(self.lib.mgpu_lp_solve_rows_dev(
            self.h, B, _dp(lb), _dp(ub), _dp(skip), _dp(vals),
            _dp(ws.head) if ws else None, _dp(ws.st) if ws else None, shared, int(iter_limit),
            _dp(status), _dp(obj), _dp(iters), _dp(x),
            _dp(ws.binv) if ws is not None and ws.binv is not None else None),
            'mgpu_lp_solve_rows_dev')

    def lp_bound(self, cols, signs, lb=None, ub=None, ws=None, iter_limit=0, want_x=False):
        """Bound LPs min sign_b * x[col_b] on one box (host arrays); ws: the
        shared warm start (head, st, binv column-major) or None."""
        p = self.problem
        cols = _np(cols, np.int32)
        signs = _np(signs, np.float64)
        B = cols.shape[0]
        lb = _np(p.vlb if lb is None else lb, np.float64)
        ub = _np(p.vub if ub is None else ub, np.float64)
        st = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros((B, p.n)) if want_x else None
        wh = wst = wb = None
        if ws is not None:
            wh, wst, wb = _np(ws.head, np.int32), _np(ws.st, np.int8), _np(ws.binv, np.float64)
        self._chk(self.lib.mgpu_lp_bound(self.h, B, _hp(lb), _hp(ub), _hp(cols), _hp(signs),
                                         _hp(wh), _hp(wst), _hp(wb), int(iter_limit), _hp(st),
                                         _hp(obj), _hp(it), _hp(x)), 'mgpu_lp_bound')
        return LpOut(st, obj, it, x)

    def lp_bound_dev(self, lb, ub, cols, signs, status, obj, iters, ws=None, iter_limit=0,
                     x=None):
        """Device-tensor form of lp_bound (asynchronous)."""
        B = int(cols.shape[0])
        self._chk(self.lib.mgpu_lp_bound_dev(
            self.h, B, _dp(lb), _dp(ub), _dp(cols), _dp(signs),
            _dp(ws.head) if ws is not None else None, _dp(ws.st) if ws is not None else None,
            _dp(ws.binv) if ws is not None else None, int(iter_limit), _dp(status), _dp(obj),
            _dp(iters), _dp(x)), 'mgpu_lp_bound_dev')

    # -- batched branch-and-bound ---------------------------------------------
    def bnb_config(self, order=0, warm=0):
        """Next tree: order 0 depth-first / 1 best-first; warm 0 root basis /
        1 parent basis (mgpu_bnb_config)."""
        self._chk(self.lib.mgpu_bnb_config(self.h, int(order), int(warm)), 'mgpu_bnb_config')

    def bnb_guided_dive(self, on):
        """Order 2: guided dive child order (IntVarHandler guided_dive)."""
        self._chk(self.lib.mgpu_bnb_guided_dive(self.h, int(on)), 'mgpu_bnb_guided_dive')

    def bnb_brancher(self, kind):
        """Next tree's brancher: 0 MaxVio, 1 reliability (mgpu_bnb_brancher)."""
        self._chk(self.lib.mgpu_bnb_brancher(self.h, int(kind)), 'mgpu_bnb_brancher')

    def bnb_growth(self, div):
        """Next tree's batch growth (mgpu_bnb_growth): a round evaluates at most
        max(1, nodes so far // div) nodes; 0 = off."""
        self._chk(self.lib.mgpu_bnb_growth(self.h, int(div)), 'mgpu_bnb_growth')

    def set_sb_chain(self, on):
        """mgpu_set_sb_chain: the reliability brancher's strong-branching
        chains in one K3 launch (1, default) or one launch per chain position
        (0); the same results."""
        self._chk(self.lib.mgpu_set_sb_chain(self.h, int(on)), 'mgpu_set_sb_chain')

    def bnb_relaxation(self, kind):
        """Next tree's relaxation: 0 the loaded LP, 1 the loaded QP by K5
        (mgpu_bnb_relaxation)."""
        self._chk(self.lib.mgpu_bnb_relaxation(self.h, int(kind)), 'mgpu_bnb_relaxation')

    def bnb_init(self, capacity, root_lb=None, root_ub=None, incumbent=math.inf):
        p = self.problem
        lb = _np(p.vlb if root_lb is None else root_lb, np.float64)
        ub = _np(p.vub if root_ub is None else root_ub, np.float64)
        self._chk(self.lib.mgpu_bnb_init(self.h, int(capacity), _hp(lb), _hp(ub),
                                         float(incumbent)), 'mgpu_bnb_init')

    def bnb_round(self, batch, incumbent=math.inf) -> BnbStats:
        st = BnbStats()
        self._chk(self.lib.mgpu_bnb_round(self.h, int(batch), float(incumbent),
                                          ctypes.byref(st)), 'mgpu_bnb_round')
        return st

    def strong_branch(self, lb, ub, cand_var, cand_val, ws=None, iter_limit=25):
        """Down/up child LPs of each candidate (host arrays); returns
        (status[2k], obj[2k], iters[2k]) with child 2c = down, 2c+1 = up."""
        cv = _np(cand_var, np.int32)
        cx = _np(cand_val, np.float64)
        k = cv.size
        st = np.zeros(2 * k, dtype=np.int32)
        ob = np.zeros(2 * k)
        it = np.zeros(2 * k, dtype=np.int32)
        wh = wst = wd = wb = None
        if ws is not None:
            wh, wst = _np(ws.head, np.int32), _np(ws.st, np.int8)
            wd, wb = _np(ws.d, np.float64), _np(ws.binv, np.float64)
        self._chk(self.lib.mgpu_strong_branch(self.h, _hp(_np(lb, np.float64)),
                                              _hp(_np(ub, np.float64)), k, _hp(cv), _hp(cx),
                                              _hp(wh), _hp(wst), _hp(wd), _hp(wb),
                                              int(iter_limit), _hp(st), _hp(ob), _hp(it)),
                  'mgpu_strong_branch')
        return st, ob, it

    # -- QP relaxation (K5) ----------------------------------------------------
    def load_qp(self, qp):
        self._qpkeep = [_np(qp.Q, np.float64), _np(qp.c, np.float64), _np(qp.A, np.float64),
                        _np(qp.b, np.float64)]
        Q, c, A, b = self._qpkeep
        self._chk(self.lib.mgpu_load_qp(self.h, qp.n, qp.m, _hp(Q), _hp(c), float(qp.k),
                                        _hp(A), _hp(b)), 'mgpu_load_qp')
        self.qp = qp

    def qp_solve(self, lb, ub, maxit=0, want_x=True):
        lb = _np(lb, np.float64)
        ub = _np(ub, np.float64)
        B = lb.shape[0]
        st = np.zeros(B, dtype=np.int32)
        ob = np.zeros(B)
        it = np.zeros(B, dtype=np.int32)
        x = np.zeros_like(lb) if want_x else None
        self._chk(self.lib.mgpu_qp_solve(self.h, B, _hp(lb), _hp(ub), int(maxit), _hp(st),
                                         _hp(ob), _hp(it), _hp(x)), 'mgpu_qp_solve')
        return st, ob, it, x

    def qp_solve_dev(self, lb, ub, status, obj, iters, x=None, maxit=0):
        self._chk(self.lib.mgpu_qp_solve_dev(self.h, int(lb.shape[0]), _dp(lb), _dp(ub),
                                             int(maxit), _dp(status), _dp(obj), _dp(iters),
                                             _dp(x)), 'mgpu_qp_solve_dev')

    def bnb_shard(self, rank, world) -> int:
        k = ctypes.c_int(0)
        self._chk(self.lib.mgpu_bnb_shard(self.h, int(rank), int(world), ctypes.byref(k)),
                  'mgpu_bnb_shard')
        return k.value

    def bnb_export(self, k):
        """Remove up to k open nodes: (lb [k,n], ub [k,n], nlb [k], depth [k])."""
        n = self.problem.n
        lb, ub = np.empty((k, n)), np.empty((k, n))
        nlb, dep = np.empty(k), np.empty(k, dtype=np.int32)
        got = ctypes.c_int(0)
        self._chk(self.lib.mgpu_bnb_export(self.h, int(k), _hp(lb), _hp(ub), _hp(nlb), _hp(dep),
                                           ctypes.byref(got)), 'mgpu_bnb_export')
        g = got.value
        return lb[:g], ub[:g], nlb[:g], dep[:g]

    def bnb_import(self, lb, ub, nlb, depth):
        k = len(nlb)
        self._chk(self.lib.mgpu_bnb_import(self.h, int(k), _hp(_np(lb, np.float64)),
                                           _hp(_np(ub, np.float64)), _hp(_np(nlb, np.float64)),
                                           _hp(_np(depth, np.int32))), 'mgpu_bnb_import')

    def bnb_pick(self, S):
        """mgpu_bnb_pick: bounds of this rank's next S candidates (np [got])."""
        lbs = np.empty(max(int(S), 1))
        got = ctypes.c_int(0)
        self._chk(self.lib.mgpu_bnb_pick(self.h, int(S), _hp(lbs), ctypes.byref(got)),
                  'mgpu_bnb_pick')
        return lbs[:got.value].copy()

    def bnb_row_width(self) -> int:
        """mgpu_bnb_row_width: f64 per migration row (2n + 2; warm mode 2
        appends the node's basis)."""
        w = self.lib.mgpu_bnb_row_width(self.h)
        self._chk(w if w < 0 else 0, 'mgpu_bnb_row_width')
        return int(w)

    def bnb_export_rows(self, idx):
        """mgpu_bnb_export_dev: the picked nodes idx leave the pool as device
        rows [k, W] (a torch tensor on this context's device; W =
        bnb_row_width(): [lb | ub | bound | depth] and, in warm mode 2, the
        node's basis)."""
        import torch
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        k = len(idx)
        buf = torch.empty((k, self.bnb_row_width()), dtype=torch.float64,
                          device=torch.device('cuda', self.device))
        self._chk(self.lib.mgpu_bnb_export_dev(self.h, k, _hp(idx) if k else None,
                                               buf.data_ptr() if k else None),
                  'mgpu_bnb_export_dev')
        return buf

    def bnb_import_rows(self, rows):
        """mgpu_bnb_import_dev: rows [k, W] (torch; moved to this device)."""
        import torch
        k = int(rows.shape[0])
        if k == 0:
            return
        W = self.bnb_row_width()
        if rows.dim() != 2 or int(rows.shape[1]) != W:
            raise MgpuError(f"bnb_import_rows: rows of shape {tuple(rows.shape)}, the pool's "
                            f"row width is {W} (mgpu_bnb_row_width)")
        buf = rows.to(device=torch.device('cuda', self.device), dtype=torch.float64).contiguous()
        self._chk(self.lib.mgpu_bnb_import_dev(self.h, k, buf.data_ptr()), 'mgpu_bnb_import_dev')

    def bnb_count(self):
        """mgpu_bnb_count: (open nodes, pool slots left for imports)."""
        o, v = ctypes.c_int(0), ctypes.c_int(0)
        self._chk(self.lib.mgpu_bnb_count(self.h, ctypes.byref(o), ctypes.byref(v)),
                  'mgpu_bnb_count')
        return o.value, v.value

    # -- round collectives (mgpu_comm_*, include/mgpu.h) ------------------------
    def comm_init(self, rank, world, uid: bytes):
        """mgpu_comm_init: an RCCL communicator (uid from comm_unique_id() on
        one rank, handed to every rank by the launcher)."""
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        self._chk(self.lib.mgpu_comm_init(self.h, int(rank), int(world), buf), 'mgpu_comm_init')

    def comm_init_host(self, rank, world, allreduce, allgather, alltoallv):
        """mgpu_comm_init_host: the host's own transport.  The three Python
        callables take numpy arrays (views of the engine's host buffers):
        allreduce(v, op) in place; allgather(send, recv[world, count]);
        alltoallv(send[rows, width], send_counts, recv[rows, width],
        recv_counts)."""
        def ar(_, v, count, op):
            try:
                allreduce(np.ctypeslib.as_array(v, shape=(count,)), int(op))
                return 0
            except Exception:                                  # noqa: BLE001
                return 1

        def ag(_, send, count, recv):
            try:
                allgather(np.ctypeslib.as_array(send, shape=(count,)),
                          np.ctypeslib.as_array(recv, shape=(self._world, count)))
                return 0
            except Exception:                                  # noqa: BLE001
                return 1

        def a2a(_, send, sc, recv, rc, width):
            try:
                P = self._world
                scn = np.ctypeslib.as_array(sc, shape=(P,)).copy()
                rcn = np.ctypeslib.as_array(rc, shape=(P,)).copy()
                ns, nr = int(scn.sum()), int(rcn.sum())
                sv = (np.ctypeslib.as_array(send, shape=(ns, width)) if ns
                      else np.empty((0, width)))
                rv = (np.ctypeslib.as_array(recv, shape=(nr, width)) if nr
                      else np.empty((0, width)))
                alltoallv(sv, scn, rv, rcn)
                return 0
            except Exception:                                  # noqa: BLE001
                return 1
        self._world = int(world)
        self._transport = HostTransport(None, ALLREDUCE_FN(ar), ALLGATHER_FN(ag),
                                        ALLTOALLV_FN(a2a))   # kept alive with the context
        self._chk(self.lib.mgpu_comm_init_host(self.h, int(rank), int(world),
                                               ctypes.byref(self._transport)),
                  'mgpu_comm_init_host')

    def comm_info(self):
        r, w = ctypes.c_int(0), ctypes.c_int(1)
        self._chk(self.lib.mgpu_comm_info(self.h, ctypes.byref(r), ctypes.byref(w)),
                  'mgpu_comm_info')
        return r.value, w.value

    def allreduce(self, vals, op):
        """mgpu_allreduce_f64 over the ranks (op OP_SUM / OP_MIN / OP_MAX)."""
        v = np.array(vals, dtype=np.float64).reshape(-1)
        self._chk(self.lib.mgpu_allreduce_f64(self.h, _hp(v), int(v.size), int(op)),
                  'mgpu_allreduce_f64')
        return v

    def round_reduce(self, inc, n_open, err=0):
        """mgpu_round_reduce -> (incumbent, max open, min open, any error)."""
        out = np.zeros(4)
        self._chk(self.lib.mgpu_round_reduce(self.h, float(inc), float(n_open), int(err),
                                             _hp(out)), 'mgpu_round_reduce')
        return float(out[0]), float(out[1]), float(out[2]), float(out[3])

    def allgather(self, vec):
        """mgpu_allgather_f64 -> [world, count]."""
        v = np.array(vec, dtype=np.float64).reshape(-1)
        _, w = self.comm_info()
        out = np.empty((w, v.size))
        self._chk(self.lib.mgpu_allgather_f64(self.h, _hp(v), int(v.size), _hp(out)),
                  'mgpu_allgather_f64')
        return out

    def alltoall_rows(self, rows, send_counts, recv_counts):
        """mgpu_alltoall_rows_dev on torch device rows [k, W] -> received rows."""
        import torch
        W = int(rows.shape[1])
        sc = np.ascontiguousarray(send_counts, dtype=np.int32)
        rc = np.ascontiguousarray(recv_counts, dtype=np.int32)
        out = torch.empty((int(rc.sum()), W), dtype=torch.float64, device=rows.device)
        inp = rows.contiguous()
        self._chk(self.lib.mgpu_alltoall_rows_dev(self.h, W, _dp(inp) if inp.numel() else None,
                                                  _hp(sc), _dp(out) if out.numel() else None,
                                                  _hp(rc)), 'mgpu_alltoall_rows_dev')
        return out

    def bnb_rebalance(self, S):
        """mgpu_bnb_rebalance: one LoadBalance_ -> (open afterwards, nodes moved,
        the bounds this rank offered, the bounds it received in deal order)."""
        _, w = self.comm_info()
        picked = np.empty(int(S))
        got = np.empty(int(S) * w)
        npk, ngot, op = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        mv = ctypes.c_longlong(0)
        self._chk(self.lib.mgpu_bnb_rebalance(self.h, int(S), _hp(picked), ctypes.byref(npk),
                                              _hp(got), ctypes.byref(ngot), ctypes.byref(mv),
                                              ctypes.byref(op)), 'mgpu_bnb_rebalance')
        return op.value, int(mv.value), picked[:npk.value].copy(), got[:ngot.value].copy()

    # -- batched spatial B&B (mgpu_glob_*) ------------------------------------
    def glob_config(self, order=0, warm=0, qt=1, lin=0, obbt=0):
        """mgpu_glob_config: the next glob_init's node order (0 stack, 2 the
        reference's heap), warm starts (0 root basis, 1 parent basis),
        tightenQuad_ rule (1 every node, 0 the first call only), linear node
        presolve (1 LinearHandler::presolveNode at every node, 0 none) and
        root OBBT (1 QuadHandler::postSolveRootNode, 0 none)."""
        self._chk(self.lib.mgpu_glob_config(self.h, int(order), int(warm), int(qt), int(lin),
                                            int(obbt)), 'mgpu_glob_config')

    def glob_brancher(self, kind):
        """mgpu_glob_brancher: the next glob_init's brancher (0 MaxVio, 1 Glob's
        relstronger: one node per round, order 2, warm 1, lin 1)."""
        self._chk(self.lib.mgpu_glob_brancher(self.h, int(kind)), 'mgpu_glob_brancher')

    def glob_lp_log(self):
        """mgpu_glob_lp_log: (status, value, pivots) of every main-engine solve
        of a relstronger tree, in order."""
        n = self.lib.mgpu_glob_lp_log(self.h, 0, None, None, None)
        if n < 0:
            self._chk(n, 'mgpu_glob_lp_log')
        st = np.zeros(n, dtype=np.int32)
        val = np.zeros(n)
        it = np.zeros(n, dtype=np.int32)
        self.lib.mgpu_glob_lp_log(self.h, n, st.ctypes.data, val.ctypes.data, it.ctypes.data)
        return st, val, it

    def glob_init(self, capacity, incumbent=math.inf):
        self._chk(self.lib.mgpu_glob_init(self.h, int(capacity), float(incumbent)),
                  'mgpu_glob_init')

    def glob_round(self, batch, incumbent=math.inf) -> GlobStats:
        st = GlobStats()
        self._chk(self.lib.mgpu_glob_round(self.h, int(batch), float(incumbent),
                                           ctypes.byref(st)), 'mgpu_glob_round')
        return st

    def glob_best(self):
        x = np.empty(self.quad.nv)
        v = ctypes.c_double(0.0)
        self._chk(self.lib.mgpu_glob_best(self.h, ctypes.byref(v), _hp(x)), 'mgpu_glob_best')
        return v.value, x

    def bnb_best(self):
        x = np.empty(self.problem.n)
        v = ctypes.c_double(0.0)
        self._chk(self.lib.mgpu_bnb_best(self.h, ctypes.byref(v), _hp(x)), 'mgpu_bnb_best')
        return v.value, x

    def root_solve(self, iter_limit=0):
        """Solve the root LP from the slack basis; returns (LpOut, WarmStart)."""
        p = self.problem
        r = self.lp_solve(p.vlb[None], p.vub[None], None, None, iter_limit, True, True)
        return r, r.ws.node(0)

    # -- node decision -------------------------------------------------------
    def node_decide_dev(self, status, obj, x, decision, incumbent=math.inf, fbbt_infeas=None,
                        inf_meas=None, cand_obj=None, abs_tol=1e-6, rel_tol=1e-6,
                        cutoff=math.inf, int_tol=1e-6):
        B = int(status.shape[0])
        self._chk(self.lib.mgpu_node_decide_dev(
            self.h, B, _dp(fbbt_infeas), _dp(status), _dp(obj), _dp(x), float(incumbent),
            float(abs_tol), float(rel_tol), float(cutoff), float(int_tol), _dp(decision),
            _dp(inf_meas), _dp(cand_obj)), 'mgpu_node_decide_dev')
