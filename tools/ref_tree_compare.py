"""The batched tree (order 2, warm 1, batch 1) against the reference's own
BranchAndBound (tests/test_ref_tree_gpu.py): one JSON line per instance with
both sides' counts and times (GPU box; writes nothing else)."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))


def main():
    import test_ref_tree_gpu as t
    from minotaur_amd.runtime import Context
    lib = t.integ.__wrapped__() if hasattr(t.integ, '__wrapped__') else None
    if lib is None:
        import ctypes
        from minotaur_amd import runtime
        runtime.load_library()
        lib = ctypes.CDLL(t.LIB, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
        lib.integ_bnb_tree.argtypes = [ctypes.c_int] * 6 + [t.P] * 9 + [ctypes.c_double, t.P, t.P]
    ctx = Context(0)
    for name, p in t._cases().items():
        for guided in (1, 0):
            ref = t.reference_tree(lib, p, guided=guided)
            gpu = t.batched_tree(ctx, p, guided=guided)
            gpu.pop("x")
            print(json.dumps({"instance": name, "guided_dive": guided, "reference": ref,
                              "batched_batch1": gpu,
                              "identical": (gpu["processed"], gpu["created"], gpu["lps"],
                                            gpu["ub"]) == (ref["processed"], ref["created"],
                                                           ref["lps"], ref["ub"])}),
                  flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
