"""CPU: the C-ABI library builds, loads, and exports every entry point that
include/mgpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from minotaur_amd import build, runtime

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def declared_symbols():
    hdr = open(os.path.join(ROOT, 'include', 'mgpu.h')).read()
    hdr = re.sub(r'/\*.*?\*/', '', hdr, flags=re.S)
    return sorted(set(re.findall(r'\b(mgpu_[a-z0-9_]+)\s*\(', hdr)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert 'mgpu_fbbt' in syms and 'mgpu_load_lp' in syms and 'mgpu_create' in syms
    assert set(syms) == set(runtime.EXPORTS)


def test_library_exports_every_declared_symbol():
    path = build.build()
    lib = ctypes.CDLL(path)
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_no_cpu_fallback_without_device():
    """Creating a context with no visible HIP device must fail loudly."""
    import torch
    if torch.cuda.is_available():
        return
    lib = runtime.load_library()
    h = ctypes.c_void_p()
    assert lib.mgpu_create(0, ctypes.byref(h)) != 0
    try:
        runtime.Context(0)
    except runtime.MgpuError:
        pass
    else:
        raise AssertionError("Context() succeeded without a GPU")


def _header_arity():
    hdr = open(os.path.join(ROOT, 'include', 'mgpu.h')).read()
    hdr = re.sub(r'/\*.*?\*/', '', hdr, flags=re.S)
    out = {}
    for name, args in re.findall(r'\b(mgpu_[a-z0-9_]+)\s*\(([^)]*)\)\s*;', hdr):
        args = args.strip()
        out[name] = 0 if args in ('', 'void') else len(args.split(','))
    return out


def test_ctypes_signatures_match_header():
    lib = runtime.load_library()
    for name, nargs in _header_arity().items():
        assert len(getattr(lib, name).argtypes) == nargs, name


def test_pfi_cap_matches_header():
    """runtime.LP_PFI_MAX (used by tests and bench.py) is the header's cap."""
    hdr = open(os.path.join(ROOT, 'include', 'mgpu.h')).read()
    m = re.search(r'#define MGPU_LP_PFI_MAX (\d+)', hdr)
    assert m and int(m.group(1)) == runtime.LP_PFI_MAX
    m = re.search(r'#define MGPU_PATH_MAX (\d+)', hdr)
    import oracle
    assert m and int(m.group(1)) == runtime.PATH_MAX == oracle.PATH_MAX


def test_reference_libraries_coexist_in_one_process():
    """The two test libraries that carry the reference objects (oracle/_ref:
    libref_fbbt.so and the integration library, loaded RTLD_GLOBAL by the
    integration tests) are linked -Bsymbolic: loading both and exiting must
    not destroy one copy of the reference's static objects twice."""
    import subprocess
    import sys
    ref = os.path.join(ROOT, 'oracle', '_ref')
    a, b = os.path.join(ref, 'libminotaur_hip_integ.so'), os.path.join(ref, 'libref_fbbt.so')
    if not (os.path.exists(a) and os.path.exists(b)):
        import pytest
        pytest.skip('oracle/_ref not built')
    code = ("import ctypes, os\n"
            f"ctypes.CDLL({a!r}, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)\n"
            f"ctypes.CDLL({b!r}, mode=os.RTLD_LAZY)\n")
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-500:]
