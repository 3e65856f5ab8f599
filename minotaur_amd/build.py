"""In-tree build of the HIP engine (libmgpu.so) for gfx950.

hipcc cross-compiles without a GPU; the .so lives next to this file so it
travels to the GPU box with the repository snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'

SOURCES = ['mgpu_runtime.cpp', 'quad_runtime.cpp', 'bnb.cpp', 'fbbt_linear.hip', 'fbbt_group.hip',
           'lp_dual.hip', 'lp_pfi.hip', 'lp_pfi_wide.hip', 'lp_large.hip', 'node_decide.hip', 'quad_fbbt.hip', 'bnb.hip',
           'bnb_select.hip', 'qp_runtime.cpp', 'rows_runtime.cpp', 'lp_rows.hip', 'bnb_rel.hip', 'bnb_migrate.hip',
           'glob_tree.hip', 'glob_runtime.cpp',
           'qp_kkt.hip', 'comm_runtime.cpp', 'serial.cpp']
# -ffp-contract=off: no fused multiply-add anywhere (bit-exact FBBT sums,
# SURVEY §7.3); -fno-gpu-rdc keeps one code object per TU.
FLAGS = ['-O3', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off',
         f'--offload-arch={ARCH}', '-Wall', '-Wno-unused-function']


def lib_path():
    return os.path.join(HERE, 'libmgpu.so')


def source_digest():
    """sha256 (first 16 hex digits) over the engine's sources and headers:
    tools/pmc_summary.py stores it with a PMC summary and bench.py compares
    it, so counters measured on other code are reported as stale."""
    import hashlib
    h = hashlib.sha256()
    names = sorted(SOURCES + [f for f in os.listdir(CSRC) if f.endswith('.h')])
    for name in names:
        h.update(name.encode())
        with open(os.path.join(CSRC, name), 'rb') as fh:
            h.update(fh.read())
    with open(os.path.join(ROOT, 'include', 'mgpu.h'), 'rb') as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def build(verbose=False, jobs=None):
    """Compile every translation unit to an object (in parallel, objects
    under build/) and link libmgpu.so; no-op when it is up to date."""
    from concurrent.futures import ThreadPoolExecutor
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    out = lib_path()
    headers = ([os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith('.h')]
               + [os.path.join(ROOT, 'include', 'mgpu.h')])
    newest_h = max(os.path.getmtime(h) for h in headers)
    newest = max([newest_h] + [os.path.getmtime(p) for p in srcs])
    if os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    objdir = os.path.join(HERE, 'build')
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != '-shared'] + ['-I', os.path.join(ROOT, 'include')]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + '.o')
        if (os.path.exists(obj) and os.path.getmtime(obj) >= max(newest_h, os.path.getmtime(src))):
            return obj
        cmd = [HIPCC] + cflags + ['-c', '-o', obj, src]
        if verbose:
            print(' '.join(cmd))
        subprocess.run(cmd, check=True)
        return obj

    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2) // 2), 8)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    # RCCL for the round collectives (comm_runtime.cpp); under torch the
    # process's one librccl.so.1 (torch's, same soname) serves both
    cmd = ([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', out] + objs +
           ['-L/opt/rocm/lib', '-lrccl'])
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True)
    return out


if __name__ == '__main__':
    print(build(verbose=True))
    sys.exit(0)
