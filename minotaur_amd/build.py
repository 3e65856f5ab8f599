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

SOURCES = ['mgpu_runtime.cpp', 'quad_runtime.cpp', 'fbbt_linear.hip', 'lp_dual.hip',
           'node_decide.hip', 'quad_fbbt.hip']
# -ffp-contract=off: no fused multiply-add anywhere (bit-exact FBBT sums,
# SURVEY §7.3); -fno-gpu-rdc keeps one code object per TU.
FLAGS = ['-O3', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off',
         f'--offload-arch={ARCH}', '-Wall', '-Wno-unused-function']


def lib_path():
    return os.path.join(HERE, 'libmgpu.so')


def build(verbose=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    out = lib_path()
    newest = max(os.path.getmtime(p) for p in srcs + [os.path.join(CSRC, h) for h in
                                                        os.listdir(CSRC) if h.endswith('.h')]
                 + [os.path.join(ROOT, 'include', 'mgpu.h')])
    if os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    cmd = [HIPCC] + FLAGS + ['-I', os.path.join(ROOT, 'include'), '-o', out] + srcs
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True)
    return out


if __name__ == '__main__':
    print(build(verbose=True))
    sys.exit(0)
