"""A/B builds of libmgpu for kernel experiments: a copy of csrc/ with textual
edits applied, compiled into tools/_stamps/<name>/libmgpu.so (unchanged
translation units reuse minotaur_amd/build/*.o).  Run a bench or probe with
MGPU_LIB=tools/_stamps/<name>/libmgpu.so to time the variant.

    python tools/variant_build.py NAME FILE 'old' 'new' [FILE 'old' 'new' ...]

(OLD = @FILE replaces FILE with the contents of the file at path NEW.)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from minotaur_amd import build as b
    name, edits = sys.argv[1], sys.argv[2:]
    assert len(edits) % 3 == 0, "edits come as FILE OLD NEW triples"
    out = os.path.join(ROOT, 'tools', '_stamps', name)
    src = os.path.join(out, 'csrc')
    if os.path.isdir(src):
        shutil.rmtree(src)
    shutil.copytree(b.CSRC, src)
    changed = set()
    for k in range(0, len(edits), 3):
        f, old, new = edits[k:k + 3]
        p = os.path.join(src, f)
        s = open(p).read()
        if old == '@FILE':   # replace the whole file with the file at path NEW
            open(p, 'w').write(open(new).read())
        else:
            assert s.count(old) >= 1, f"{f}: pattern not found: {old!r}"
            open(p, 'w').write(s.replace(old, new))
        changed.add(f)
    b.build()   # the reference objects are current
    objs = []
    cflags = [x for x in b.FLAGS if x != '-shared'] + ['-I', os.path.join(ROOT, 'include')]
    for s in b.SOURCES:
        if s in changed:
            o = os.path.join(out, s + '.o')
            subprocess.run([b.HIPCC] + cflags + ['-c', '-o', o, os.path.join(src, s),
                            '-Rpass-analysis=kernel-resource-usage'], check=True,
                           stderr=open(os.path.join(out, s + '.remarks'), 'w'))
            objs.append(o)
        else:
            objs.append(os.path.join(b.HERE, 'build', s + '.o'))
    lib = os.path.join(out, 'libmgpu.so')
    subprocess.run([b.HIPCC, '-shared', '-fPIC', f'--offload-arch={b.ARCH}', '-o', lib] + objs +
                   ['-L/opt/rocm/lib', '-lrccl'],
                   check=True)
    print(lib)


if __name__ == '__main__':
    main()
