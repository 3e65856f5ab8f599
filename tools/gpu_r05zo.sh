set -o pipefail
export TMPDIR=/tmp
for v in pair1; do
  TAG=$v MGPU_LIB=tools/_stamps/$v/libmgpu.so timeout -k 10 120 python tools/k1g_pair_dbg.py 2>&1 | grep -v amdgpu || exit 1
done

