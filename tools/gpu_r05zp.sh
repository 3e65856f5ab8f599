set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zp; mkdir -p $O
TAG=pair timeout -k 10 120 python tools/k1g_pair_dbg.py 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fbbt_gpu.py tests/test_tls4_oa_gpu.py tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py tests/test_bnb_gpu.py tests/test_glob_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
for v in base pair; do
  if [ $v = base ]; then L=tools/_stamps/k1gbase/libmgpu.so; else L=minotaur_amd/libmgpu.so; fi
  echo "== $v rep $rep"
  MGPU_LIB=$L timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 2>&1 | grep -v amdgpu | tail -1 || exit 1
  MGPU_LIB=$L timeout -k 10 120 python tools/oa_tree_one.py 2>&1 | grep -v amdgpu | tail -1 || exit 1
done
done
