set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zs; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py tests/test_tls4_oa_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
for v in base fused; do
  if [ $v = base ]; then L=tools/_stamps/relbase/libmgpu.so; else L=minotaur_amd/libmgpu.so; fi
  echo "== $v rep $rep $(MGPU_LIB=$L timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 2>&1 | grep -v amdgpu | tail -1)" || exit 1
done
done
