set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zb; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lp_gpu.py tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py tests/test_lp_pfi_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 > $O/w1g2.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/w1g2.txt
