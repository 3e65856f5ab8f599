set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 > $O/w1g2.txt 2>&1 || exit 1
TAG=r05f VARIANTS="base w12 r8 g2" timeout -k 10 1000 bash tools/ab_headline.sh > $O/ab.txt 2>&1
tail -3 $O/tests.txt; grep -v amdgpu $O/w1g2.txt; cat $O/ab.txt
