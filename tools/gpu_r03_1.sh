set -o pipefail
O=gpurun_out/r03_g18
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ref_tree_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo done
