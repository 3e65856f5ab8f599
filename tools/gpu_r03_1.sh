set -o pipefail
O=gpurun_out/r03_g31
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ref_tree_gpu.py tests/test_integration_gpu.py -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -2 $O/tests.txt
exit $rc
