set -o pipefail
O=gpurun_out/r03_g19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lp_gpu.py tests/test_integration_gpu.py -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
exit $rc
