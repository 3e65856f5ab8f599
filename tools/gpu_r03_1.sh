set -o pipefail
O=gpurun_out/r03_g9
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bnb_gpu.py tests/test_tls4_oa_gpu.py tests/test_bnb_rel_gpu.py tests/test_lp_path_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
echo done
