set -o pipefail
O=gpurun_out/r03_g6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_lp_pfi_gpu.py tests/test_tls4_oa_gpu.py tests/test_nvs08_gpu.py tests/test_bnb_gpu.py tests/test_bnb_rel_gpu.py tests/test_obbt_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
echo done
