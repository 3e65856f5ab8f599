set -o pipefail
O=gpurun_out/r03_g16
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_lp_pfi_gpu.py tests/test_lp_path_gpu.py tests/test_tls4_oa_gpu.py tests/test_bnb_gpu.py tests/test_obbt_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
export STAMP_LIB=$PWD/diag/libmgpu_stamps.so
PROBE_WARM=2 timeout -k 10 300 python -u tools/lp_stamps.py --tree > $O/stamps_w2.txt 2>&1 || exit $?
unset STAMP_LIB
timeout -k 10 600 python -u bench.py --steps 10 --no-cpu-baseline --no-bnb --no-convex --no-qp --no-knapsack --no-glob > $O/bench.json 2> $O/bench.err || exit $?
echo done
