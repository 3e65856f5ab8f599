set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fbbt_gpu.py tests/test_tls4_oa_gpu.py > gpurun_out/r05j_tests.txt 2>&1 || { tail -30 gpurun_out/r05j_tests.txt; exit 1; }
tail -3 gpurun_out/r05j_tests.txt
TAG=r05j VARIANTS="base base+MGPU_FBBT_NOSLOTS=1" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05j.txt 2>&1; cat gpurun_out/r05j.txt
