set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fbbt_gpu.py tests/test_tls4_oa_gpu.py > gpurun_out/r05o_tests.txt 2>&1 || { tail -30 gpurun_out/r05o_tests.txt; exit 1; }
tail -2 gpurun_out/r05o_tests.txt
TAG=r05o VARIANTS="k1head base+MGPU_FBBT_NOSLOTS=1 base" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05o.txt 2>&1; cat gpurun_out/r05o.txt
