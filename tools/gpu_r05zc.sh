set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lp_pfi_gpu.py tests/test_tls4_oa_gpu.py > gpurun_out/r05zc/tests.txt 2>&1 || { tail -30 gpurun_out/r05zc/tests.txt; exit 1; }
tail -2 gpurun_out/r05zc/tests.txt
TAG=r05zc32 timeout -k 10 400 bash tools/ab_headline.sh > gpurun_out/r05zc/ab32.txt 2>&1 || exit 1
TAG=r05zc24 ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --eta-cap 24" timeout -k 10 400 bash tools/ab_headline.sh > gpurun_out/r05zc/ab24.txt 2>&1 || exit 1
TAG=r05zc28 ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --eta-cap 28" timeout -k 10 400 bash tools/ab_headline.sh > gpurun_out/r05zc/ab28.txt 2>&1 || exit 1
cat gpurun_out/r05zc/ab32.txt gpurun_out/r05zc/ab24.txt gpurun_out/r05zc/ab28.txt
