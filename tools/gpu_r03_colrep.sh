#!/bin/bash
# K3R column replacement: parity tests, then the glob batch / glob tree timings
set -o pipefail
TAG=${TAG:-r03g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_rows_gpu.py tests/test_glob_gpu.py tests/test_quad_gpu.py -x -q --timeout 240 --timeout-method thread > $O/colrep_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-fixed > $O/glob_bench.json 2> $O/glob_bench.err || exit $?
echo done
