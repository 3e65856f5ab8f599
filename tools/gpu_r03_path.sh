#!/bin/bash
# path warm starts handing children the starting path on overflow: parity, then the headline
set -o pipefail
TAG=${TAG:-r03i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_lp_path_gpu.py tests/test_bnb_gpu.py tests/test_tls4_oa_gpu.py tests/test_lp_pfi_gpu.py -x -q --timeout 200 --timeout-method thread > $O/path_tests.txt 2>&1 || exit $?
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
timeout -k 10 300 python -u bench.py $ARGS --batch 131072 --warm 2 > $O/w2_131k.json 2> $O/w2_131k.err || exit $?
timeout -k 10 300 python -u bench.py $ARGS > $O/w2_524k.json 2> $O/w2_524k.err || exit $?
echo done
