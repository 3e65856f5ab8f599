#!/bin/bash
# headline A/B: path warm starts (warm 2) vs parent bases (warm 1, dense inverse per node)
set -o pipefail
TAG=${TAG:-r03h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
timeout -k 10 300 python -u bench.py $ARGS --batch 131072 --warm 2 > $O/w2_131k.json 2> $O/w2_131k.err || exit $?
timeout -k 10 300 python -u bench.py $ARGS --batch 131072 --warm 1 > $O/w1_131k.json 2> $O/w1_131k.err || exit $?
echo done
