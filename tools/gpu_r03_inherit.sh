#!/bin/bash
# headline sweep of the longest inherited path (MGPU_PATH_INHERIT) now that
# the replay builds its etas four columns at a time
set -o pipefail
TAG=${TAG:-r03p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
for inh in 24 28 32 20; do
  MGPU_PATH_INHERIT=$inh timeout -k 10 300 python -u bench.py $ARGS > $O/inh$inh.json 2> $O/inh$inh.err || exit $?
  echo "inherit $inh done"
done
echo done
