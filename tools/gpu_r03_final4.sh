#!/bin/bash
# final evidence: full GPU suite, smoke, the default bench line and a
# kernel-trace summary of the headline
set -o pipefail
TAG=${TAG:-r03o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
echo "suite done"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 360 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench done"
(cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/prof_bench.json 2> $O/prof_bench.err) || exit $?
echo done
