#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then separate PMC passes for FETCH_SIZE and
#   WRITE_SIZE (MI355X_MICROARCH.md: TCC slots; FETCH_SIZE reads half of a
#   wide stream -> doubled when converted to bytes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-$R/gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --batch 524288 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --no-oa-tree}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_write.log 2>&1 || exit $?
echo "profiles done"
