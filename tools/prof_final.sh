set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06zj_prof BENCH_ARGS="--steps 20 --warmup 3 --batch 524288 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --no-oa-tree" bash tools/prof_run.sh
