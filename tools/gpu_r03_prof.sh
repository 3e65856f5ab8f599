#!/bin/bash
# Headline evidence on the box (repo root): K3P section stamps inside the
# tree rounds (diagnostic build diag/libmgpu_stamps.so), then rocprof kernel
# stats and the PMC traffic passes of the headline (tools/prof_run.sh).
set -o pipefail
TAG=${TAG:-r03b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -f diag/libmgpu_stamps.so ]; then
  STAMP_LIB=$R/diag/libmgpu_stamps.so timeout -k 10 240 python -u tools/lp_stamps.py --tree > $O/stamps_tree.txt 2>&1 || exit $?
fi
# instruction-fetch pressure of the headline kernels (K3P's code is 159 KB)
ARGS="--steps 3 --warmup 1 --batch 524288 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $O/icache -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/icache.log 2>&1) || echo "icache pmc pass failed rc=$?"
OUT=$O/prof bash tools/prof_run.sh || exit $?
echo profiles done
# the N>1 path rehearsed on this one-GPU box (2 ranks over gloo)
TAG=$TAG bash tools/gpu_r03_rehearse.sh || exit $?
echo rehearsal done
