#!/bin/bash
# K3P path replay in groups of four columns + BTRAN zero-product skip:
# parity tests with the new library, then the headline A/B against the
# previous kernel (ab/base) and the replay change alone (ab/replay)
set -o pipefail
TAG=${TAG:-r03l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_lp_path_gpu.py tests/test_lp_pfi_gpu.py tests/test_bnb_gpu.py tests/test_tls4_oa_gpu.py \
  tests/test_ref_tree_gpu.py tests/test_bnb_rel_gpu.py > $O/tests.txt 2>&1 || exit $?
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob"
for rep in 1 2; do
  for v in base replay new; do
    if [ $v = new ]; then L=$R/minotaur_amd/libmgpu.so; else L=$R/ab/$v/libmgpu.so; fi
    MGPU_LIB=$L timeout -k 10 300 python -u bench.py $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit $?
    echo "$v $rep done"
  done
done
echo done
