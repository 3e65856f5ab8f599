#!/bin/bash
# K3PW BTRAN zero-product skip, and K3P replay groups of 8 vs 4:
# parity tests with the new library, then the headline + convex-batch A/B
# against the previous kernels (ab/base) and 8-column replay groups (ab/rg8)
set -o pipefail
TAG=${TAG:-r03m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_lp_pfi_wide_gpu.py tests/test_lp_path_gpu.py \
  tests/test_lp_large_gpu.py > $O/tests.txt 2>&1 || exit $?
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-knapsack --no-glob --no-fixed"
for rep in 1 2; do
  for v in base new rg8; do
    if [ $v = new ]; then L=$R/minotaur_amd/libmgpu.so; else L=$R/ab/$v/libmgpu.so; fi
    MGPU_LIB=$L timeout -k 10 300 python -u bench.py $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit $?
    echo "$v $rep done"
  done
done
echo done
