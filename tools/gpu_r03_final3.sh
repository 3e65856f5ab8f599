#!/bin/bash
# K3P rho / primal B0 loops with eight loads in flight: headline A/B against
# the previous kernel (ab/base), then the full GPU suite, smoke, the default
# bench line and a kernel-trace summary of the headline with the new library
set -o pipefail
TAG=${TAG:-r03n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_lp_path_gpu.py tests/test_lp_pfi_gpu.py > $O/k3p_tests.txt 2>&1 || exit $?
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob"
for rep in 1 2; do
  for v in base new; do
    if [ $v = new ]; then L=$R/minotaur_amd/libmgpu.so; else L=$R/ab/$v/libmgpu.so; fi
    MGPU_LIB=$L timeout -k 10 300 python -u bench.py $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit $?
    echo "$v $rep done"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
echo "suite done"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 360 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench done"
(cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/prof_bench.json 2> $O/prof_bench.err) || exit $?
echo done
