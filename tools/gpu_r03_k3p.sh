#!/bin/bash
# K3P A/B on the box: LP / tree parity tests, the headline alone, its
# instruction-fetch counters.
set -o pipefail
TAG=${TAG:-r03c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_lp_pfi_gpu.py tests/test_lp_path_gpu.py tests/test_bnb_gpu.py tests/test_tls4_oa_gpu.py tests/test_obbt_gpu.py -x -q --timeout 200 --timeout-method thread > $O/k3p_tests.txt 2>&1 || exit $?
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
timeout -k 10 300 python -u bench.py $ARGS > $O/headline.json 2> $O/headline.err || exit $?
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $O/icache -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed > $O/icache.log 2>&1) || echo "icache pass rc=$?"
echo done
