#!/bin/bash
# Round-end evidence on the GPU box (repo root): the GPU test suite, smoke(),
# the default bench line, rocprof kernel stats of the same bench, and the
# headline's PMC passes (tools/prof_run.sh).  Output under gpurun_out/$TAG.
set -o pipefail
TAG=${TAG:-r03a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit $?
cd $R
OUT=$O/pmc bash tools/prof_run.sh || exit $?
echo done
