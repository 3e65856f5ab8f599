#!/bin/bash
# Round-end profiles on the box: rocprof kernel stats of the whole default
# bench, then the headline's PMC passes (tools/prof_run.sh).
set -o pipefail
TAG=${TAG:-r03f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace_all -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit $?
cd $R
OUT=$O/prof bash tools/prof_run.sh || exit $?
echo done
