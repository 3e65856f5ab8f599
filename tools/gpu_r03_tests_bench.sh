#!/bin/bash
# GPU suite + smoke + default bench line on the box (repo root), output under gpurun_out/$TAG.
set -o pipefail
TAG=${TAG:-r03b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 360 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo done
