#!/bin/bash
# per-node rows beyond 64 rows (K3L) and the glob tree on them
set -o pipefail
TAG=${TAG:-r03e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_rows_gpu.py tests/test_glob_gpu.py tests/test_lp_large_gpu.py tests/test_lp_gpu.py -x -v --timeout 240 --timeout-method thread > $O/rows_tests.txt 2>&1 || exit $?
echo done
