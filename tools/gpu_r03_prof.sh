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
OUT=$O/prof bash tools/prof_run.sh || exit $?
echo done
