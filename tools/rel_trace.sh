#!/bin/bash
# Kernel trace + stats of config 2's reliability tree (tools/rel_time.py: a
# warm-up solve and 7 timed solves) on the GPU box, from the repo root.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-rel_trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/rel_time.py 7 > $O/rel_time.txt 2>&1 || { tail -20 $O/rel_time.txt; exit 1; }
grep median $O/rel_time.txt
