set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o relprof --output-format csv -- python3 tools/rel_ab.py 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*stats*" | head
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-220
