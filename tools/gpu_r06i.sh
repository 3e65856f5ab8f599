set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
STAMP_LIB=tools/_stamps/libmgpu_stamps.so timeout -k 10 300 python -u tools/lp_stamps.py --rel > $O/rel_stamps.txt 2>&1 || { tail -20 $O/rel_stamps.txt; exit 1; }
cat $O/rel_stamps.txt
