set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
STAMP_LIB=tools/_stamps/libmgpu_stamps.so PROBE_BATCH=524288 timeout -k 10 300 python tools/lp_stamps.py --tree > $O/stamps_tree.txt 2>&1 || { tail -20 $O/stamps_tree.txt; exit 1; }
OUT=$GRAFT_REPO_ROOT/$O/prof timeout -k 10 900 bash tools/prof_run.sh || exit 1
cat $O/stamps_tree.txt | grep -v amdgpu.ids
