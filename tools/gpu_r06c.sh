set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rel -o rel -- python3 $GRAFT_REPO_ROOT/tools/rel_tls4_one.py > $GRAFT_REPO_ROOT/$O/rel.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/rel.log; exit 1; }
cd $GRAFT_REPO_ROOT && cat $O/rel.log | grep -v amdgpu.ids | tail -5
find $O/rel -name "*stats*" | head
