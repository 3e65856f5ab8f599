set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 > $O/w1g2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o rel -- python3 tools/rel_tls4_one.py 131072 1 2 > $O/prof.txt 2>&1
cat $O/w1g2.txt | grep -v amdgpu.ids
