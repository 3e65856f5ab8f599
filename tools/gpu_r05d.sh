set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bnb_rel_gpu.py -k "growth" -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 > $O/w1g2.txt 2>&1 && timeout -k 10 120 python tools/rel_tls4_one.py 131072 0 2 > $O/w0g2.txt 2>&1 && timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 0 > $O/w1g0.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o rel -- python3 tools/rel_tls4_one.py 131072 1 2 > $O/prof.txt 2>&1
tail -3 $O/tests.txt; cat $O/w1g2.txt $O/w0g2.txt $O/w1g0.txt | grep -v amdgpu.ids
