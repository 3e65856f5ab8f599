set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zh; mkdir -p $O
timeout -k 10 120 python tools/rel_tls4_one.py 131072 1 2 > $O/rel_before_tests.txt 2>&1 || { cat $O/rel_before_tests.txt; exit 1; }
grep -v amdgpu $O/rel_before_tests.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py tests/test_tls4_oa_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $O/prof -o run -- python3 tools/rel_tls4_one.py 131072 1 2 > $O/prof.txt 2>&1 || exit 1
python3 tools/trace_summary.py $(find $O/prof -name '*.db' | head -1) > $O/trace.txt 2>&1 || true
head -20 $O/trace.txt
