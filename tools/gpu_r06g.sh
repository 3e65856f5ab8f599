set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_bnb_rel_gpu.py tests/test_ref_tree_gpu.py > $O/rel_tests.txt 2>&1 || { grep -E "FAILED|ERROR|passed|failed|Error" $O/rel_tests.txt | tail -30; exit 1; }
tail -2 $O/rel_tests.txt
timeout -k 10 300 python -u tools/rel_ab.py 5 > $O/rel_ab.jsonl 2> $O/rel_ab.err || { tail -20 $O/rel_ab.err; exit 1; }
cat $O/rel_ab.jsonl
