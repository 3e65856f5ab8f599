set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || { grep -E "FAILED|ERROR|passed|failed|Error" $O/gpu_tests.txt | tail -30; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u tools/rel_ab.py 5 > $O/rel_ab.jsonl 2> $O/rel_ab.err || { tail -20 $O/rel_ab.err; exit 1; }
tail -1 $O/rel_ab.jsonl
