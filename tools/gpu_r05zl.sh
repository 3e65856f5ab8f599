set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zl; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_glob_ref_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "seed|passed|failed" $O/tests.txt | tail -30
