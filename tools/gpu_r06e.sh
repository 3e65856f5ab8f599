set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.txt | tail -40
exit $rc
