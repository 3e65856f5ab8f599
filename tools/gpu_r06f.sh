set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_glob_pin_gpu.py tests/test_glob_gpu.py tests/test_glob_ref_gpu.py tests/test_glob_squares_gpu.py tests/test_simplex_cuts_gpu.py > $O/glob_tests.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/glob_tests.txt | tail -40
exit $rc
