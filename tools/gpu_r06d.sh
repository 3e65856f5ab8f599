set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_glob_pin_gpu.py -s > $O/pin.txt 2>&1; rc=$?
grep -E "seed|PASS|FAIL|passed|failed|Error" $O/pin.txt | tail -60
exit $rc
