set -o pipefail
O=gpurun_out/r03_g30
mkdir -p $O

timeout -k 10 300 python -u tools/b1_timing.py > $O/b1t.txt 2>&1
rc=$?
tail -c 300 $O/b1t.txt
exit $rc
