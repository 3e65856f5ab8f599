set -o pipefail
O=gpurun_out/r03_g7
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo done
