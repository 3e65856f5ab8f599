set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05q
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05q/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r05q/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05q/gpu_tests.txt
TAG=r05q VARIANTS="k1head base" timeout -k 10 600 bash tools/ab_headline.sh > gpurun_out/r05q/ab.txt 2>&1; cat gpurun_out/r05q/ab.txt
