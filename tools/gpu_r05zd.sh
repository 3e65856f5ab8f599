set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zd
TAG=r05zd VARIANTS="base k1o4" timeout -k 10 600 bash tools/ab_headline.sh > gpurun_out/r05zd/ab.txt 2>&1; cat gpurun_out/r05zd/ab.txt
