set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
TAG=r05v VARIANTS="base k1cls" timeout -k 10 600 bash tools/ab_headline.sh > gpurun_out/r05v/ab.txt 2>&1; cat gpurun_out/r05v/ab.txt
