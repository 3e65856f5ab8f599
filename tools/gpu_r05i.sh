set -o pipefail
TAG=r05i VARIANTS="base nofuse" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05i.txt 2>&1; cat gpurun_out/r05i.txt
