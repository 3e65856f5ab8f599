set -o pipefail
TAG=r05f VARIANTS="base w12 r8 g2" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05f.txt 2>&1; cat gpurun_out/r05f.txt
