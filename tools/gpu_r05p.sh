set -o pipefail
export TMPDIR=/tmp
TAG=r05p VARIANTS="k1head base+MGPU_FBBT_NOSLOTS=1 k1unr+MGPU_FBBT_NOSLOTS=1" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05p.txt 2>&1; cat gpurun_out/r05p.txt
