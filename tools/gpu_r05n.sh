set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05n
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fbbt_gpu.py tests/test_tls4_oa_gpu.py > gpurun_out/r05n_tests.txt 2>&1 || { tail -30 gpurun_out/r05n_tests.txt; exit 1; }
tail -2 gpurun_out/r05n_tests.txt
TAG=r05n VARIANTS="base base+MGPU_FBBT_OCC=2 base+MGPU_FBBT_NOSLOTS=1" timeout -k 10 1000 bash tools/ab_headline.sh > gpurun_out/r05n.txt 2>&1; cat gpurun_out/r05n.txt
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r05n/counters_list.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*" $R/gpurun_out/r05n/counters_list.txt | sort -u | head
for V in slots noslots; do
  if [ $V = noslots ]; then export MGPU_FBBT_NOSLOTS=1; else unset MGPU_FBBT_NOSLOTS; fi
  MGPU_FBBT_INST=tls4_oa timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --kernel-trace -d $R/gpurun_out/r05n/ic_$V -o run --output-format csv -- python3 $R/tools/fbbt_once.py 524288 3 > $R/gpurun_out/r05n/ic_$V.txt 2>&1 || { echo "icache pass failed"; tail -5 $R/gpurun_out/r05n/ic_$V.txt; exit 0; }
  tail -1 $R/gpurun_out/r05n/ic_$V.txt
done
