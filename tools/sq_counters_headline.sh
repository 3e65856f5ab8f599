set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06al; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES --kernel-trace -d $O/sq -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --batch 524288 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --no-oa-tree > $O/bench_sq.log 2>&1 || { tail -20 $O/bench_sq.log; exit 1; }
find $O/sq -name "*counter_collection.csv" | head -3
