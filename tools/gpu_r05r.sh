# K5 counters: MFMA f64 instructions / ops / busy cycles per
# qp_* kernel, clock, and the f64 VALU mix; one pass per run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05r
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/qp_once.py 1024 > $OUT/p$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.txt; exit 1; }
  grep "^qp B" $OUT/p$i.txt | tail -1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/tools/qp_once.py 1024 > $OUT/stats.txt 2>&1 || { echo "stats failed"; exit 1; }
echo "k5 passes done"
