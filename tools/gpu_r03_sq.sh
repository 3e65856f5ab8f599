#!/bin/bash
# SQ counter passes over the headline tree rounds (K3P, K1), one rocprofv3 run per pass.
set -o pipefail
TAG=${TAG:-r03d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG/sq
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed"
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INST_LEVEL_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PASS --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo "sq passes done"
