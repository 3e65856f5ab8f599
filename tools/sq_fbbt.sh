#!/bin/bash
# SQ counter passes over K1 alone (tools/fbbt_once.py), one pass per run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sqf
ARGS=${FBBT_ARGS:-65536 1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" \
            "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SENDMSG SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/fbbt_once.py $ARGS > $OUT/p$i.txt 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "sq passes done"
