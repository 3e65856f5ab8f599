#!/bin/bash
# SQ counter passes over the LP step alone (tools/lp_pfi_probe.py, one mode),
# one rocprofv3 run per pass.  Usage: PROBE_MODES=0:24 bash tools/sq_lp.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sqlp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INST_LEVEL_LDS SQ_IFETCH_LEVEL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/lp_pfi_probe.py > $OUT/p$i.txt 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "sq passes done"
