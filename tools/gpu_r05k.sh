# SQ + traffic counters over K1 alone (tls4-OA, 524 288 nodes, persistent
# variant), with and without the bit slots
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05k
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MGPU_FBBT_INST=tls4_oa
for V in slots noslots; do
  i=0; mkdir -p $OUT/$V
  for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
              "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    if [ $V = noslots ]; then export MGPU_FBBT_NOSLOTS=1; else unset MGPU_FBBT_NOSLOTS; fi
    timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-trace -d $OUT/$V/p$i -o run --output-format csv -- python3 $R/tools/fbbt_once.py 524288 3 > $OUT/$V/p$i.txt 2>&1 || { echo "pass $V $i failed"; tail $OUT/$V/p$i.txt; exit 1; }
    tail -1 $OUT/$V/p$i.txt
  done
done
echo "sq passes done"
