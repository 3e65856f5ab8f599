#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks on device 0 over gloo
# (RCCL refuses a shared device): the headline's per-round all-reduce and the
# complete trees with bound-aware rebalancing (pick / device rows / all-to-all).
set -o pipefail
TAG=${TAG:-r03b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
MGPU_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 \
  --batch 65536 --no-cpu-baseline --no-fixed --no-convex --no-qp --no-knapsack --no-glob \
  > $O/rehearse2.json 2> $O/rehearse2.err || exit $?
echo done
