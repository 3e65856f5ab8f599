#!/bin/bash
# Persistent K1: time the headline batch with a wave refilling after 1 / 8 /
# 16 / 32 idle lanes (MGPU_FBBT_REFILL); run on the GPU box from the repo root.
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fbbt_gpu.py > gpurun_out/t_refill.log 2>&1 || exit $?
for r in 1 8 16 32; do
  MGPU_FBBT_REFILL=$r timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-glob --no-knapsack --no-convex > gpurun_out/b_refill$r.json 2> gpurun_out/b_refill$r.err || exit $?
done
