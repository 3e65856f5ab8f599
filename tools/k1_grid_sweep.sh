#!/bin/bash
# Persistent K1: time the headline batch over the persistent grid size
# (MGPU_FBBT_WAVES) and the waves per workgroup (MGPU_FBBT_WG); run on the
# GPU box from the repo root.
export TMPDIR=/tmp
for w in 1536 2048 2560 3072; do
  MGPU_FBBT_WAVES=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-glob --no-knapsack --no-convex > gpurun_out/b_grid$w.json 2> gpurun_out/b_grid$w.err || exit $?
done
MGPU_FBBT_WG=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-glob --no-knapsack --no-convex > gpurun_out/b_gridwg1.json 2> gpurun_out/b_gridwg1.err || exit $?
