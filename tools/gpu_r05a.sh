set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tls4_oa_gpu.py -k "small_eta" -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
MGPU_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 8 --warmup 2 --batch 131072 --lb-every 4 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --no-oa-tree --supp-out $O/reh_supp.json > $O/rehearse2.json 2> $O/rehearse2.err || { tail -30 $O/rehearse2.err; exit 1; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --supp-out $O/supp1.json > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
tail -3 $O/tests.txt; head -c 1500 $O/rehearse2.json; echo; head -c 1500 $O/bench1.json
