set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --supp-out $O/supp1.json > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
tail -3 $O/gpu_tests.txt; python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05h/bench1.json'))
print(d['value'], d['ms_per_step'], d['kernels'], d['tls4_oa_tree'].get('nodes_per_s'), d.get('tls4_oa_rel_tree'))
PY
