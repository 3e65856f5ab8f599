set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lp_pfi_gpu.py tests/test_lp_path_gpu.py tests/test_tls4_oa_gpu.py tests/test_bnb_gpu.py -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --supp-out $O/supp1.json > $O/bench1.json 2> $O/bench1.err || { tail -30 $O/bench1.err; exit 1; }
tail -3 $O/tests.txt; python - <<'PY'
import json
d=json.load(open('gpurun_out/r05c/bench1.json'))
print(d['value'], d['ms_per_step'], d['kernels'], d['tls4_oa_tree'].get('nodes_per_s'), d['tls4_oa_tree'].get('seconds'))
PY
