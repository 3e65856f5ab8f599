set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qp_gpu.py tests/test_qp_tree_gpu.py > gpurun_out/r05x/tests.txt 2>&1 || { tail -30 gpurun_out/r05x/tests.txt; exit 1; }
tail -2 gpurun_out/r05x/tests.txt
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-bnb --no-convex --no-knapsack --no-glob --no-fixed --no-oa-tree --supp-out gpurun_out/r05x/supp.json > gpurun_out/r05x/bench.json 2> gpurun_out/r05x/bench.err || { tail -20 gpurun_out/r05x/bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/r05x/supp.json'))['qp_relaxation']
print(json.dumps({k: d[k] for k in ('qp_per_s','ms_per_batch','roofline','kernels','whole_solve_roofline')}, indent=1))
"
