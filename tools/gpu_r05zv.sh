set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zv; mkdir -p $O
MGPU_BENCH_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed --supp-out $O/supp2.json > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms/step', d['ms_per_step'], 'scaling', d['scaling'], 'rccl_ms', d.get('rccl_ms_total'))
"
python3 -c "
import json
d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1])
print('allocs', d['tls4_oa_tree'].get('timed_device_allocations'), d['tls4_oa_rel_tree'].get('timed_device_allocations'))
"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_comm_gpu.py tests/test_bnb_gpu.py tests/test_bnb_rel_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
