set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_simplex_cuts_gpu.py tests/test_integration_gpu.py > $O/gpu_tests.txt 2>&1 || { tail -60 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
MGPU_BENCH_REHEARSAL=1 timeout -k 10 900 python -u bench.py --gpus 2 --supp-out $O/supp2.json > $O/bench2.json 2> $O/bench2.err || { grep -v amdgpu.ids $O/bench2.err | tail -30; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms/step', d['ms_per_step'])
print(d.get('tree_rounds', {}).get('device_allocs_timed'), d['tls4_oa_tree'].get('timed_device_allocations'), d['tls4_oa_rel_tree'].get('timed_device_allocations'))
"
