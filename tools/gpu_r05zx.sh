set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zx; mkdir -p $O
MGPU_BENCH_REHEARSAL=1 timeout -k 10 1000 python -u bench.py --gpus 2 --supp-out $O/supp2.json > $O/bench2.json 2> $O/bench2.err || { grep -v amdgpu.ids $O/bench2.err | tail -30; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms/step', d['ms_per_step'], 'allocs', d['tls4_oa_tree'].get('timed_device_allocations'), d['tls4_oa_rel_tree'].get('timed_device_allocations'))
print(d.get('supplementary'))
"
