#!/bin/bash
# End-of-round checks on the GPU box (from the repo root): the whole -m gpu
# suite, smoke(), then the default bench line.  TAG names the output dir.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06zj}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d = json.loads([l for l in open('$O/bench.json') if l.startswith('{')][-1])
print('value', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'roofline', d.get('roofline'))
print('cpu_baseline', d.get('cpu_baseline'))
"
