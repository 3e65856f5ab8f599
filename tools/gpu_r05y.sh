set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 900 python -u bench.py --supp-out $O/bench_supplementary.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
l=[x for x in open('$O/bench.json') if x.startswith('{')][-1]
d=json.loads(l)
print(d['value'], d['ms_per_step'], len(l))
print(json.dumps(d['cpu_baseline'], indent=1)[:2500])
"
