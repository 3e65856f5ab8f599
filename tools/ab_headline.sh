#!/bin/bash
# A/B of libmgpu variants on the headline (run on the GPU box from the repo
# root): VARIANTS="base name1 name2 ..." (base = minotaur_amd/libmgpu.so,
# others tools/_stamps/<name>/libmgpu.so from tools/variant_build.py; name+VAR=1
# adds environment settings); each
# runs the headline twice, one JSON summary line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-ab}; mkdir -p $O; cd $R; export TMPDIR=/tmp
ARGS=${ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-bnb --no-qp --no-convex --no-knapsack --no-glob --no-fixed}
for rep in 1 2; do
for v in ${VARIANTS:-base}; do
  # a variant is a library name, optionally followed by +VAR=value env settings
  lib=${v%%+*}; envs=""; [ "$lib" != "$v" ] && envs=$(echo "${v#*+}" | tr '+' ' ')
  if [ "$lib" = base ]; then L=$R/minotaur_amd/libmgpu.so; else L=$R/tools/_stamps/$lib/libmgpu.so; fi
  env $envs MGPU_LIB=$L timeout -k 10 300 python -u bench.py $ARGS --supp-out $O/${v}_supp.json > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$O/$v.json') if l.startswith('{')][-1])
k = d['kernels']
print('$v', 'rep $rep', round(d['value']/1e6, 3), 'M nodes/s', round(d['ms_per_step'], 2), 'ms/step', 'K3P', k['lp_pfi']['ms'], 'ovf', k['lp_pfi']['overflow_resolve_ms'], 'K1', k['fbbt']['ms'], 'piv', k['lp_pfi']['pivots_per_solve'], 'tree', d['tls4_oa_tree']['nodes_per_s'])
" || exit 1
done
done
echo AB DONE
