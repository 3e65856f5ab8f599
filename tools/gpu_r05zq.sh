set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/r05zq; mkdir -p $O
for v in base pair; do
  if [ $v = base ]; then L=$(pwd)/tools/_stamps/k1gbase/libmgpu.so; else L=$(pwd)/minotaur_amd/libmgpu.so; fi
  MGPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/oa_tree_one.py > $O/$v.log 2>&1 || exit 1
  rm -f $O/$v/run_kernel_trace.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'fbbt_group' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs'])/1e6, 3), 'ms total', round(float(r['AverageNs'])/1e3, 1), 'us avg')
"
done
