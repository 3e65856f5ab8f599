"""Summarise a tools/prof_run.sh run into profiles/<tag>_*.

Copies rocprofv3's kernel stats CSV and writes <tag>_pmc.json with, per
engine kernel, the average duration (kernel trace) and the HBM traffic per
launch from the PMC passes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half of a wide stream on gfx950;
our access widths are uncalibrated)."""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def short(name):
    for k in ('fbbt_linear_kernel', 'fbbt_linear_persist', 'fbbt_group_kernel', 'lp_pfi_kernel',
              'lp_dual_kernel', 'pfi_t0_kernel',
              'node_decide_kernel', 'lp_large_kernel',
              'fbbt_quad_kernel',
              'obbt'):
        if k in name:
            return k
    return None


def main(src, tag, bench_args):
    out = os.path.join(ROOT, 'profiles')
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                os.path.join(out, f'{tag}_kernel_stats.csv'))
    # keep, per kernel, only the launches of the dominant grid size (the
    # batch launches; e.g. drops the B=1 root LP solve)
    dur = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_trace.csv'))):
        k = short(r['Kernel_Name'])
        if k:
            dur[k][r['Grid_Size_X']].append(
                (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    grid = {k: max(v, key=lambda g: len(v[g])) for k, v in dur.items()}
    dur = {k: v[grid[k]] for k, v in dur.items()}
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for part in ('fetch', 'write'):
        f = os.path.join(src, part, 'run_counter_collection.csv')
        for r in csv.DictReader(open(f)):
            k = short(r['Kernel_Name'])
            if k and str(r['Grid_Size']) == str(grid.get(k)):
                ctr[k][r['Counter_Name']].append(float(r['Counter_Value']))
    # the bench's headline since round 3 is the tree round (bench.py
    # tree_rounds); bench.pmc_traffic matches summaries by this key
    sys.path.insert(0, ROOT)
    from minotaur_amd.build import source_digest
    res = {"bench_args": bench_args, "workload": "tree_rounds",
           "source_digest": source_digest(), "kernels": {}}
    for k in sorted(set(dur) | set(ctr)):
        d = dur.get(k, [])
        fe = ctr[k].get('FETCH_SIZE', [])
        wr = ctr[k].get('WRITE_SIZE', [])
        fe_kb = sum(fe) / len(fe) if fe else None
        wr_kb = sum(wr) / len(wr) if wr else None
        res["kernels"][k] = {
            "grid_size": grid.get(k),
            "launches": len(d),
            "avg_ms": sum(d) / len(d) if d else None,
            "fetch_size_kb": fe_kb,
            "write_size_kb": wr_kb,
            "hbm_bytes_per_launch": (2 * fe_kb + wr_kb) * 1024 if fe and wr else None,
        }
    with open(os.path.join(out, f'{tag}_pmc.json'), 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else '')
