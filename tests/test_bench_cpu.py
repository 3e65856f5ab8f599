"""CPU: bench.py's PMC traffic lookup (bench.py:73).  The
roofline's HBM traffic comes only from a summary measured at the same batch
and eta cap, and is marked stale when the summary's engine-source digest
differs from the sources in the tree."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)


def _summary(path, args, digest, bytes_):
    d = {"bench_args": args, "workload": "tree_rounds",
         "kernels": {"lp_pfi_kernel": {"hbm_bytes_per_launch": bytes_}}}
    if digest is not None:
        d["source_digest"] = digest
    with open(path, 'w') as fh:
        json.dump(d, fh)


def test_pmc_traffic_matches_batch_cap_and_digest(tmp_path, monkeypatch):
    import bench
    from minotaur_amd.build import source_digest
    prof = tmp_path / 'profiles'
    prof.mkdir()
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    cur = source_digest()
    _summary(prof / 'r01_pmc.json', '--batch 1024', None, 1.0)
    _summary(prof / 'r02_pmc.json', '--batch 1024 --eta-cap 24', cur, 2.0)
    _summary(prof / 'r03_pmc.json', '--batch 2048', 'not-this-tree', 3.0)
    _summary(prof / 'r04_pmc.json', '--batch 4096', cur, 4.0)
    cap = bench.PFI_DEFAULT
    # default cap, batch 1024: r02 is at another cap, r01 predates digests
    assert bench.pmc_traffic('lp_pfi', 1024, cap, tree=True) == (1.0, 'r01_pmc.json', None)
    assert bench.pmc_traffic('lp_pfi', 1024, 24, tree=True) == (2.0, 'r02_pmc.json', True)
    assert bench.pmc_traffic('lp_pfi', 2048, cap, tree=True) == (3.0, 'r03_pmc.json', False)
    assert bench.pmc_traffic('lp_pfi', 4096, cap, tree=True) == (4.0, 'r04_pmc.json', True)
    assert bench.pmc_traffic('lp_pfi', 8192, cap, tree=True) == (None, None, None)


def test_source_digest_tracks_engine_sources():
    from minotaur_amd import build
    d = build.source_digest()
    assert len(d) == 16 and d == build.source_digest()
