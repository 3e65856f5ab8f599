"""Prints the scipy-HiGHS MILP optima of bench.py's convex batch (config 5:
knapsack outer-approximation LPs, f terms, N = 3 f) — the values bench.py
checks its GPU trees against (run in the build container; HiGHS is the
checker, never part of the measured path)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402
from minotaur_amd.problem import knapsack_oa  # noqa: E402

for f in (16, 20, 24, 28):
    p = knapsack_oa(f=f, N=3 * f)
    st, obj = oracle.highs_milp(p)
    print(f"({f}, {3 * f}, {obj!r}),  # m = {p.m}, status {st}")
