"""How many tls4-lin bench nodes run each FBBT sweep, and how many rows they
tighten there (C restatement, one thread): sizes the wave-compaction idea
for K1."""
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402

p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
LB, UB = random_boxes(p, 8192, 20261015)
lib = oracle.lib()
lib.orc_fbbt_stats.restype = ctypes.POINTER(ctypes.c_long)
for inc in (None, 11.3):
    st = lib.orc_fbbt_stats(1)
    f = oracle.linear_fbbt(p, LB, UB, inc)
    runs = [st[k] for k in range(16)]
    rows = [st[16 + k] for k in range(16)]
    lib.orc_fbbt_stats(0)
    print(f"incumbent {inc}: nodes per sweep {runs[:10]}")
    print(f"   rows tightened per sweep {rows[:10]}  total rows {sum(rows)}  "
          f"rows in sweeps >= 3: {sum(rows[2:]) / max(1, sum(rows)):.2%}")
