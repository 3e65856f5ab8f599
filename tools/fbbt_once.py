"""Runs K1 alone (tls4-lin, B nodes, variant/npw from argv) a few times: a
target for rocprofv3 counter passes.  python tools/fbbt_once.py B variant
(MGPU_FBBT_INST names the instance, default tls4_lin; MGPU_FBBT_INC the
incumbent, default 1.2)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd.problem import LinProblem, random_boxes  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', os.environ.get('MGPU_FBBT_INST', 'tls4_lin') + '.npz'))
ctx = Context(0)
ctx.load(p)
dev = torch.device('cuda', 0)
LB, UB = random_boxes(p, B, 20261015)
lb = torch.from_numpy(LB).to(dev)
ub = torch.from_numpy(UB).to(dev)
olb, oub = torch.empty_like(lb), torch.empty_like(ub)
inf = torch.zeros(B, dtype=torch.int32, device=dev)
nm = torch.zeros(B, dtype=torch.int32, device=dev)
ctx.set_fbbt_variant(variant)
for _ in range(3):
    ctx.fbbt_dev(lb, ub, olb, oub, inf, nm, float(os.environ.get('MGPU_FBBT_INC', '1.2')))
    ctx.sync()
    print(f"fbbt B={B} variant={variant} {ctx.last_kernel_ms('fbbt'):.3f} ms", flush=True)
