import os, sys, time, math
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import numpy as np, torch
from minotaur_amd.problem import LinProblem, random_boxes
from minotaur_amd.runtime import Context, WarmStart
p = LinProblem.load('minotaur_amd/instances/tls4_lin.npz')
B = 65536
LB, UB = random_boxes(p, B, 1)
dev = torch.device('cuda', 0)
ctx = Context(0); ctx.load(p); root, wsh = ctx.root_solve()
s = torch.cuda.Stream()
ctx.set_stream(s.cuda_stream)
print('stream', s.cuda_stream, torch.cuda.current_stream().cuda_stream)
with torch.cuda.stream(s):
    ws = WarmStart(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (wsh.head, wsh.st, wsh.d, wsh.binv)))
    lb0 = torch.from_numpy(LB).to(dev); ub0 = torch.from_numpy(UB).to(dev)
    lb1 = torch.empty_like(lb0); ub1 = torch.empty_like(ub0)
    I = lambda: torch.zeros(B, dtype=torch.int32, device=dev)
    infeas, nmods, status, iters, decision = I(), I(), I(), I(), I()
    obj = torch.zeros(B, dtype=torch.float64, device=dev); cand = torch.zeros_like(obj)
    x = torch.zeros((B, p.n), dtype=torch.float64, device=dev)
    s.synchronize()
    for it in range(6):
        t = [time.perf_counter()]
        ctx.fbbt_dev(lb0, ub0, lb1, ub1, infeas, nmods, math.inf); t.append(time.perf_counter())
        ctx.lp_solve_dev(lb1, ub1, status, obj, iters, ws=ws, skip=infeas, x=x); t.append(time.perf_counter())
        ctx.node_decide_dev(status, obj, x, decision, math.inf, fbbt_infeas=infeas, cand_obj=cand); t.append(time.perf_counter())
        best = cand.min(); t.append(time.perf_counter())
        b = best.item(); t.append(time.perf_counter())
        f = ctx.last_kernel_ms('fbbt'); l = ctx.last_kernel_ms('lp'); t.append(time.perf_counter())
        print('host ms', [round(1e3*(t[i+1]-t[i]),3) for i in range(len(t)-1)], 'kern', round(f,3), round(l,3))
    for v in (1, 2):
        ctx.set_fbbt_variant(v)
        for it in range(3):
            t0 = time.perf_counter(); ctx.fbbt_dev(lb0, ub0, lb1, ub1, infeas, nmods, math.inf); s.synchronize()
            print('variant', v, 'wall', round(1e3*(time.perf_counter()-t0),3), 'kern', round(ctx.last_kernel_ms('fbbt'),3))
