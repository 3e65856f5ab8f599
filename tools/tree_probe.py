"""Config 2's complete tree (tls4-OA, depth-first, MaxVio, warm 2) at a given
batch: rounds, seconds, nodes/s and the per-round wall time, to see where a
launch-bound tree's rounds go (run it under rocprofv3 --kernel-trace for the
kernels' share).

    python tools/tree_probe.py [batch ...]
"""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from minotaur_amd.problem import LinProblem
    from minotaur_amd.runtime import Context
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    ctx = Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    ctx.load(p)
    warm = int(os.environ.get('PROBE_WARM', '2'))
    for B in [int(a) for a in sys.argv[1:]] or [16384]:
        for rep in range(3):
            ctx.bnb_config(0, warm)
            ctx.bnb_brancher(0)
            ctx.bnb_init(1 << 21)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ts, inc, st = [], math.inf, None
            while True:
                st = ctx.bnb_round(B, inc)
                inc = st.incumbent
                ts.append(time.perf_counter())
                if st.open == 0:
                    break
            el = time.perf_counter() - t0
            d = [1e3 * (b - a) for a, b in zip([t0] + ts[:-1], ts)]
            print(f"batch {B} rep {rep}: {st.nodes} nodes {st.rounds} rounds {el * 1e3:.1f} ms "
                  f"{st.nodes / el / 1e6:.2f} M nodes/s pivots/LP {st.pivots / max(st.lps, 1):.2f} "
                  f"inc {inc} round ms min {min(d):.3f} med {sorted(d)[len(d) // 2]:.3f} "
                  f"max {max(d):.3f}", flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
