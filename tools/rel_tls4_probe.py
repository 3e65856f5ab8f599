"""Probe: the tls4-OA reliability tree (the reference's default brancher) at
several batch sizes on the GPU: rounds, nodes, strong-branching LPs and the
time per round, to see where time-to-proof goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

from minotaur_amd.problem import LinProblem  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def run(ctx, p, B, order, warm, verbose=False):
    ctx.load(p)
    ctx.bnb_config(order, warm)
    ctx.bnb_brancher(1)
    ctx.bnb_init(1 << 20)
    t0 = time.perf_counter()
    per = []
    while True:
        t = time.perf_counter()
        st = ctx.bnb_round(B)
        per.append((time.perf_counter() - t, st.last_batch, st.sb_lps))
        if st.open == 0:
            break
    el = time.perf_counter() - t0
    print(f"B={B} order={order} warm={warm}: rounds {st.rounds} nodes {st.nodes} lps {st.lps} "
          f"sb {st.sb_lps} inc {st.incumbent} {el * 1e3:.1f} ms", flush=True)
    if verbose:
        prev = 0
        for k, (dt, nb, sb) in enumerate(per):
            print(f"   round {k + 1}: batch {nb} sb+{sb - prev} {dt * 1e3:.2f} ms")
            prev = sb


if __name__ == '__main__':
    ctx = Context(0)
    p = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_oa.npz'))
    for B in (131072, 131072, 1024, 256, 64, 16):
        run(ctx, p, B, 1, 0, verbose=(B == 1024))
    run(ctx, p, 1, 2, 1)
    ctx.close()
