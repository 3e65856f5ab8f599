"""Probe: reliability-branching trees on the bench instances, one line per
round (nodes, strong-branching LPs, seconds) so slow phases show up."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

from minotaur_amd.problem import LinProblem, random_mkp  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def run(ctx, p, B, order, warm, brancher, max_s=60.0):
    ctx.load(p)
    ctx.bnb_config(order, warm)
    ctx.bnb_brancher(brancher)
    ctx.bnb_init(1 << 23)
    t0 = time.perf_counter()
    r = 0
    while True:
        t = time.perf_counter()
        st = ctx.bnb_round(B)
        r += 1
        dt = time.perf_counter() - t
        if r <= 30 or r % 10 == 0 or st.open == 0:
            print(f"  round {r} batch {st.last_batch} open {st.open} nodes {st.nodes} "
                  f"sb_lps {st.sb_lps} {dt * 1e3:.1f} ms", flush=True)
        if st.open == 0 or time.perf_counter() - t0 > max_s:
            break
    print(f"{p.name} B={B} order={order} warm={warm} br={brancher}: nodes {st.nodes} "
          f"lps {st.lps} sb {st.sb_lps} inc {st.incumbent} "
          f"{time.perf_counter() - t0:.2f}s", flush=True)


if __name__ == '__main__':
    ctx = Context(0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    tls = LinProblem.load(os.path.join(ROOT, 'minotaur_amd', 'instances', 'tls4_lin.npz'))
    run(ctx, tls, B, 1, 0, 1)
    run(ctx, random_mkp(1, 60, 8), B, 1, 1, 1)
    ctx.close()
