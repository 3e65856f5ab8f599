"""GPU tree-search throughput of the batched B&B driver on a weak-bound
MILP (multi-dimensional knapsack): nodes/s per round and to completion."""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT)
from minotaur_amd.problem import random_mkp  # noqa: E402
from minotaur_amd.runtime import Context  # noqa: E402


def main():
    ctx = Context(0)
    for (n, m, B) in [(30, 5, 4096), (50, 5, 16384), (50, 5, 65536), (60, 8, 65536)]:
        p = random_mkp(1, n, m)
        ctx.load(p)
        ctx.bnb_init(1 << 22)
        t0 = time.perf_counter()
        st = None
        rounds = 0
        while True:
            st = ctx.bnb_round(B)
            rounds += 1
            if st.open == 0 or time.perf_counter() - t0 > 20:
                break
        dt = time.perf_counter() - t0
        print(f"mkp n={n} m={m} B={B}: {st.nodes} nodes in {dt:.2f}s ({rounds} rounds) "
              f"{st.nodes / dt / 1e6:.2f} M nodes/s  open={st.open} inc={st.incumbent} "
              f"dec={list(st.ndec)}", flush=True)


if __name__ == '__main__':
    main()
