"""Kernel time per name from a rocprofv3 --kernel-trace database (the second
half of the run: after the largest launch gap in its middle third, i.e. the
timed solve after its warm-up), plus the gaps between kernels."""
import re
import sqlite3
import sys
from collections import defaultdict


def main(path, top=25):
    db = sqlite3.connect(path)
    rows = list(db.execute("select name, start, end from kernels order by start"))

    def nm(s):
        s = s.replace('(anonymous namespace)::', '')
        s = re.sub(r'^void ', '', s)
        i = s.find('(')
        return (s[:i] if i > 0 else s)[:70]
    st = [r[1] for r in rows]
    en = [r[2] for r in rows]
    n = len(rows)
    gaps = [(st[i + 1] - en[i], i) for i in range(n // 3, 2 * n // 3)]
    i0 = max(gaps)[1] + 1
    tot, cnt = defaultdict(float), defaultdict(int)
    for i in range(i0, n):
        tot[nm(rows[i][0])] += (en[i] - st[i]) / 1e6
        cnt[nm(rows[i][0])] += 1
    span = (en[-1] - st[i0]) / 1e6
    gap = sum(max(0, st[i + 1] - en[i]) for i in range(i0, n - 1)) / 1e6
    print(f"span {span:.2f} ms, kernels {sum(tot.values()):.2f} ms, gaps {gap:.2f} ms, "
          f"launches {n - i0}")
    for k, v in sorted(tot.items(), key=lambda t: -t[1])[:top]:
        print(f"{v:8.3f} ms {cnt[k]:5d}  {k}")


if __name__ == '__main__':
    main(sys.argv[1])
