"""Per-kernel totals of a rocprofv3 rocpd database between the a-th and b-th launch of a
marker kernel: count, total us, median and max per launch.

    python scripts/kbreak_db.py results.db [marker=bcd_objective] [a=1] [b=2]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "bcd_objective"
a = int(sys.argv[3]) if len(sys.argv) > 3 else 1
b = int(sys.argv[4]) if len(sys.argv) > 4 else 2
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
ms = [r[1] for r in rows if marker in r[0]]
lo, hi = ms[a], ms[b]
d = defaultdict(list)
for n, s, e in rows:
    if lo <= s < hi:
        d[n[:80]].append(e - s)
tot = sum(sum(v) for v in d.values())
print(f"window {(hi - lo) / 1e3:.1f} us, kernel sum {tot / 1e3:.1f} us")
for n, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    v.sort()
    print(f"{len(v):6d} {sum(v) / 1e3:9.1f} us  med {v[len(v) // 2] / 1e3:7.2f} max {v[-1] / 1e3:8.1f}  {n}")
