"""Busy / overlap of a rocprofv3 rocpd database (results.db) over a steady-state window:
the dispatches between the a-th and b-th launch of a marker kernel (one per step).

    python scripts/kbusy_db.py results.db [marker=tp_fwd_bwd] [a=20] [b=80]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "tp_fwd_bwd"
a = int(sys.argv[3]) if len(sys.argv) > 3 else 20
b = int(sys.argv[4]) if len(sys.argv) > 4 else 80
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
ms = [r[1] for r in rows if marker in r[0]]
lo, hi = ms[a], ms[b]
steps = b - a
win = [r for r in rows if lo <= r[1] < hi]
iv = sorted((max(r[1], lo), min(r[2], hi)) for r in win)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
tot = sum(e - s for s, e in iv)
span = hi - lo
print(f"{steps} steps: {span / steps / 1e3:.1f} us/step  busy {busy / span:.1%}  "
      f"kernel-sum {tot / steps / 1e3:.1f} us/step  concurrency {tot / busy:.2f}")
agg = defaultdict(lambda: [0, 0])
for r in win:
    k = r[0].replace("psamd::", "").replace("void ", "").split("(")[0]
    agg[k][0] += 1
    agg[k][1] += r[2] - r[1]
for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:18]:
    print(f"  {n / steps:5.2f}/step {d / steps / 1e3:8.1f} us/step  {k[:90]}")
