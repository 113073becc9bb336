"""Which kernels run beside a target kernel: for every dispatch of ``target`` in the
steady-state window (the a-th .. b-th launch of the marker), the time each other
kernel overlaps it, averaged per dispatch, plus the target's mean duration.

    python scripts/koverlap_db.py results.db target [marker=tp_fwd_bwd] [a=40] [b=100]"""
import sqlite3
import sys
from collections import defaultdict

db, target = sys.argv[1], sys.argv[2]
marker = sys.argv[3] if len(sys.argv) > 3 else "tp_fwd_bwd"
a = int(sys.argv[4]) if len(sys.argv) > 4 else 40
b = int(sys.argv[5]) if len(sys.argv) > 5 else 100
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
ms = [r[1] for r in rows if marker in r[0]]
lo, hi = ms[a], ms[b]
win = [r for r in rows if lo <= r[1] < hi]
short = lambda n: n.replace("psamd::", "").replace("void ", "").split("(")[0]  # noqa: E731
tg = [r for r in win if target in r[0]]
ov = defaultdict(float)
alone = 0.0
for t in tg:
    segs = []
    for r in win:
        if r is t:
            continue
        s, e = max(r[1], t[1]), min(r[2], t[2])
        if e > s:
            ov[short(r[0])] += e - s
            segs.append((s, e))
    segs.sort()
    cov, cs, ce = 0, None, None
    for s, e in segs:
        if cs is None or s > ce:
            if cs is not None:
                cov += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        cov += ce - cs
    alone += (t[2] - t[1]) - cov
n = len(tg)
dur = sum(t[2] - t[1] for t in tg) / n
print(f"{short(tg[0][0])}: {n} dispatches, {dur / 1e3:.1f} us mean, {alone / n / 1e3:.1f} us alone")
for k, v in sorted(ov.items(), key=lambda kv: -kv[1]):
    print(f"  beside {k[:70]:70s} {v / n / 1e3:7.1f} us")
