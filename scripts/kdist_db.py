"""Per-kernel duration distribution (min / p25 / median, us) of a rocprofv3 rocpd database
over its last three quarters of dispatches.

    python scripts/kdist_db.py results.db [top=8]"""
import sqlite3
import statistics as st
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = c.execute("select name, start, end from kernels order by start").fetchall()
d = defaultdict(list)
for n, s, e in rows[len(rows) // 4:]:
    d[n.replace("psamd::", "").replace("void ", "").split("(")[0]].append((e - s) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    v = sorted(v)
    print(f"  {k[:44]:44s} n={len(v):4d} min={v[0]:7.1f} p25={v[len(v) // 4]:7.1f} "
          f"med={st.median(v):7.1f}")
