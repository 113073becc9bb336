#!/usr/bin/env python3
"""Print the per-kernel summary of a rocprofv3 SQLite (rocpd) output:
calls, total us, avg us, % -- usage: rocpd_top.py <results.db> [N] [steps]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels limit ?", (n,)).fetchall()
    for name, calls, tot, avg, pct in rows:
        per = f"{tot / steps:9.1f} us/step" if steps else ""
        print(f"{calls:6d} {tot:10.1f} us {avg:9.2f} us avg {pct:5.1f}% {per}  {name[:110]}")


if __name__ == "__main__":
    main()
