#!/usr/bin/env python3
"""Per-call durations of the kernels whose name contains a pattern, from a rocprofv3
rocpd SQLite: usage rocpd_calls.py <results.db> <pattern> [last N calls]. Prints count,
median, mean, min, max (us) of the last N calls (steady state after setup calls)."""
import sqlite3
import statistics
import sys


def main():
    db, pat = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x from kernels where name like ? order by start",
                     (f"%{pat}%",)).fetchall()
    if last:
        rows = rows[-last:]
    d = [r[1] / 1e3 for r in rows]
    if not d:
        print("no calls")
        return
    print(f"{pat}: {len(d)} calls, median {statistics.median(d):.1f} us, mean "
          f"{statistics.mean(d):.1f}, min {min(d):.1f}, max {max(d):.1f}  ({rows[-1][0][:60]})")


if __name__ == "__main__":
    main()
