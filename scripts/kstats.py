"""Summarise a rocprofv3 kernel_stats.csv: per-step microseconds (total / steps)."""
import csv
import sys

f, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = list(csv.DictReader(open(f)))
for x in rows[:n]:
    print(f"{int(x['Calls']):5d} {int(x['TotalDurationNs']) / 1e3 / steps:9.1f} us/step "
          f"{float(x['AverageNs']) / 1e3:9.1f} us avg  {x['Name'][:100]}")
