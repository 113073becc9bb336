"""Per-kernel medians from a rocprofv3 kernel_trace.csv: calls, median / mean / min us."""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
d = defaultdict(list)
for x in rows:
    d[x["Kernel_Name"]].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
tot = sorted(d.items(), key=lambda kv: -sum(kv[1]))
for name, v in tot[:n]:
    print(f"{len(v):6d} calls  total {sum(v):10.1f} us  median {statistics.median(v):8.1f}  "
          f"mean {statistics.mean(v):8.1f}  min {min(v):8.1f}  {name[:90]}")
