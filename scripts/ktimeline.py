"""Timeline of the last N kernel dispatches of a rocprofv3 kernel_trace.csv: start offset,
duration, gap since the previous kernel on the same queue, queue id, short name."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
last_end = {}
for x in rows:
    s, e, q = int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Queue_Id"]
    gap = (s - last_end[q]) / 1e3 if q in last_end else float("nan")
    last_end[q] = e
    name = x["Kernel_Name"].replace("psamd::", "").replace("void ", "")
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:7.1f}  q{q:>2}  {name[:70]}")
