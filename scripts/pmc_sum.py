"""Per-kernel mean of rocprofv3 --pmc counters: python scripts/pmc_sum.py <dir with p1/ p2/ ...> [substr]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "psamd"
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if sub not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(ids[k])
        print(os.path.basename(os.path.dirname(f)), k, n, {c: round(x / n) for c, x in sorted(v.items())})
