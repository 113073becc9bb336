"""Busy / overlap summary of a rocprofv3 kernel_trace.csv over its last N dispatches:
wall span, union of kernel-busy time (any kernel running), idle time, sum of kernel
durations and their average concurrency, plus the top kernels by summed duration.

    python scripts/kbusy.py gpurun_out/.../kernel_trace.csv [N] [steps]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    rows = rows[-n:]
    iv = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows)
    t0, t1 = iv[0][0], max(e for _, e in iv)
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(e - s for s, e in iv)
    span = t1 - t0
    per = f" ({span / steps / 1e3:.1f} us/step)" if steps else ""
    print(f"dispatches {len(iv)}  span {span / 1e3:.1f} us{per}  busy {busy / 1e3:.1f} us "
          f"({busy / span:.1%})  idle {(span - busy) / 1e3:.1f} us  kernel-sum {tot / 1e3:.1f} us "
          f"concurrency {tot / max(busy, 1):.2f}")
    agg = defaultdict(lambda: [0, 0])
    for x in rows:
        k = x["Kernel_Name"].replace("psamd::", "").replace("void ", "").split("(")[0]
        agg[k][0] += 1
        agg[k][1] += int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
        ps = f" {d / steps / 1e3:7.1f} us/step" if steps else ""
        print(f"  {c:6d} {d / 1e3:10.1f} us{ps}  {k[:80]}")


if __name__ == "__main__":
    main()
