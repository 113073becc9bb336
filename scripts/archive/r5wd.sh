cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5wd; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2; do
timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 > $O/b$i.log 2>&1 || exit 3
grep -h '^{' $O/b$i.log | python -c "import sys,json; [print('wd', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4)) for d in map(json.loads, sys.stdin)]"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $R/benchmarks/bench_wide_deep.py --steps 30 > $O/prof.log 2>&1 || exit 4
python - <<PY
import sqlite3
from collections import defaultdict
rows = sqlite3.connect('$O/prof/run_results.db').execute("select name, start, end from kernels order by start").fetchall()
# last 20 steps: find a marker = the most frequent kernel name with count ~ steps
from collections import Counter
c = Counter(r[0] for r in rows)
print(len(rows), "kernels")
t_end = rows[-1][2]
span_lo = rows[int(len(rows)*0.4)][1]
d = defaultdict(list)
for n, s, e in rows:
    if s >= span_lo: d[n[:90]].append(e - s)
tot = sum(sum(v) for v in d.values())
print(f"window {(t_end-span_lo)/1e3:.1f} us kernel sum {tot/1e3:.1f} us")
for n, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:30]:
    v.sort(); print(f"{len(v):6d} {sum(v)/1e3:9.1f} us med {v[len(v)//2]/1e3:7.2f}  {n}")
PY
