#!/bin/bash
# round 6: where the cached file-fed app's time goes (host waits for minibatches vs step issue)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6zc; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for io in 8 16; do
  timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 --io-threads $io --report-steps 100000 > $O/app_io$io.log 2>&1 || { echo "app $io failed"; tail -5 $O/app_io$io.log; exit 1; }
  tail -1 $O/app_io$io.log | python -c "
import sys,json
d=json.loads(sys.stdin.read())
for r in d['runs']: print('io', $io, {k: (round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k in ('source','seconds','examples_per_s','host_feed_wait_s','host_step_issue_s','feeder_only_examples_per_s','trainer_only_examples_per_s','h2d_gb_per_s')})"
done
cd /tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/p_app -o run -- python $R/benchmarks/bench_app.py --rows 4000000 --files 8 --minibatch 65536 --io-threads 8 --report-steps 100000 > $R/$O/p_app.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $R/$O/p_app/run_results.db 10
python - "$R/$O/p_app/run_results.db" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
mc = [t for t in tabs if 'memory_copy' in t and not t.startswith('rocpd_memory_copy_')]
print("copy tables", mc[:4])
for t in mc[:1]:
    cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
    print(cols)
    rows = c.execute(f"select * from {t} limit 3").fetchall()
    for r in rows: print(r)
    n = c.execute(f"select count(*), sum(end-start) from {t}").fetchone()
    print("copies", n)
PY
