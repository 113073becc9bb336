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
