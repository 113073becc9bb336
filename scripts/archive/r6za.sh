#!/bin/bash
# round 6: every BASELINE config on the final tree (+ the tail-filtered step)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6za; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 bash scripts/baseline_configs.sh > $O/baseline.out 2>&1; echo "baseline rc=$?"; cp gpurun_out/baseline_configs.log $O/
grep -E "^## |FAILED" gpurun_out/baseline_configs.log | cut -c1-120
python - <<'PY'
import json
for l in open("gpurun_out/baseline_configs.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print("   ", round(d["ms_per_step"], 4), "ms", round(d["value"] / 1e6, 1), "M/s")
PY
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4))")"; }
run tail1 --steps 100 --warmup 10 --tail-freq 1
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1
