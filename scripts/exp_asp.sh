#!/bin/bash
# ASP / fixing-float costs at 8 emulated peers (ms/step, host issue ms/step)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 200 python bench.py --steps 100 --warmup 10 "$@" 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'host', round(d['host_issue_ms_per_step'],4))" || exit 1; }
run --emulate-peers 8
run --emulate-peers 8 --consistency asp
run --emulate-peers 8 --consistency ssp:1
run --emulate-peers 8 --consistency asp --graph 0
