#!/bin/bash
# preparation streams at 8 emulated peers through a real 1-rank RCCL communicator
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 200 python bench.py --steps 200 --warmup 20 --emulate-peers 8 --emulate-backend nccl "$@" 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'host', round(d['host_issue_ms_per_step'],4))" || exit 1; }
run --prep-streams 2
run --prep-streams 3
run --prep-streams 2
run --prep-streams 3
