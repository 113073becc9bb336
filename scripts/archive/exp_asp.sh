#!/bin/bash
# ASP at 8 emulated peers: owner-apply partition count (fewer, longer apply workgroups
# steal less of the CU time the worker half needs); ms/step, host issue ms/step
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --consistency asp "$@" 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'host', round(d['host_issue_ms_per_step'],4))" || exit 1; }
run
PSAMD_APPLY_LGP=8 run
PSAMD_APPLY_LGP=7 run
PSAMD_APPLY_LGP=6 run
run
PSAMD_APPLY_LGP=7 run --fixing-float 1
run --fixing-float 1
