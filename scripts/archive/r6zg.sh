#!/bin/bash
# round 6: final tree -- populated tables and the 300-step headline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6zg; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), 'occupied', d['train'].get('table_occupied_rank0'))")"; }
run base200 --steps 200 --warmup 10 || exit 1
run pf5e8 --steps 200 --warmup 10 --prefill 5e8 || exit 1
run pf1e9 --steps 200 --warmup 10 --prefill 1e9 || exit 1
run s300 --steps 300 --warmup 10 || exit 1
run s300b --steps 300 --warmup 10 || exit 1
