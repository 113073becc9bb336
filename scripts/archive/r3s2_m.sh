#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do for g in 1 0; do for st in 300 20; do
  w=10; [ $st -eq 20 ] && w=5
  timeout -k 10 120 python bench.py --steps $st --warmup $w --graph $g > gpurun_out/o_${g}_${st}_$rep.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/o_${g}_${st}_$rep.log').read().strip().splitlines()[-1]); print('graph=$g steps=$st', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['table_occupied_rank0'])"
done; done; done
