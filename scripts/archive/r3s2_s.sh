#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { local n=$1; shift
  env "$@" > gpurun_out/t_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/t_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/t_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['table_occupied_rank0'])"
}
for rep in 1 2; do
for np in 3 2 4; do
run np${np}_$rep X=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --prep-streams $np || exit 1
done
run prio0_$rep PSAMD_PREP_PRIORITY=0 timeout -k 10 200 python bench.py --steps 300 --warmup 10 || exit 1
done
