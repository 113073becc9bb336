#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { local n=$1; shift
  env "$@" > gpurun_out/w_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/w_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/w_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['table_occupied_rank0'])"
}
for rep in 1 2 3; do
for g in 0 2; do
run g${g}_300_$rep X=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --graph $g || exit 1
run g${g}_20_$rep X=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --graph $g || exit 1
done
run g2np3_300_$rep X=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --graph 2 --prep-streams 3 || exit 1
done
