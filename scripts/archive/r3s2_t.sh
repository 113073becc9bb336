#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { local n=$1; shift
  env "$@" > gpurun_out/u_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/u_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/u_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4))"
}
for rep in 1 2 3; do
for np in 3 2; do
run np${np}_20_$rep X=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --prep-streams $np || exit 1
run np${np}_300_$rep X=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --prep-streams $np || exit 1
done; done
