#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { # name args...
  local n=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/p_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/p_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/p_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), round(d['train']['loss'],4))"
}
for g in 1 0; do
  run e8_g$g --steps 200 --warmup 10 --emulate-peers 8 --graph $g || exit 1
  run b10k_g$g --steps 300 --warmup 10 --minibatch 10000 --graph $g || exit 1
  run e8b10k_g$g --steps 200 --warmup 10 --minibatch 10000 --emulate-peers 8 --graph $g || exit 1
  run asp8_g$g --steps 200 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --graph $g || exit 1
done
