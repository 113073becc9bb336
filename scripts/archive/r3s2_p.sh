#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { local n=$1; shift
  env "$@" > gpurun_out/q_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/q_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/q_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), round(d['train']['loss'],4))"
}
for rep in 1 2; do
run e8_pc1_$rep X=1 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 || exit 1
run e8_pc0_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 || exit 1
run g1_pc0_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --graph 1 || exit 1
run eager_$rep X=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 || exit 1
done
