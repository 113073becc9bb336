#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2 3; do
  PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c_b20_$i.log 2>&1 || exit $?
  grep step_events gpurun_out/c_b20_$i.log
  python -c "import json,sys; d=json.loads(open('gpurun_out/c_b20_$i.log').read().strip().splitlines()[-1]); print('b20', d['ms_per_step'], d['value']/1e6)"
done
