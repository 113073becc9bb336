#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in "256 256" "128 256" "192 256" "384 256" "256 192" "256 320" "256 256"; do
  set -- $cfg
  PSAMD_BCD_W=$1 PSAMD_BCD_WHOT=$2 timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/f_darlin_$1_$2.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/f_darlin_$1_$2.log').read().strip().splitlines()[-1]); print('W=$1 Whot=$2', d['ms_per_pass'])"
done
