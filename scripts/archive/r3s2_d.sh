#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py > gpurun_out/d_pytest_darlin.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/d_pytest_darlin.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  PSAMD_DARLIN_FUSE=$f timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/d_darlin_f$f.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/d_darlin_f$f.log').read().strip().splitlines()[-1]); print('darlin fuse=$f', d['ms_per_pass'], d.get('train', d.get('progress')))" 
done
for i in 1 2 3; do
  PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/d_b20_$i.log 2>&1 || exit $?
  grep step_events gpurun_out/d_b20_$i.log
  python -c "import json,sys; d=json.loads(open('gpurun_out/d_b20_$i.log').read().strip().splitlines()[-1]); print('b20', d['ms_per_step'], d['value']/1e6)"
done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > gpurun_out/d_b300.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/d_b300.log').read().strip().splitlines()[-1]); print('b300', d['ms_per_step'], d['value']/1e6)"
