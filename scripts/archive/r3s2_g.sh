#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py > gpurun_out/g_pytest_darlin.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/g_pytest_darlin.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
  PSAMD_DARLIN_FUSE=$f timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/g_darlin_f$f.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/g_darlin_f$f.log').read().strip().splitlines()[-1]); print('darlin fuse=$f', d['ms_per_pass'], d.get('train', d.get('progress')))"
done
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau 8 > gpurun_out/g_darlin_tau8.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/g_darlin_tau8.log').read().strip().splitlines()[-1]); print('darlin tau8', d['ms_per_pass'])"
