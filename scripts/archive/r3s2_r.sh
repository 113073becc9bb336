#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bench_pipeline_gpu.py > gpurun_out/s_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/s_pytest.log
[ $rc -eq 0 ] || exit $rc
run() { local n=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/s_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/s_$n.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/s_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), round(d['train']['loss'],4), d['train']['trains'])"
}
for rep in 1 2; do
run asp8_$rep --steps 200 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 || exit 1
run aspftrl8_$rep --steps 200 --warmup 10 --emulate-peers 8 --consistency asp --fixing-float 1 || exit 1
run e8_$rep --steps 200 --warmup 10 --emulate-peers 8 || exit 1
done
