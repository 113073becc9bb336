#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bench_pipeline_gpu.py > gpurun_out/r_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r_pytest.log
[ $rc -eq 0 ] || exit $rc
for st in 300 20; do
  w=10; [ $st -eq 20 ] && w=5
  timeout -k 10 120 python bench.py --steps $st --warmup $w > gpurun_out/r_b$st.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r_b$st.log').read().strip().splitlines()[-1]); print('steps=$st', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['table_occupied_rank0'], round(d['train']['loss'],4))"
done
bash scripts/baseline_configs.sh > /dev/null 2>&1; cat gpurun_out/baseline_configs.log | cut -c1-250
