#!/bin/bash
# W&D: HIP-graph step vs eager, host issue time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_wide_deep_gpu.py > gpurun_out/b_pytest_wd.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/b_pytest_wd.log
for g in auto mfma; do for gr in 0 1; do
  timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm $g --graph $gr > gpurun_out/b_wd_${g}_g$gr.log 2>&1 || { echo "fail $g $gr"; tail -20 gpurun_out/b_wd_${g}_g$gr.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b_wd_${g}_g$gr.log').read().strip().splitlines()[-1]); print('$g graph=$gr', d['ms_per_step'], d['host_issue_ms_per_step'], d['train']['loss'], d['train']['auc'])"
done; done
