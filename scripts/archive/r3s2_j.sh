#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_wide_deep_gpu.py tests/test_fm_gpu.py tests/test_embedding_checkpoint.py > gpurun_out/j_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/j_pytest.log
[ $rc -eq 0 ] || exit $rc
for g in auto mfma; do
  timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm $g > gpurun_out/j_wd_$g.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/j_wd_$g.log').read().strip().splitlines()[-1]); print('$g', d['ms_per_step'], d['host_issue_ms_per_step'], d['train']['loss'], d['train']['auc'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/j_wd_prof -o run --output-format csv -- python3 $R/benchmarks/bench_wide_deep.py --steps 20 --gemm auto > $R/gpurun_out/j_wd_prof.log 2>&1 || exit $?
cd $R; python scripts/kmed.py gpurun_out/j_wd_prof/run_kernel_trace.csv 30
