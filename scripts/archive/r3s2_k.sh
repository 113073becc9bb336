#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for g in auto mfma; do for ov in 1 0; do for gr in 0 1; do
  timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 40 --gemm $g --overlap-wgrad $ov --graph $gr > gpurun_out/k_wd_${g}_$ov$gr.log 2>&1 || { echo "fail $g $ov $gr"; tail -5 gpurun_out/k_wd_${g}_$ov$gr.log; continue; }
  python -c "import json; d=json.loads(open('gpurun_out/k_wd_${g}_$ov$gr.log').read().strip().splitlines()[-1]); print('$g overlap=$ov graph=$gr', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), round(d['train']['loss'],4))"
done; done; done
