#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/bench_gemm256.py > gpurun_out/i_gemm.log 2>&1; rc=$?
python - <<'PY'
import json
for l in open('gpurun_out/i_gemm.log'):
    if l.startswith('{') and 'gemm256w4_tflops' in l:
        d=json.loads(l); print(d['shape'], 'err', [round(e,4) for e in d['max_rel_err_vs_fp32']], {k: round(v) for k, v in d.items() if k.endswith('tflops')})
PY
exit $rc
