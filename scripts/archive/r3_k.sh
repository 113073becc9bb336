#!/bin/bash
# collectives captured into the step graphs: pipeline equivalence, clean exit, e8 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_bench_pipeline_gpu.py > gpurun_out/r3_pytest_k.log 2>&1 || { tail -40 gpurun_out/r3_pytest_k.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_k.log
for c in 0 1 0 1; do
  PSAMD_CAPTURE_COMM=$c timeout -k 10 120 python bench.py --steps 400 --warmup 20 --emulate-peers 8 > gpurun_out/r3_k_e8_c$c.log 2>&1 || exit $?
  echo "capture=$c $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r3_k_e8_c$c.log') if l.startswith('{')][-1]); print(round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['loss'], d['config']['consistency'][:20])")"
done
for cons in asp bsp; do
  timeout -k 10 120 python bench.py --steps 400 --warmup 20 --emulate-peers 8 --consistency $cons > gpurun_out/r3_k_e8_$cons.log 2>&1 || exit $?
  echo "$cons $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r3_k_e8_$cons.log') if l.startswith('{')][-1]); print(round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['loss'])")"
done
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --emulate-peers 8 --minibatch 10000 > gpurun_out/r3_k_e8_b10k.log 2>&1 || exit $?
echo "b10k $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r3_k_e8_b10k.log') if l.startswith('{')][-1]); print(round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d['train']['loss'])")"
