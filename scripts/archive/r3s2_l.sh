#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bench_pipeline_gpu.py tests/test_trainer_gpu.py tests/test_gpu_ops.py > gpurun_out/l_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/l_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/l_b20_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/l_b20_$i.log').read().strip().splitlines()[-1]); print('b20', d['ms_per_step'], d['value']/1e6)"
done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > gpurun_out/l_b300.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/l_b300.log').read().strip().splitlines()[-1]); print('b300', d['ms_per_step'], d['value']/1e6, d['train'])"
