#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_train_quality_gpu.py > gpurun_out/r3_pytest_l.log 2>&1 || { tail -40 gpurun_out/r3_pytest_l.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_l.log
bash scripts/r3_prefill.sh
