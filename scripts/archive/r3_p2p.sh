#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_p2p_gpu.py tests/test_sharded_kv.py > gpurun_out/r3_pytest_p2p.log 2>&1; rc=$?
tail -15 gpurun_out/r3_pytest_p2p.log; exit $rc
