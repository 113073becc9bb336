#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py -k "grad_rows" > gpurun_out/r3_pytest_darlin_rows.log 2>&1
tail -30 gpurun_out/r3_pytest_darlin_rows.log | cut -c 1-200
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_p2p_gpu.py > gpurun_out/r3_pytest_p2p.log 2>&1; rc=$?
grep -v "^E   *[-0-9]\|^E  *0\." gpurun_out/r3_pytest_p2p.log | tail -40 | cut -c 1-250; exit $rc
