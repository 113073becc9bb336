#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python benchmarks/tn256_determinism.py 2>&1 | grep shape
PSAMD_TN256=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider "tests/test_wide_deep_gpu.py::test_padded_exchange_matches_exact" > gpurun_out/r3_p_off.log 2>&1; echo "tn off rc=$?"; tail -1 gpurun_out/r3_p_off.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider "tests/test_wide_deep_gpu.py::test_padded_exchange_matches_exact" > gpurun_out/r3_p_on.log 2>&1; echo "tn on rc=$?"; tail -1 gpurun_out/r3_p_on.log
