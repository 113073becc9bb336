#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py > gpurun_out/r3_pytest_darlin.log 2>&1 || { tail -30 gpurun_out/r3_pytest_darlin.log; exit 1; }
tail -1 gpurun_out/r3_pytest_darlin.log
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/r3_darlin_t1.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t1.log | cut -c 1-400
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --tau 8 --device-data > gpurun_out/r3_darlin_t8.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t8.log | cut -c 1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof2 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_darlin.py --rows 4000000 --passes 3 --device-data > $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof2.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_p2p_gpu.py > gpurun_out/r3_pytest_p2p.log 2>&1; rc=$?
tail -8 gpurun_out/r3_pytest_p2p.log; exit $rc
