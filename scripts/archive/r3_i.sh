#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py tests/test_tploc_gpu.py > gpurun_out/r3_pytest_i.log 2>&1 || { tail -30 gpurun_out/r3_pytest_i.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_i.log
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/r3_darlin_t1.log 2>&1 && tail -1 gpurun_out/r3_darlin_t1.log | cut -c 1-250
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --tau 8 --device-data > gpurun_out/r3_darlin_t8.log 2>&1 && tail -1 gpurun_out/r3_darlin_t8.log | cut -c 1-250
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_darlin_prof4 -o run -- python3 $R/benchmarks/bench_darlin.py --rows 4000000 --passes 3 --device-data > $R/gpurun_out/r3_darlin_prof4.log 2>&1
cd $R && bash scripts/r3_hostprof.sh
