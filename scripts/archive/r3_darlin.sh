#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/r3_darlin_t1.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t1.log | cut -c 1-300
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --tau 8 --device-data > gpurun_out/r3_darlin_t8.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t8.log | cut -c 1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_darlin.py --rows 4000000 --passes 3 --device-data > $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof.log 2>&1 || exit $?
