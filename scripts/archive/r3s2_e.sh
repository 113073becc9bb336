#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/e_darlin -o run --output-format csv -- python3 $R/benchmarks/bench_darlin.py --rows 4000000 --passes 3 --device-data > $R/gpurun_out/e_darlin.log 2>&1 || exit $?
cd $R; python scripts/kmed.py gpurun_out/e_darlin/run_kernel_trace.csv 16
