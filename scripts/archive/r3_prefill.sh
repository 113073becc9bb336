#!/bin/bash
# populated-table regime at design load (>= 45 % of the slots), 1 GPU and 8 emulated peers
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --prefill 3e9 > gpurun_out/r3_prefill_1gpu.log 2>&1 || exit $?
grep prefill gpurun_out/r3_prefill_1gpu.log; tail -1 gpurun_out/r3_prefill_1gpu.log | cut -c 1-300
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > gpurun_out/r3_empty_1gpu.log 2>&1 || exit $?
tail -1 gpurun_out/r3_empty_1gpu.log | cut -c 1-300
timeout -k 10 400 python bench.py --steps 100 --warmup 20 --emulate-peers 8 --prefill 1.25e8 > gpurun_out/r3_prefill_e8.log 2>&1 || exit $?
grep prefill gpurun_out/r3_prefill_e8.log; tail -1 gpurun_out/r3_prefill_e8.log | cut -c 1-300
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_prefill_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --pipeline 0 --graph 0 --prefill 3e9 > $R/gpurun_out/r3_prefill_prof.log 2>&1 || exit $?
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_prefill_e8_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --emulate-peers 8 --prefill 1.25e8 > $R/gpurun_out/r3_prefill_e8_prof.log 2>&1 || exit $?
