#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_tp_fused_gpu.py tests/test_tploc_gpu.py tests/test_darlin_gpu.py tests/test_trainer_gpu.py tests/test_bench_pipeline_gpu.py > gpurun_out/r3_pytest_h.log 2>&1 || { tail -30 gpurun_out/r3_pytest_h.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_h.log
for s in 1 2; do timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/r3_h_b1_$s.log 2>&1 || exit $?; tail -1 gpurun_out/r3_h_b1_$s.log | cut -c 150-260; done
PSAMD_FUSED_UPDATE=0 timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/r3_h_b1_unfused.log 2>&1 || exit $?; tail -1 gpurun_out/r3_h_b1_unfused.log | cut -c 150-260
timeout -k 10 240 python bench.py --steps 300 --warmup 20 --minibatch 10000 > gpurun_out/r3_h_b10k.log 2>&1 || exit $?; tail -1 gpurun_out/r3_h_b10k.log | cut -c 150-260
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/r3_darlin_t1.log 2>&1 && tail -1 gpurun_out/r3_darlin_t1.log | cut -c 1-250
timeout -k 10 120 python benchmarks/prof_tp_phases.py > gpurun_out/r3_tp_phases2.log 2>&1 && head -10 gpurun_out/r3_tp_phases2.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_seq3 -o run -- python3 $R/bench.py --steps 50 --warmup 5 --pipeline 0 --graph 0 > $R/gpurun_out/r3_seq3.log 2>&1
