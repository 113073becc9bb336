#!/bin/bash
# TN weight-gradient GEMM: numerics, kernel bench, W&D step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py tests/test_wide_deep_gpu.py > gpurun_out/r3_pytest_o.log 2>&1 || { tail -40 gpurun_out/r3_pytest_o.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_o.log
timeout -k 10 300 python benchmarks/bench_gemm256.py > gpurun_out/r3_o_gemm.log 2>&1 || { tail -20 gpurun_out/r3_o_gemm.log; exit 1; }
grep dW gpurun_out/r3_o_gemm.log | cut -c 1-400
for g in auto mfma; do
  timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm $g > gpurun_out/r3_o_wd_$g.log 2>&1 || exit $?
  tail -1 gpurun_out/r3_o_wd_$g.log | cut -c 1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_o_wd_prof -o run -- python3 $R/benchmarks/bench_wide_deep.py --steps 20 --gemm mfma > $R/gpurun_out/r3_o_wd_prof.log 2>&1
