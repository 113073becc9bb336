#!/bin/bash
# wide & deep (BASELINE config 5) and FM: step times per GEMM backend + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
for g in auto mfma hipblaslt; do
  timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm $g > gpurun_out/r3_wd_$g.log 2>&1 || exit $?
  tail -1 gpurun_out/r3_wd_$g.log | cut -c 1-260
done
timeout -k 10 300 python benchmarks/bench_fm.py --steps 30 > gpurun_out/r3_fm.log 2>&1 && tail -1 gpurun_out/r3_fm.log | cut -c 1-400
timeout -k 10 300 python benchmarks/bench_gemm256.py > gpurun_out/r3_gemm256.log 2>&1; tail -8 gpurun_out/r3_gemm256.log | cut -c 1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_wd_prof -o run -- python3 $R/benchmarks/bench_wide_deep.py --steps 20 --gemm mfma > $R/gpurun_out/r3_wd_prof.log 2>&1
