#!/bin/bash
# One build -> measure iteration for the tp step kernels: GPU numerics tests of the tp /
# fused / pipeline paths, standalone tp microbenchmark, 1-GPU bench, 2 PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/iter; export TMPDIR=/tmp PYTHONUNBUFFERED=1
R="$GRAFT_REPO_ROOT"; O=gpurun_out/iter
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tp_fused_gpu.py tests/test_tploc_gpu.py tests/test_bench_pipeline_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PSAMD_LOC_MODES=tp timeout -k 10 120 python benchmarks/bench_localize.py > $O/loc.log 2>&1 || exit 1
grep -v amdgpu $O/loc.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value']/1e6)"
timeout -k 10 120 python benchmarks/prof_tp_phases.py > $O/phases.log 2>&1 && grep -v amdgpu $O/phases.log | tail -9
[ "${PMC:-1}" = "1" ] || exit 0
cd /tmp; i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" ; do
  i=$((i+1))
  PSAMD_LOC_MODES=tp timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d "$R/$O/p$i" -o run --output-format csv -- python3 "$R/benchmarks/bench_localize.py" > "$R/$O/p$i.log" 2>&1 || exit 1
done
