#!/bin/bash
# driver-exact bench x3 + long run; W&D kernel breakdown (auto / mfma)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/a_b20_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/a_b20_$i.log').read().strip().splitlines()[-1]); print('b20', d['ms_per_step'], d['value']/1e6)"
done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > gpurun_out/a_b300.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/a_b300.log').read().strip().splitlines()[-1]); print('b300', d['ms_per_step'], d['value']/1e6)"
for g in auto mfma; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/a_wd_$g -o run --output-format csv -- python3 $R/benchmarks/bench_wide_deep.py --steps 20 --gemm $g > $R/gpurun_out/a_wd_$g.log 2>&1 || exit $?
  cd $R
done
timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm auto > gpurun_out/a_wd_auto_t.log 2>&1 && tail -1 gpurun_out/a_wd_auto_t.log | cut -c 1-200
timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --gemm mfma > gpurun_out/a_wd_mfma_t.log 2>&1 && tail -1 gpurun_out/a_wd_mfma_t.log | cut -c 1-200
