#!/bin/bash
# pair-bucket tp localisation: numerics, phases, step time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_tploc_gpu.py tests/test_tp_fused_gpu.py tests/test_trainer_gpu.py tests/test_train_quality_gpu.py tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py > gpurun_out/r3_pytest_m.log 2>&1 || { tail -40 gpurun_out/r3_pytest_m.log | cut -c 1-300; exit 1; }
tail -1 gpurun_out/r3_pytest_m.log
timeout -k 10 120 python benchmarks/prof_tp_phases.py > gpurun_out/r3_m_phases.log 2>&1 && head -12 gpurun_out/r3_m_phases.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r3_m_bench$i.log 2>&1 || exit $?; python -c "import json; d=json.loads([l for l in open('gpurun_out/r3_m_bench$i.log') if l.startswith('{')][-1]); print('bench', round(d['ms_per_step'],4), '%.4g'%d['value'], d['train']['loss'])"; done
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --minibatch 10000 > gpurun_out/r3_m_b10k.log 2>&1 && python -c "import json; d=json.loads([l for l in open('gpurun_out/r3_m_b10k.log') if l.startswith('{')][-1]); print('b10k', round(d['ms_per_step'],4), '%.4g'%d['value'])"
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --emulate-peers 8 > gpurun_out/r3_m_e8.log 2>&1 && python -c "import json; d=json.loads([l for l in open('gpurun_out/r3_m_e8.log') if l.startswith('{')][-1]); print('e8', round(d['ms_per_step'],4), '%.4g'%d['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_m_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --pipeline 0 --graph 0 > $R/gpurun_out/r3_m_prof.log 2>&1
