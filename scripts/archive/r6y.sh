#!/bin/bash
# round 6: tile gate in the merged (8-peer) pipeline, A/B interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6y; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "rccl" > $O/pytest_g0.log 2>&1 || { echo "pytest g0 failed"; tail -3 $O/pytest_g0.log; exit 1; }
PSAMD_MX_TILE_GATE=1 timeout -k 10 600 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "rccl" > $O/pytest_g1.log 2>&1 || { echo "pytest g1 failed"; tail -3 $O/pytest_g1.log; exit 1; }
echo "pytest ok"
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4))")"; }
for i in 1 2; do
  run e8_g0_$i --steps 100 --warmup 10 --emulate-peers 8 || exit 1
  PSAMD_MX_TILE_GATE=1 run e8_g1_$i --steps 100 --warmup 10 --emulate-peers 8 || exit 1
done
run c4_g0 --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 1
PSAMD_MX_TILE_GATE=1 run c4_g1 --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 1
run e8t_g0 --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
PSAMD_MX_TILE_GATE=1 run e8t_g1 --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
run e2_g0 --steps 100 --warmup 10 --emulate-peers 2 || exit 1
PSAMD_MX_TILE_GATE=1 run e2_g1 --steps 100 --warmup 10 --emulate-peers 2 || exit 1
