#!/bin/bash
# round 6: overflow poll through a numpy view of the pinned word (per-step host path)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6zh; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "overflow or rccl or merged or padded" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))")"; }
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run c4 --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 1
run c4sgd --steps 100 --warmup 10 --algo sgd --consistency asp --fixing-float 2 --emulate-peers 8 --emulate-backend nccl || exit 1
