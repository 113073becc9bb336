#!/bin/bash
# round 6: merged pipeline with the tail filter: only the filter launches ordered
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6r; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "tail or kw27 or kw28 or kw29 or rccl" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -cE "PASSED" $O/pytest.log; grep FAILED $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4))")"; }
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run e8tailb --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
