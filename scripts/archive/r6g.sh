#!/bin/bash
# round 6: tail filter with the unit's sketch words staged in LDS (tests + tail benches +
# profile), asp merged / G2 defaults, cached app with more reader threads
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_tpf_gpu.py tests/test_gpu_ops.py tests/test_bench_pipeline_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "tail_filter or countmin or kw27 or kw28 or kw29 or 3-1-1 or 2-0-1 or rccl" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED" $O/pytest.log | sed 's/.*:://' | head -30; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), d['config'].get('consistency','')[:12], round(d['train'].get('loss'),4))")"; }
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run c4ftrl --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 1
run c4sgd --steps 100 --warmup 10 --algo sgd --consistency asp --fixing-float 2 --emulate-peers 8 --emulate-backend nccl || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_tail -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_tail.log 2>&1 || exit 6
echo "== tail"; python $R/scripts/kbusy_db.py $O/p_tail/run_results.db tp_fwd_bwd 40 100
cd $R
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 --io-threads 12 > $O/app8m_io12.log 2>&1; echo "app rc=$?"; tail -1 $O/app8m_io12.log
