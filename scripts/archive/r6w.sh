#!/bin/bash
# round 6: owner apply chains ordered in LDS runs (hot keys in every source row)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6w; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu.py tests/test_bench_pipeline_gpu.py tests/test_owner_apply_gpu.py tests/test_owner_split_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep FAILED $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4))")"; }
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run c4ftrl --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 1
run e8b --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run c4sgd --steps 100 --warmup 10 --algo sgd --consistency asp --fixing-float 2 --emulate-peers 8 --emulate-backend nccl || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_e8 -o run -- python $R/bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/p_e8.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_e8/run_results.db 8
