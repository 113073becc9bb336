#!/bin/bash
# round 6: near-distinct ids -- early-abort pair build + batched register-light units;
# headline / tail unchanged?; the cached file-fed app on bench_app's skewed files
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6m; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python benchmarks/probe_skew_loc.py > $O/skew.log 2>&1 || { tail -5 $O/skew.log; exit 1; }
grep '^{' $O/skew.log
for d in criteo pow4; do
  PROBE_DIST=$d timeout -k 10 200 python benchmarks/probe_app_step.py > $O/app_$d.log 2>&1 || exit 1
  grep '^{' $O/app_$d.log
done
timeout -k 10 500 python -u -m pytest tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -x -q -k "not rccl or tail" --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_tpf.log 2>&1; rc=$?; echo "pytest tpf rc=$rc"; tail -2 $O/pytest_tpf.log; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), round(d['train'].get('loss'),4))")"; }
run base100 --steps 100 --warmup 10 || exit 1
run b20 --steps 20 --warmup 5 || exit 1
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100b --steps 100 --warmup 10 || exit 1
cd /tmp
PROBE_DISTS=pow4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_pow4 -o run -- python $R/benchmarks/probe_skew_loc.py > $O/p_pow4.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_pow4/run_results.db 4
cd $R
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 --io-threads 8 > $O/app8m.log 2>&1; echo "app rc=$?"; grep breakdown $O/app8m.log; tail -1 $O/app8m.log
