#!/bin/bash
# round 6: blocked CountMin (a key's cells in one 64-cell block) on the tail-filtered step;
# the cost of ordering the bucket kernels (PSAMD_TAIL_ORDER_MEASURE=0: unordered, timing only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6o; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), round(d['train'].get('loss'),4))")"; }
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
PSAMD_TAIL_ORDER_MEASURE=0 run tail1_unordered --steps 100 --warmup 10 --tail-freq 1 || exit 1
run tail1b --steps 100 --warmup 10 --tail-freq 1 || exit 1
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_tail -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_tail.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_tail/run_results.db 6
cd $R
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 --io-threads 8 --report-steps 100000 > $O/app8m_norep.log 2>&1; echo "app rc=$?"; tail -1 $O/app8m_norep.log
