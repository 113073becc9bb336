#!/bin/bash
# round 6: where the tail filter's bucket-kernel time goes (PSAMD_CM_DEBUG 2: no filter work
# past the occurrence counts, 1: no sketch traffic, 0: full) + cached app breakdown
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
for m in 2 1 0; do
  PSAMD_CM_DEBUG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_dbg$m -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_dbg$m.log 2>&1 || exit 6
  echo "== dbg $m: $(grep '^{' $O/p_dbg$m.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4))")"
  python $R/scripts/kdist_db.py $O/p_dbg$m/run_results.db 5
done
cd $R
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/tail1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/base100.log 2>&1 || exit 1
for n in tail1 base100; do echo "$n $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4))")"; done
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 --io-threads 8 > $O/app8m.log 2>&1; echo "app rc=$?"; grep breakdown $O/app8m.log; tail -1 $O/app8m.log
