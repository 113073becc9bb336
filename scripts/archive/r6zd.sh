#!/bin/bash
# round 6: final-tree kernel traces (headline, tail filter, 8 emulated peers, config 4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6zd; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
prof() { n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$n -o run -- python $R/bench.py "$@" > $O/p_$n.log 2>&1 || return 6
  echo "== $n: $(grep '^{' $O/p_$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'ms (under the tracer)')")"
  python $R/scripts/kdist_db.py $O/p_$n/run_results.db 12; }
prof headline --steps 100 --warmup 10 || exit 6
prof tail --steps 100 --warmup 10 --tail-freq 1 || exit 6
prof e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 6
prof c4 --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl || exit 6
