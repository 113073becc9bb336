#!/bin/bash
# round 6: where config 4 (asp FTRL, fixing-float 1 B, 8 emulated peers) spends its kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6u; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_c4 -o run -- python $R/bench.py --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl > $O/p_c4.log 2>&1 || exit 6
grep '^{' $O/p_c4.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('c4', round(d['ms_per_step'],4))"
python $R/scripts/kdist_db.py $O/p_c4/run_results.db 16
