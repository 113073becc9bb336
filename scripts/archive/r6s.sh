#!/bin/bash
# round 6: merged tail ordering check (r6r), an 8-peer kernel trace, every BASELINE config
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6s; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/archive/r6r.sh || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_e8 -o run -- python $R/bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/p_e8.log 2>&1 || exit 6
python $R/scripts/kbusy_db.py $O/p_e8/run_results.db tp_fwd_bwd 40 100
python $R/scripts/kdist_db.py $O/p_e8/run_results.db 14
cd $R
timeout -k 10 900 bash scripts/baseline_configs.sh > $O/baseline.out 2>&1; echo "baseline rc=$?"; grep -E "^## |FAILED|ms_per_step" gpurun_out/baseline_configs.log | python -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('   ', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,1), 'M/s', 'host', round(d.get('host_issue_ms_per_step') or 0,4))
    else: print(l[:150])
"
cp gpurun_out/baseline_configs.log $O/
