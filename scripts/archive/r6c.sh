#!/bin/bash
# round 6: 1e10 slowdown (tile / fwd-bwd co-scheduling), tile gate A/B, filter profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for g in 0 1; do
  for nf in 1e9 1e10; do
    PSAMD_TILE_GATE=$g timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features $nf > $O/b_${nf}_g$g.log 2>&1 || exit 3; j $O/b_${nf}_g$g.log "gate=$g nf=$nf 300"
    PSAMD_TILE_GATE=$g timeout -k 10 200 python bench.py --steps 20 --warmup 5 --num-features $nf > $O/b20_${nf}_g$g.log 2>&1 || exit 3; j $O/b20_${nf}_g$g.log "gate=$g nf=$nf 20"
  done
done
cd /tmp
for g in 0 1; do
for nf in 1e9 1e10; do
  PSAMD_TILE_GATE=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_${nf}_g$g -o run -- python $R/bench.py --steps 100 --warmup 10 --num-features $nf > $O/p_${nf}_g$g.log 2>&1 || exit 6
  echo "== gate $g $nf"; python $R/scripts/kbusy_db.py $O/p_${nf}_g$g/run_results.db tp_fwd_bwd 40 100
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_tail -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_tail.log 2>&1 || exit 6
echo "== tail"; python $R/scripts/kbusy_db.py $O/p_tail/run_results.db tp_fwd_bwd 40 100
