cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5ze; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do for t in wt_a wt_b cur; do
  d=$R/$t; [ $t = cur ] && d=$R
  (cd $d && timeout -k 10 200 python bench.py --steps 200 --warmup 10 --minibatch 10000 --emulate-peers 8 > $O/e8_${t}_$i.log 2>&1) || exit 3; j $O/e8_${t}_$i.log "e8 B10k $t"
done; done
cd /tmp
for t in wt_a cur; do
  d=$R/$t; [ $t = cur ] && d=$R
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_$t -o run -- python $d/bench.py --pipeline 0 --steps 60 --warmup 10 --minibatch 10000 --emulate-peers 8 > $O/seq_$t.log 2>&1 || exit 6
  echo "== $t"; python $R/scripts/kbusy_db.py $O/seq_$t/run_results.db tp_fwd_bwd 20 60
done
