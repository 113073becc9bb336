cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5z2; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for nf in 1e9 1e10 4e9 5e9; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features $nf > $O/b_$nf.log 2>&1 || exit 3; j $O/b_$nf.log "nf=$nf"
done
cd /tmp
for nf in 1e9 1e10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$nf -o run -- python $R/bench.py --steps 100 --warmup 10 --num-features $nf > $O/p_$nf.log 2>&1 || exit 6
  echo "== $nf"; python $R/scripts/kbusy_db.py $O/p_$nf/run_results.db tp_fwd_bwd 40 100
done
