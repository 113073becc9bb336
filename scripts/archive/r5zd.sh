cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5zd; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do
for t in wt_a wt_b .; do
  (cd $R/$t && timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/b10k_${t#./}_$i.log 2>&1) || exit 3; j $O/b10k_${t#./}_$i.log "B10k $t"
done; done
for t in wt_a .; do
  (cd $R/$t && timeout -k 10 200 python bench.py --steps 200 --warmup 10 --minibatch 10000 --emulate-peers 8 > $O/e8_${t#./}.log 2>&1) || exit 3; j $O/e8_${t#./}.log "e8 B10k $t"
done
