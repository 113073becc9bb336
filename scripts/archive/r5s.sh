cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5s; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do
  (cd $R/old_r4 && timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/old_asp_$i.log 2>&1) || exit 3; j $O/old_asp_$i.log "r4tree e8 asp1"
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/new_asp_$i.log 2>&1 || exit 3; j $O/new_asp_$i.log "r5tree e8 asp1"
done
(cd $R/old_r4 && timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl > $O/old_ssp.log 2>&1) || exit 3; j $O/old_ssp.log "r4tree e8 ssp4"
(cd $R/old_r4 && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/old_b1.log 2>&1) || exit 3; j $O/old_b1.log "r4tree 1gpu-20"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/new_b1.log 2>&1 || exit 3; j $O/new_b1.log "r5tree 1gpu-20"
