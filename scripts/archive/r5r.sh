cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5r; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do
for a in "asp1 --consistency asp --fixing-float 1" "ssp4 " "asp0 --consistency asp"; do set -- $a; n=$1; shift
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl "$@" > $O/$n_$i.log 2>&1 || exit 3; j $O/$n_$i.log "e8 $n"
done; done
for l in 7 8 10; do
  PSAMD_APPLY_LGP=$l timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/asp_l$l.log 2>&1 || exit 3; j $O/asp_l$l.log "e8 asp1 lgP=$l"
done
