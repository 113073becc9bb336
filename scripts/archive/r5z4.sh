cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5z4; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do
for c in "p-1n2 -1 2" "p0n2 0 2" "p-1n3 -1 3" "p0n3 0 3"; do set -- $c
  PSAMD_PREP_PRIORITY=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --prep-streams $3 > $O/$1_$i.log 2>&1 || exit 3; j $O/$1_$i.log "20 $1"
done; done
for c in "p-1n2 -1 2" "p0n2 0 2"; do set -- $c
  PSAMD_PREP_PRIORITY=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --prep-streams $3 > $O/l$1.log 2>&1 || exit 3; j $O/l$1.log "300 $1"
done
