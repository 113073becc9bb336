cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5sweep; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do
for cfg in "PSAMD_XD=2" "PSAMD_XD=1" "PSAMD_PREP_PRIORITY=0" "PSAMD_XD=2"; do
env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1 || exit 3; j $O/e8.log "e8 $cfg"
done; done
