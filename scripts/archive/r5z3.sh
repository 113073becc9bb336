cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5z3; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features 1e9 > $O/a.log 2>&1 || exit 3; j $O/a.log "1e9"
PSAMD_TP_QUOT=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features 1e9 > $O/b.log 2>&1 || exit 3; j $O/b.log "1e9 quot-tile"
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features 1e10 --prep-streams 3 > $O/c.log 2>&1 || exit 3; j $O/c.log "1e10 prep3"
PSAMD_NATIVE_ITER=0 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features 1e10 > $O/d.log 2>&1 || exit 3; j $O/d.log "1e10 eager"
