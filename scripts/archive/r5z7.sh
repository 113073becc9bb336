cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z7; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for i in 1 2; do for k in 0 2; do
  PSAMD_PRE_TIMING_ITERS=$k PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/e${k}_$i.log 2>&1 || exit 3
  echo "pre=$k"; grep step_events_ms $O/e${k}_$i.log | cut -c1-200
done; done
for i in 1 2 3; do for k in 0 2; do
  PSAMD_PRE_TIMING_ITERS=$k timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b${k}_$i.log 2>&1 || exit 3; j $O/b${k}_$i.log "20 pre=$k"
done; done
