cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5zb; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4))"; }
for nf in 1e9 1e10 1e9 1e10; do
  PSAMD_FB_CLOCK=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features $nf > $O/c_$nf.log 2>&1 || exit 3; j $O/c_$nf.log "nf=$nf"; grep fb_clock $O/c_$nf.log
done
PSAMD_FB_CLOCK=1 timeout -k 10 200 python bench.py --pipeline 0 --steps 100 --warmup 10 --num-features 1e10 > $O/s.log 2>&1 || exit 3; j $O/s.log "seq nf=1e10"; grep fb_clock $O/s.log
PSAMD_FB_CLOCK=1 timeout -k 10 200 python bench.py --pipeline 0 --steps 100 --warmup 10 --num-features 1e9 > $O/s9.log 2>&1 || exit 3; j $O/s9.log "seq nf=1e9"; grep fb_clock $O/s9.log
