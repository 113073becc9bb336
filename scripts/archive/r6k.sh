#!/bin/bash
# round 6: flat layout on skewed / near-distinct ids: pair workgroups vs one fine bucket per
# workgroup (PSAMD_TPF_PAIR=0), headline and tail runs under both
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6k; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for p in 1 0; do
  PSAMD_TPF_PAIR=$p timeout -k 10 200 python benchmarks/probe_skew_loc.py > $O/skew_p$p.log 2>&1 || { echo "skew $p failed"; tail -5 $O/skew_p$p.log; exit 1; }
  echo "== pair $p"; grep '^{' $O/skew_p$p.log
  for d in criteo pow4; do
    PSAMD_TPF_PAIR=$p PROBE_DIST=$d timeout -k 10 200 python benchmarks/probe_app_step.py > $O/app_${d}_p$p.log 2>&1 || exit 1
    grep '^{' $O/app_${d}_p$p.log
  done
done
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), round(d['train'].get('loss'),4))")"; }
run base_p1 --steps 100 --warmup 10 || exit 1
PSAMD_TPF_PAIR=0 run base_p0 --steps 100 --warmup 10 || exit 1
run base_p1b --steps 100 --warmup 10 || exit 1
PSAMD_TPF_PAIR=0 run base_p0b --steps 100 --warmup 10 || exit 1
run tail_p1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
PSAMD_TPF_PAIR=0 run tail_p0 --steps 100 --warmup 10 --tail-freq 1 || exit 1
