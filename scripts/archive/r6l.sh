#!/bin/bash
# round 6: overflowing bucket pairs on skewed / near-distinct ids: bounded probe chains, and
# the per-fine-bucket LDS build (PSAMD_TPF_FINE=1, default) vs the register-light form (0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6l; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for f in 1 0; do
  echo "== fine $f"
  PSAMD_TPF_FINE=$f timeout -k 10 200 python benchmarks/probe_skew_loc.py > $O/skew_f$f.log 2>&1 || { tail -5 $O/skew_f$f.log; exit 1; }
  grep '^{' $O/skew_f$f.log
  PSAMD_TPF_FINE=$f PROBE_DIST=pow4 timeout -k 10 200 python benchmarks/probe_app_step.py > $O/app_pow4_f$f.log 2>&1 || exit 1
  grep '^{' $O/app_pow4_f$f.log
done
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), round(d['train'].get('loss'),4))")"; }
run base_f1 --steps 100 --warmup 10 || exit 1
PSAMD_TPF_FINE=0 run base_f0 --steps 100 --warmup 10 || exit 1
run base_f1b --steps 100 --warmup 10 || exit 1
PSAMD_TPF_FINE=0 run base_f0b --steps 100 --warmup 10 || exit 1
cd /tmp
PROBE_DISTS=pow4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_pow4 -o run -- python $R/benchmarks/probe_skew_loc.py > $O/p_pow4.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_pow4/run_results.db 6
cd $R
timeout -k 10 400 python -u -m pytest tests/test_tpf_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_tpf.log 2>&1; echo "pytest tpf rc=$?"; tail -2 $O/pytest_tpf.log
