#!/bin/bash
# round 6: the eager step on bench_app's skewed ids (N * U^4) vs bench.py's generator
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6j; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for d in criteo pow4 pow2; do
  PROBE_DIST=$d timeout -k 10 200 python benchmarks/probe_app_step.py > $O/probe_$d.log 2>&1 || { echo "probe $d failed"; tail -5 $O/probe_$d.log; exit 1; }
  grep '^{' $O/probe_$d.log
done
cd /tmp
PROBE_DIST=pow4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_pow4 -o run -- python $R/benchmarks/probe_app_step.py > $O/p_pow4.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_pow4/run_results.db 10
