#!/bin/bash
# tile imbalance probe: 313 tiles (B = 65536) vs 250 tiles (B = 52500) vs 188 (B = 39400)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
for B in 65536 52500 39400; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_n_prof_$B -o run -- python3 $R/bench.py --steps 40 --warmup 5 --pipeline 0 --graph 0 --minibatch $B > $R/gpurun_out/r3_n_prof_$B.log 2>&1 || exit 1
done
