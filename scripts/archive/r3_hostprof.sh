#!/bin/bash
# host-side profile of the 8-emulated-peer step (is the exchange issue host-bound?)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -m cProfile -o gpurun_out/r3_e8_host.prof bench.py --steps 2000 --warmup 20 --emulate-peers 8 ${EXTRA:-} > gpurun_out/r3_e8_hostprof.log 2>&1 || exit $?
tail -1 gpurun_out/r3_e8_hostprof.log | cut -c 150-330
python - <<'PY' > gpurun_out/r3_e8_host_top.txt
import pstats
p = pstats.Stats("gpurun_out/r3_e8_host.prof")
p.sort_stats("tottime").print_stats(40)
p.sort_stats("cumulative").print_stats(40)
PY
