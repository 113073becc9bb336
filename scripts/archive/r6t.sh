#!/bin/bash
# round 6: per-step GPU times of the driver-shape run (fill / drain of the pipeline)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6t; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2 3; do
  PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/ev$i.log 2>&1 || exit 1
  grep step_events_ms $O/ev$i.log | cut -c1-400
  echo "ev$i: $(grep '^{' $O/ev$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4))")"
done
for pre in 0 6; do
  PSAMD_PRE_TIMING_ITERS=$pre PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/pre$pre.log 2>&1 || exit 1
  grep step_events_ms $O/pre$pre.log | cut -c1-400
  echo "pre$pre: $(grep '^{' $O/pre$pre.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4))")"
done
