#!/bin/bash
# round 6: final-tree GPU suite + smoke + driver-shape bench x3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${RUN_TAG:-r6x}; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit 1
  echo "b20_$i: $(grep '^{' $O/b20_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4))")"
done
timeout -k 10 200 python bench.py > $O/bdef.log 2>&1 || exit 1
echo "defaults: $(grep '^{' $O/bdef.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), d['steps'], d['warmup'])")"
