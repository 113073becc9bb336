#!/bin/bash
# round 6: final-tree GPU suite, smoke and driver-shape bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6zi; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }; tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -5 $O/bench20.log; exit 1; }; grep '^{' $O/bench20.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }; grep '^{' $O/bench_default.log
