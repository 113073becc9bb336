#!/bin/bash
# Targeted GPU check: selected test files, then 1-GPU and emulated-peer benches.
# usage: TESTS="tests/a.py tests/b.py" BENCHES="1|e8|e8n" scripts/gpu_quick.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_quick.log
  [ $rc -eq 0 ] || exit $rc
fi
for b in ${BENCHES:-}; do
  case $b in
    1) extra="" ;;
    e2) extra="--emulate-peers 2" ;;
    e8) extra="--emulate-peers 8" ;;
    e8n) extra="--emulate-peers 8 --emulate-backend nccl" ;;
    e8asp) extra="--emulate-peers 8 --consistency asp" ;;
    *) extra="$b" ;;
  esac
  timeout -k 10 240 python bench.py --steps ${STEPS:-50} --warmup 10 $extra > gpurun_out/bench_$b.log 2>&1
  rc=$?; echo "bench $b rc=$rc"; grep '^{' gpurun_out/bench_$b.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['consistency'])" || tail -5 gpurun_out/bench_$b.log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
