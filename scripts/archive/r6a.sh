#!/bin/bash
# round 6: changed-path GPU tests, 20-step headline, populated-table headline (5e8 / 1e9 keys)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6a
timeout -k 10 400 python -u -m pytest tests/test_tpf_gpu.py tests/test_dist_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "csr or merged_exchange_caller or protocol" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1 || exit $?
grep '^{' $O/b20.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > $O/b200.log 2>&1 || exit $?
grep '^{' $O/b200.log | cut -c1-200
for p in 5e8 1e9; do
  timeout -k 10 400 python bench.py --steps 200 --warmup 10 --prefill $p > $O/prefill_$p.log 2>&1 || exit $?
  grep -v '^{' $O/prefill_$p.log | tail -3; grep '^{' $O/prefill_$p.log | cut -c1-200
done
