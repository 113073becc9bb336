# round 4 (z9): final tree after the exchange / W&D changes: full GPU suite, smoke, headline, 8 emulated peers, W&D
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z9
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit $?; done
timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_wide_deep.py > $O/wd_1.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_wide_deep.py > $O/wd_2.log 2>&1 || exit $?
