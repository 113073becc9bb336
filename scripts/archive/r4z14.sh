# round 4 (z14): last tree: full GPU suite, smoke, driver-shape bench, W&D
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z14
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python benchmarks/bench_wide_deep.py > $O/wd.log 2>&1 || exit $?
