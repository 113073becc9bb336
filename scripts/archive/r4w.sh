# round 4 (w): final tree: full GPU suite, smoke, headline (20/5 x3, 300), 8 emulated peers, Darlin, W&D, kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit $?; done
timeout -k 10 120 python bench.py > $O/b_default.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 1 > $O/darlin.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_wide_deep.py --gemm auto > $O/wd_auto.log 2>&1 || exit $?
timeout -k 10 120 python benchmarks/micro/tpf_step_probe.py > $O/probe.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
