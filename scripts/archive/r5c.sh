# full GPU suite + smoke + kernel profiles of the merged 8-peer step and the 1-GPU step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r5c/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c/smoke.log 2>&1 || exit 5
tail -2 gpurun_out/r5c/smoke.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5c/prof_e8m" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/gpurun_out/r5c/prof_e8m.log" 2>&1
echo "prof rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5c/prof_csr" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_csr.py" --minibatch 1000 10000 --steps 50 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/r5c/prof_csr.log" 2>&1
echo "prof csr rc=$?"
