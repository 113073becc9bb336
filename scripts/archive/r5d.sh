cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5d
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_train_quality_gpu.py tests/test_trainer_gpu.py tests/test_wide_deep_gpu.py \
  tests/test_dist_gpu.py tests/test_gpu_ops.py -m gpu > gpurun_out/r5d/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5d/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  for e in 8 2; do
    PSAMD_OWNER_FUSED=$f timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers $e > gpurun_out/r5d/e${e}_f$f.log 2>&1 || exit 3
    grep '^{' gpurun_out/r5d/e${e}_f$f.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('e$e fused=$f', d['value']/1e6, d['ms_per_step'])"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5d/prof_e8" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/gpurun_out/r5d/prof_e8.log" 2>&1
echo "prof e8 rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5d/prof_csr" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_csr.py" --minibatch 1000 10000 --steps 50 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/r5d/prof_csr.log" 2>&1
echo "prof csr rc=$?"
