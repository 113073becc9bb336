cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5a
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -k "flat or overflow or fp32" > gpurun_out/r5a/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/b1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > gpurun_out/r5a/e8.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 2 > gpurun_out/r5a/e2.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5a/prof_e8 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --emulate-peers 8 > $GRAFT_REPO_ROOT/gpurun_out/r5a/prof_e8.log 2>&1
echo rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/r5a/pytest.log
