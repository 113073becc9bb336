# round 4 (x): the unrolled generator loop: generator tests, benches, sequential kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4x
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit $?; done
timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1
