# round 4 (s): multi-peer path after batching the pack / unpack / apply loads
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4s
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_p2p_gpu.py tests/test_train_quality_gpu.py tests/test_bench_pipeline_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 4 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 4 > $O/e4.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 2 > $O/e2.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/e8prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/$O/e8prof.log" 2>&1
