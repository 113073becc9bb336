# round 4 (v): lock-step bucket search (tile / fwd-bwd reverted): correctness, device-only probe, benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_tploc_gpu.py tests/test_tpf_gpu.py tests/test_tp_fused_gpu.py tests/test_trainer_gpu.py tests/test_dist_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/micro/tpf_step_probe.py > $O/probe.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || exit $?; done
timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1
