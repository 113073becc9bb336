# round 4 (z): 8 emulated peers through the RCCL loopback: graph-mixing support off / group launch mode
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bench_pipeline_gpu.py > $O/pipe_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_nccl.log 2>&1 || exit $?
NCCL_GRAPH_MIXING_SUPPORT=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_nomix.log 2>&1 || exit $?
NCCL_LAUNCH_MODE=GROUP timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_group.log 2>&1 || exit $?
NCCL_GRAPH_MIXING_SUPPORT=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_nomix2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_nccl2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --ssp-apply pre > $O/e8_pre.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend copy --ssp-apply pre > $O/e8_copy_pre.log 2>&1 || exit $?
export NCCL_GRAPH_MIXING_SUPPORT=0
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/nomix_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/$O/nomix_prof.log" 2>&1
