# round 4 (y): 8 emulated peers: RCCL loopback vs device copies, captured vs eager collectives, graphs off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_nccl.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend copy > $O/e8_copy.log 2>&1 || exit $?
PSAMD_CAPTURE_COMM=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_eagercomm.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --graph 0 > $O/e8_nograph.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/e8copy_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 --emulate-backend copy > "$GRAFT_REPO_ROOT/$O/e8copy_prof.log" 2>&1
