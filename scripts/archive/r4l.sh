# round 4 (l): 8 emulated peers, kernel profiles (pipelined default + sequential)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/e8" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/$O/e8.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/e8_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/e8_seq.log" 2>&1
