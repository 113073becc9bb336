cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2 3; do
  PSAMD_STEP_EVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a/b20_$i.log 2>&1 || exit $?
done
timeout -k 10 120 python bench.py --steps 300 --warmup 10 > gpurun_out/r4a/b300.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r4a/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r4a/prof.log" 2>&1
