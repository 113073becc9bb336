# round 4 (i): tile-count balance probe (256 vs 313 tiles) under kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp && for b in 53760 65536 32768; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tb_$b" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/micro/tile_balance_probe.py" $b > "$GRAFT_REPO_ROOT/$O/tb_$b.log" 2>&1 || exit $?
done
