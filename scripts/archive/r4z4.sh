# round 4 (z4): wide & deep step: kernel breakdown, localisation / graph A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z4
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_base.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py --localize part > $O/wd_part.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py --graph 1 > $O/wd_graph.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/wd_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_wide_deep.py" --steps 20 > "$GRAFT_REPO_ROOT/$O/wd_prof.log" 2>&1
