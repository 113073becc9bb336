# round 4 (z5): wide & deep with the wide gradient fused into the embedding segment reduction
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z5
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wide_deep_gpu.py tests/test_fm_gpu.py > $O/wd_tests.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_a.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py --localize part > $O/wd_part.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_b.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/wd_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_wide_deep.py" --steps 20 > "$GRAFT_REPO_ROOT/$O/wd_prof.log" 2>&1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PSAMD_DX_WT=1 timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_dxwt.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_c.log 2>&1 || exit $?
PSAMD_DX_WT=1 timeout -k 10 200 python benchmarks/bench_wide_deep.py > $O/wd_dxwt2.log 2>&1 || exit $?
