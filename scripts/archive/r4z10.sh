# round 4 (z10): wide & deep: split-K reduces of the weight gradients held to the end of the side stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z10
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PSAMD_WD_DEFER_REDUCE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_deep_gpu.py tests/test_gemm_gpu.py > $O/tests.log 2>&1 || exit $?
W="python benchmarks/bench_wide_deep.py"
for r in 1 2 3; do
timeout -k 10 200 $W > $O/base_$r.log 2>&1 || exit $?
PSAMD_WD_DEFER_REDUCE=1 timeout -k 10 200 $W > $O/defer_$r.log 2>&1 || exit $?
PSAMD_WD_DEFER_REDUCE=1 PSAMD_WD_FUSE=1 timeout -k 10 200 $W > $O/defer_fuse_$r.log 2>&1 || exit $?
done
