# round 4 (z6): wide & deep A/B on one box: fused wide gradient + fused wide update (default) vs
# separate passes (PSAMD_WD_FUSE=0), batched cross kernel, transposed-weight layer-0 input gradient
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z6
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_deep_gpu.py > $O/wd_tests.log 2>&1 || exit $?
W="python benchmarks/bench_wide_deep.py"
for r in 1 2; do
timeout -k 10 200 $W > $O/fuse_$r.log 2>&1 || exit $?
PSAMD_WD_FUSE=0 timeout -k 10 200 $W > $O/nofuse_$r.log 2>&1 || exit $?
PSAMD_CROSS_BATCH=1 timeout -k 10 200 $W > $O/crossb_$r.log 2>&1 || exit $?
PSAMD_DX_WT=1 timeout -k 10 200 $W > $O/dxwt_$r.log 2>&1 || exit $?
PSAMD_WD_FUSE=0 PSAMD_DX_WT=1 timeout -k 10 200 $W > $O/nofuse_dxwt_$r.log 2>&1 || exit $?
done
