# round 4 (z8): wide & deep: weight gradients on a side stream (default) vs in line, x fused passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z8
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
W="python benchmarks/bench_wide_deep.py"
for r in 1 2; do
timeout -k 10 200 $W > $O/base_$r.log 2>&1 || exit $?
timeout -k 10 200 $W --overlap-wgrad 0 > $O/inline_$r.log 2>&1 || exit $?
PSAMD_WD_FUSE=1 timeout -k 10 200 $W --overlap-wgrad 0 > $O/inline_fuse_$r.log 2>&1 || exit $?
PSAMD_WD_FUSE=1 timeout -k 10 200 $W > $O/fuse_$r.log 2>&1 || exit $?
done
