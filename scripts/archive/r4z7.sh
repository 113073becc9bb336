# round 4 (z7): wide & deep weight gradients through hipBLASLt vs the 256x256 TN kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z7
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
W="python benchmarks/bench_wide_deep.py"
for r in 1 2; do
timeout -k 10 200 $W > $O/base_$r.log 2>&1 || exit $?
PSAMD_DW_LIB=1 timeout -k 10 200 $W > $O/dwlib_$r.log 2>&1 || exit $?
PSAMD_DW_LIB=1 PSAMD_DX_WT=1 timeout -k 10 200 $W > $O/dwlib_dxwt_$r.log 2>&1 || exit $?
done
