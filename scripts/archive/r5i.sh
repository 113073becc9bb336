cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/bench_owner.py --lgp 9 10 --fresh 12 --capacity 134217728 2147483648 > $O/owner2.log 2>&1; grep '^{' $O/owner2.log; tail -3 $O/owner2.log
