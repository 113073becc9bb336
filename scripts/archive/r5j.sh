cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5j; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
for nat in 0 1; do
  PSAMD_NATIVE_ITER=$nat timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b10k_n$nat -o run -- python $R/bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/b10k_n$nat.log 2>&1 || exit 6
  grep '^{' $O/b10k_n$nat.log | cut -c1-300
  python $R/scripts/kbusy_db.py $O/b10k_n$nat/run_results.db tp_fwd_bwd 100 300
done
echo rc=0
