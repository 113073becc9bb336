cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5z; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
for nf in 1e9 1e10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_$nf -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 --num-features $nf > $O/seq_$nf.log 2>&1 || exit 6
  echo "== $nf"; python $R/scripts/kbusy_db.py $O/seq_$nf/run_results.db tp_fwd_bwd 20 60
done
