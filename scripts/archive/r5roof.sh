cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5roof; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
for B in 65536 10000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq$B -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 --minibatch $B > $O/seq$B.log 2>&1 || exit 4
echo "== B=$B sequential"; python $R/scripts/kbreak_db.py $O/seq$B/run_results.db tp_fwd_bwd 20 60
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pip$B -o run -- python $R/bench.py --steps 60 --warmup 10 --minibatch $B > $O/pip$B.log 2>&1 || exit 5
echo "== B=$B pipelined"; python $R/scripts/kbusy_db.py $O/pip$B/run_results.db tp_fwd_bwd 20 60
done
