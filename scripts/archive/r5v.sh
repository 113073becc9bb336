cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5v; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/e8 -o run -- python $R/bench.py --steps 60 --warmup 10 --emulate-peers 8 --emulate-backend nccl > $O/e8.log 2>&1 || exit 6
python $R/scripts/kbusy_db.py $O/e8/run_results.db tp_fwd_bwd 20 60
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b1 -o run -- python $R/bench.py --steps 60 --warmup 10 > $O/b1.log 2>&1 || exit 7
python $R/scripts/kbusy_db.py $O/b1/run_results.db tp_fwd_bwd 20 60
