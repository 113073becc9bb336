cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5t; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/old -o run -- python $R/old_r4/bench.py --steps 60 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/old.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run -- python $R/bench.py --steps 60 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/new.log 2>&1 || exit 7
for t in old new; do echo "== $t"; python $R/scripts/kbusy_db.py $O/$t/run_results.db tp_fwd_bwd 20 60; done
