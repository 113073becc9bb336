cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5darlin; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 3 --data groups --tau 8 > $O/groups_t8.log 2>&1 || exit 3
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $R/benchmarks/bench_darlin.py --rows 4000000 --passes 2 --data groups --tau 8 > $O/prof.log 2>&1 || exit 4
python $R/scripts/kbusy_db.py $O/prof/run_results.db bcd_objective 1 2 > $O/kbusy.log 2>&1; cat $O/kbusy.log
