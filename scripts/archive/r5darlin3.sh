cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5darlin3; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_darlin_gpu.py tests/test_app_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
for h in "" 1024; do
for a in "--data groups --tau 8"; do
PSAMD_BCD_HOT=$h timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 3 $a > $O/b.log 2>&1 || exit 3
grep -h '^{' $O/b.log | python -c "import sys,json; [print('hot=$h $a', round(d['ms_per_pass'],3), d['config']['blocks'], d['train']['objective']) for d in map(json.loads, sys.stdin)]"
done; done
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 3 --data groups --tau 1 > $O/b.log 2>&1 || exit 3
grep -h '^{' $O/b.log | python -c "import sys,json; [print('tau1 groups', round(d['ms_per_pass'],3), d['train']['objective']) for d in map(json.loads, sys.stdin)]"
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --tau 1 > $O/b.log 2>&1 || exit 3
grep -h '^{' $O/b.log | python -c "import sys,json; [print('tau1 criteo', round(d['ms_per_pass'],3), d['train']['objective']) for d in map(json.loads, sys.stdin)]"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $R/benchmarks/bench_darlin.py --rows 4000000 --passes 2 --data groups --tau 8 > $O/prof.log 2>&1 || exit 4
python $R/scripts/kbreak_db.py $O/prof/run_results.db
