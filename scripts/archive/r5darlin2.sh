cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5darlin2; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_darlin_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -3 $O/pytest.log
for a in "--data groups --tau 8" "--data groups --tau 1" "--tau 1"; do
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 3 $a > $O/b.log 2>&1 || exit 3
grep -h '^{' $O/b.log | python -c "import sys,json; [print('$a', round(d['ms_per_pass'],3), d['config']['blocks'], d['train']['objective']) for d in map(json.loads, sys.stdin)]"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $R/benchmarks/bench_darlin.py --rows 4000000 --passes 2 --data groups --tau 8 > $O/prof.log 2>&1 || exit 4
