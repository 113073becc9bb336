cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5tn; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
true
tail -1 $O/pytest.log
for i in 1 2; do for f in 1 0; do
PSAMD_TN_FUSED_REDUCE=$f timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 > $O/b$f.log 2>&1 || exit 3
grep -h '^{' $O/b$f.log | python -c "import sys,json; [print('wd fused_reduce=$f', round(d['ms_per_step'],4), round(d['host_issue_ms_per_step'],4), d.get('train',{}).get('loss')) for d in map(json.loads, sys.stdin)]"
done; done
