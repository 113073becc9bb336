cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5darlin5; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for w in 0 4 8 32 64 0; do
PSAMD_BCD_FUSED_W=$w timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 3 --data groups --tau 8 > $O/b.log 2>&1 || exit 3
grep -h '^{' $O/b.log | python -c "import sys,json; [print('W=$w', round(d['ms_per_pass'],3), d['train']['objective']) for d in map(json.loads, sys.stdin)]"
done
