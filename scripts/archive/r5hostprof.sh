cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5hostprof; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -m cProfile -o $O/e8.prof bench.py --emulate-peers 8 --steps 2000 --warmup 10 > $O/e8.log 2>&1 || exit 3
grep '^{' $O/e8.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_issue_ms_per_step'])"
python - <<PY
import pstats
p = pstats.Stats('$O/e8.prof')
p.sort_stats('tottime').print_stats(30)
PY
