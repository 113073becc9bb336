cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5mxn; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bench_pipeline_gpu.py -k "kw16 or kw23 or kw24" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
grep -E "passed|failed" $O/pytest.log | tail -1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['train']['loss'])"; }
for i in 1 2; do for f in 0 1; do
PSAMD_MX_NATIVE=$f timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 > $O/e8_$f.log 2>&1 || { tail -20 $O/e8_$f.log; exit 3; }; j $O/e8_$f.log "e8 B64k native=$f"
PSAMD_MX_NATIVE=$f timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 2 > $O/e2_$f.log 2>&1 || exit 3; j $O/e2_$f.log "e2 B64k native=$f"
done; done
