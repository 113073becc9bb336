cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5mxt; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py tests/test_train_quality_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('ssp_apply'), d['comm'].get('captured'))"; }
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1 || exit 3; j $O/e8.log "e8 default"
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --consistency asp --fixing-float 1 --emulate-peers 8 > $O/asp.log 2>&1 || exit 3; j $O/asp.log "e8 asp ff1"
