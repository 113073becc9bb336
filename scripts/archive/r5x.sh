cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5x; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'))"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bench_pipeline_gpu.py -k flat_pipeline > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
for p in 2 3 4; do
  PSAMD_ITER_GRAPH=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams $p > $O/g_p$p.log 2>&1 || exit 3; j $O/g_p$p.log "B10k itergraph prep=$p"
done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/e_p3.log 2>&1 || exit 3; j $O/e_p3.log "B10k eager prep=3"
for B in 20000 32768 65536; do
  PSAMD_ITER_GRAPH=1 PSAMD_NATIVE_ITER=0 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --minibatch $B > $O/g_$B.log 2>&1 || exit 3; j $O/g_$B.log "B$B itergraph"
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --minibatch $B > $O/d_$B.log 2>&1 || exit 3; j $O/d_$B.log "B$B default"
done
