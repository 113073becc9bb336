cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5u; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  (cd $R/old_r4 && timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/old_asp_$i.log 2>&1) || exit 3; j $O/old_asp_$i.log "r4tree e8 asp1"
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp --fixing-float 1 > $O/new_asp_$i.log 2>&1 || exit 3; j $O/new_asp_$i.log "r5tree e8 asp1"
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl > $O/new_ssp_$i.log 2>&1 || exit 3; j $O/new_ssp_$i.log "r5tree e8 ssp4 (merged)"
done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl --exchange-merge off > $O/new_sspoff.log 2>&1 || exit 3; j $O/new_sspoff.log "r5tree e8 ssp4 two-collective"
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 2 --emulate-backend nccl > $O/new_e2.log 2>&1 || exit 3; j $O/new_e2.log "r5tree e2 ssp4 (merged)"
