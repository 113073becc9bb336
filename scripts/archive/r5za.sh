cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5za; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py tests/test_owner_apply_gpu.py tests/test_dist_gpu.py tests/test_tploc_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl > $O/e8_$i.log 2>&1 || exit 3; j $O/e8_$i.log "e8"
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 2 --emulate-backend nccl > $O/e2_$i.log 2>&1 || exit 3; j $O/e2_$i.log "e2"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_e8 -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 --emulate-peers 8 > $O/seq_e8.log 2>&1 || exit 6
python $R/scripts/kbusy_db.py $O/seq_e8/run_results.db tp_fwd_bwd 20 60
