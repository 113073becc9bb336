cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5h
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4))"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_owner_apply_gpu.py tests/test_bench_pipeline_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
for m in on off on; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --exchange-merge $m > $O/e8_$m.log 2>&1 || exit 3; j $O/e8_$m.log "e8 merge=$m"
done
cd /tmp
for lg in 9 8 10; do
  PSAMD_APPLY_LGP=$lg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_e8_lg$lg -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 --emulate-peers 8 > $O/seq_e8_lg$lg.log 2>&1 || exit 6
  python $R/scripts/kbusy_db.py $O/seq_e8_lg$lg/run_results.db tp_fwd_bwd 20 60 | grep -E "steps|apply_part|resolve_rows"
done
echo rc=0
