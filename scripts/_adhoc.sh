cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
PSAMD_CAPTURE_COMM=1 timeout -k 10 500 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests capture rc=$rc"; tail -4 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for c in 0 1; do
PSAMD_CAPTURE_COMM=$c timeout -k 10 240 python bench.py --steps 300 --warmup 10 --emulate-peers 8 > gpurun_out/e8n_cc${c}_$i.log 2>&1; rc=$?; echo "e8n capture=$c rc=$rc"; grep -o '"host_issue_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/e8n_cc${c}_$i.log; [ $rc -eq 0 ] || exit $rc
done; done
