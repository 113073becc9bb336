cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for p in 1 0; do
PSAMD_NCCL_HIGH_PRIO=$p timeout -k 10 240 python bench.py --steps 300 --warmup 10 --emulate-peers 8 > gpurun_out/e8n_p${p}_$i.log 2>&1; echo "e8n prio=$p rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_p${p}_$i.log
done; done
timeout -k 10 240 python bench.py --steps 300 --warmup 10 --emulate-peers 8 --consistency asp --fixing-float 1 > gpurun_out/e8n_asp.log 2>&1; echo "e8n asp ff1 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_asp.log
