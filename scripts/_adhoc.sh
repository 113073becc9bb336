cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl > gpurun_out/e8n_$i.log 2>&1; echo "e8n rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_$i.log
done
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 > gpurun_out/e8.log 2>&1; echo "e8 copy rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8.log
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency asp > gpurun_out/e8n_asp.log 2>&1; echo "e8n asp rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_asp.log
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl --consistency ssp:1 > gpurun_out/e8n_ssp1.log 2>&1; echo "e8n ssp1 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_ssp1.log
PSAMD_PREP_STREAMS=3 timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl --prep-streams 3 > gpurun_out/e8n_p3.log 2>&1; echo "e8n p3 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_p3.log
