cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_owner_split_gpu.py tests/test_bench_pipeline_gpu.py tests/test_dist_gpu.py tests/test_wide_deep_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --emulate-backend nccl > gpurun_out/e8n_$i.log 2>&1; echo "e8n rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_$i.log
done
for m in sort part; do
timeout -k 10 240 python benchmarks/bench_wide_deep.py --steps 30 --localize $m > gpurun_out/wd_$m.log 2>&1; echo "wd $m rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/wd_$m.log
timeout -k 10 240 python benchmarks/bench_fm.py --steps 30 --minibatch 65536 --localize $m > gpurun_out/fm_$m.log 2>&1; echo "fm $m rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/fm_$m.log
done
for a in stream tail; do
PSAMD_ASP_APPLY=$a timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --consistency asp > gpurun_out/asp_$a.log 2>&1; echo "asp $a rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/asp_$a.log
PSAMD_ASP_APPLY=$a timeout -k 10 240 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --consistency asp --fixing-float 1 > gpurun_out/asp_ff_$a.log 2>&1; echo "asp ff1 $a rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/asp_ff_$a.log
done
