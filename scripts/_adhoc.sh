cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for n in 2 4 8; do
timeout -k 10 240 python bench.py --steps 300 --warmup 10 --emulate-peers $n --emulate-backend nccl > gpurun_out/e${n}n.log 2>&1; echo "e${n}n rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e${n}n.log
done
bash scripts/baseline_configs.sh > gpurun_out/bc.out 2>&1; echo "baseline rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/profe8n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --emulate-peers 8 --emulate-backend nccl > "$GRAFT_REPO_ROOT/gpurun_out/profe8n.log" 2>&1; echo prof rc=$?
