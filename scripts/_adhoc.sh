cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_wide_deep_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python benchmarks/bench_wide_deep.py --steps 30 > gpurun_out/wd_$i.log 2>&1; echo "wd rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/wd_$i.log
done
timeout -k 10 240 python benchmarks/bench_wide_deep.py --steps 30 --emulate-peers 8 > gpurun_out/wd_e8.log 2>&1; echo "wd e8 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/wd_e8.log
