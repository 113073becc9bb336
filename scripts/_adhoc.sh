cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
PSAMD_XD=3 timeout -k 10 500 python -u -m pytest tests/test_bench_pipeline_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests xd3 rc=$rc"; tail -2 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for x in 2 3; do
PSAMD_XD=$x timeout -k 10 240 python bench.py --steps 300 --warmup 10 --emulate-peers 8 > gpurun_out/e8n_xd${x}_$i.log 2>&1; echo "e8n xd=$x rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_xd${x}_$i.log
done; done
