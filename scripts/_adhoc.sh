cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_darlin_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_darlin.py > gpurun_out/darlin.log 2>&1; echo "darlin rc=$?"; tail -3 gpurun_out/darlin.log
