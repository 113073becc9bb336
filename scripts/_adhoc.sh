cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k rehearsal_json > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/pytest_q.log
