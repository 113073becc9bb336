cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5f
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r5f/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.log 2>&1 && tail -2 gpurun_out/r5f/smoke.log &&
timeout -k 10 200 python bench.py > gpurun_out/r5f/bench.log 2>&1 && grep '^{' gpurun_out/r5f/bench.log &&
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 --kind unique rcv1 > gpurun_out/r5f/csr.log 2>&1 && cut -c1-330 gpurun_out/r5f/csr.log | grep '^{'
