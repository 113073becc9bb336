cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
TESTS="tests/test_gemm256_gpu.py" bash scripts/gpu_quick.sh || exit 1
timeout -k 10 200 python benchmarks/bench_gemm256.py > gpurun_out/g256.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/g256.log | tail -8
