cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
TESTS="tests/test_gemm256_gpu.py tests/test_gemm_gpu.py tests/test_wide_deep_gpu.py" bash scripts/gpu_quick.sh || exit 1
timeout -k 10 200 python benchmarks/bench_wide_deep.py --steps 20 --warmup 5 --gemm mfma > gpurun_out/wd_mfma.log 2>&1; echo wd rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/wd_mfma.log
timeout -k 10 200 python benchmarks/bench_wide_deep.py --steps 20 --warmup 5 > gpurun_out/wd_auto.log 2>&1; echo wd rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/wd_auto.log
