cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS="tests/test_partloc_gpu.py tests/test_bench_pipeline_gpu.py" BENCHES="e8 1 --localize=part" bash scripts/gpu_quick.sh || exit 1
timeout -k 10 200 python bench.py --emulate-peers 8 --localize part --steps 50 --warmup 10 > gpurun_out/e8_part.log 2>&1; echo e8part rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8_part.log
