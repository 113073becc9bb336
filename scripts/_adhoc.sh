cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_tploc_gpu.py tests/test_tp_fused_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
PSAMD_LOC_MODES=tp timeout -k 10 120 python benchmarks/bench_localize.py > gpurun_out/loc30.log 2>&1; echo "loc30 rc=$?"; grep -o '"localize_us": [0-9.]*' gpurun_out/loc30.log
PSAMD_TP_QUOT=1 PSAMD_LOC_MODES=tp timeout -k 10 120 python benchmarks/bench_localize.py > gpurun_out/loc30q.log 2>&1; echo "loc30q rc=$?"; grep -o '"localize_us": [0-9.]*' gpurun_out/loc30q.log
PSAMD_LOC_BITS=34 PSAMD_LOC_MODES=tp timeout -k 10 120 python benchmarks/bench_localize.py > gpurun_out/loc34.log 2>&1; echo "loc34 rc=$?"; grep -o '"localize_us": [0-9.]*' gpurun_out/loc34.log
timeout -k 10 240 python bench.py --steps 300 --warmup 10 --num-features 1e10 > gpurun_out/b1e10.log 2>&1; echo "1e10 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b1e10.log
timeout -k 10 240 python bench.py --steps 300 --warmup 10 > gpurun_out/b1.log 2>&1; echo "1e9 rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b1.log
