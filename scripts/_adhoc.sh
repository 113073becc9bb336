cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS="tests/test_tploc_gpu.py" bash scripts/gpu_quick.sh || exit 1
PSAMD_LOC_MODES=sort,tp timeout -k 10 120 python benchmarks/bench_localize.py > gpurun_out/loc.log 2>&1; echo loc rc=$?; grep '^{' gpurun_out/loc.log
cd /tmp && PSAMD_LOC_MODES=tp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/proftp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_localize.py > $GRAFT_REPO_ROOT/gpurun_out/proftp.log 2>&1; echo prof rc=$?
cd $GRAFT_REPO_ROOT && BENCHES="--localize=tp" bash scripts/gpu_quick.sh || exit 1
