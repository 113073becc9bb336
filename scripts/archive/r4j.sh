# round 4 (j): Darlin row pass (32-bit offsets) tests + benches; 8 emulated peers eager host issue
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_darlin_gpu.py tests/test_gpu_ops.py tests/test_tpf_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_darlin.log 2>&1
for t in 1 0; do
  step timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 $t > $O/darlin_t32_$t.log 2>&1
done
step env PSAMD_CAPTURE_COMM=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_eager.log 2>&1
step timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b300_b10k.log 2>&1
step timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_darlin" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_darlin.py" --rows 4000000 --passes 3 --device-data --tau32 1 > "$GRAFT_REPO_ROOT/$O/prof_darlin.log" 2>&1
cd "$GRAFT_REPO_ROOT"
step timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_wide_deep_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_wd.log 2>&1
for g in auto mfma; do
  step timeout -k 10 300 python benchmarks/bench_wide_deep.py --gemm $g > $O/wd_$g.log 2>&1
  step env PSAMD_GEMM_NT256=0 timeout -k 10 300 python benchmarks/bench_wide_deep.py --gemm $g > $O/wd_${g}_v0.log 2>&1
done
step env PSAMD_NATIVE_ITER=1 timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 1 > $O/b10k_native_p1.log 2>&1
step env PSAMD_NATIVE_ITER=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 1 > $O/b10k_eager_p1.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 --pipeline 0 > $O/b10k_seq.log 2>&1
