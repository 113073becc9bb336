# round 4 (c): native-iteration fix check + the r4b benches (PSAMD_FLAT=0 baseline, native iteration on/off) + kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_tpf_gpu.py tests/test_darlin_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r4c/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c/smoke.log 2>&1 || exit $?
for i in 1 2; do
  for v in "PSAMD_FLAT=0" "PSAMD_FLAT=1 PSAMD_NATIVE_ITER=0" "PSAMD_FLAT=1"; do
    tag=$(echo $v | tr ' =' '__')
    env $v PSAMD_STEP_EVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r4c/b20_${tag}_$i.log 2>&1 || exit $?
  done
done
for v in "PSAMD_FLAT=0" "PSAMD_FLAT=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 120 python bench.py --steps 300 --warmup 10 > gpurun_out/r4c/b300_$tag.log 2>&1 || exit $?
done
timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > gpurun_out/r4c/b300_b10k.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > gpurun_out/r4c/e8.log 2>&1 || exit $?
PSAMD_FLAT=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > gpurun_out/r4c/e8_f0.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_gemm256.py > gpurun_out/r4c/gemm256.log 2>&1 || exit $?
for t in 0 1; do
  timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 $t > gpurun_out/r4c/darlin_t32_$t.log 2>&1 || exit $?
done
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --data groups --tau 8 > gpurun_out/r4c/darlin_groups_tau8.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --data groups --tau 1 > gpurun_out/r4c/darlin_groups_tau1.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4c/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r4c/prof.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4c/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/gpurun_out/r4c/prof_seq.log" 2>&1
