# round 4 (d): LaunchList event diagnostic, GEMM ring variant check, the flat-path benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
# a python exception (rc 1) does not stop the script; a timeout / signal / abort does
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 120 python scripts/archive/diag_launchlist.py > $O/diag.log 2>&1
step timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gemm.log 2>&1
for i in 1 2; do
  step timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_native_$i.log 2>&1
  step env PSAMD_NATIVE_ITER=0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_flat_eager_$i.log 2>&1
  step env PSAMD_FLAT=0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_compact_$i.log 2>&1
done
step env PSAMD_STEP_EVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_native_stepev.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_native.log 2>&1
step env PSAMD_NATIVE_ITER=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_flat_eager.log 2>&1
step env PSAMD_FLAT=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_compact.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b300_b10k.log 2>&1
step env PSAMD_FLAT=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b300_b10k_compact.log 2>&1
step timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1
step env PSAMD_FLAT=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_compact.log 2>&1
step timeout -k 10 300 python benchmarks/bench_gemm256.py > $O/gemm256.log 2>&1
for t in 0 1; do
  step timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 $t > $O/darlin_t32_$t.log 2>&1
done
step timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --data groups --tau 8 > $O/darlin_groups_tau8.log 2>&1
step timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --data groups --tau 1 > $O/darlin_groups_tau1.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1
