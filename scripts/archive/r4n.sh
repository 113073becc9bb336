# round 4 (n): full GPU suite (bucket-major toff, 6-wave generator, Darlin 32-bit offsets,
# ring GEMM for W&D), then the benches in priority order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
step timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for i in 1 2 3; do
  step timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1
done
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1
step timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 1 > $O/darlin_t32_1.log 2>&1
step timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1
step env PSAMD_CAPTURE_COMM=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_eager.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b10k.log 2>&1
step env PSAMD_NATIVE_ITER=1 timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 1 > $O/b10k_native_p1.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 --pipeline 0 > $O/b10k_seq.log 2>&1
for g in auto mfma; do
  step timeout -k 10 300 python benchmarks/bench_wide_deep.py --gemm $g > $O/wd_$g.log 2>&1
done
step env PSAMD_GEMM_NT256=0 timeout -k 10 300 python benchmarks/bench_wide_deep.py --gemm mfma > $O/wd_mfma_v0.log 2>&1
step timeout -k 10 120 python benchmarks/micro/tpf_step_probe.py > $O/probe.log 2>&1
step timeout -k 10 200 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data --tau32 0 > $O/darlin_t32_0.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/e8prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --emulate-peers 8 > "$GRAFT_REPO_ROOT/$O/e8prof.log" 2>&1
