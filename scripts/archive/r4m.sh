# round 4 (m): full GPU suite after the bucket-major toff + generator change, benches, profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4m
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
step timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1
step timeout -k 10 120 python benchmarks/micro/tpf_step_probe.py > $O/probe.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1
