# round 4 (g): overlapped tpf_step2 kernel: bitwise test vs v1, A/B benches, sequential profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_tpf_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
for i in 1 2; do
  step timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_v2_$i.log 2>&1
  step env PSAMD_TPF_STEP_V1=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_v1_$i.log 2>&1
done
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_v2.log 2>&1
step env PSAMD_TPF_STEP_V1=1 timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_v1.log 2>&1
step timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
