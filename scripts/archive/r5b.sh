cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_tpf_gpu.py > gpurun_out/r5b/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5b/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in on off; do
  for e in 8 2; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers $e --exchange-merge $m > gpurun_out/r5b/e${e}_$m.log 2>&1 || exit 3
    grep '^{' gpurun_out/r5b/e${e}_$m.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('e$e $m', d['value']/1e6, d['ms_per_step'], d['config']['consistency'][:60])"
  done
done
for g in 1 0 1 0; do  # (PSAMD_PREP_GATE)
  PSAMD_PREP_GATE=$g timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5b/b1_gate$g.log 2>&1 || exit 4
  grep '^{' gpurun_out/r5b/b1_gate$g.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('b1 gate $g', d['value']/1e6, d['ms_per_step'])"
done
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 > gpurun_out/r5b/csr.log 2>&1; cat gpurun_out/r5b/csr.log | cut -c1-300
