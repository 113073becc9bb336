cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5k; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tploc_gpu.py tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py tests/test_gpu_ops.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
for lts in 13 12 11 10 0; do
  PSAMD_TILE_LTS=$lts timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/b10k_l$lts.log 2>&1 || exit 3; j $O/b10k_l$lts.log "B10k lts=$lts native=0"
done
for lts in 13 11 10; do
  PSAMD_TILE_LTS=$lts PSAMD_NATIVE_ITER=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/b10k_nl$lts.log 2>&1 || exit 3; j $O/b10k_nl$lts.log "B10k lts=$lts native=1"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b1.log 2>&1 && j $O/b1.log "1gpu-20" &&
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 --kind rcv1 ctr > $O/csr.log 2>&1 && cut -c1-330 $O/csr.log | grep '^{'
echo rc=$?
