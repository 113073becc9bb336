cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5w
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r5w/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5w/smoke.log 2>&1 && tail -2 gpurun_out/r5w/smoke.log &&
timeout -k 10 200 python bench.py > gpurun_out/r5w/bench.log 2>&1 && grep '^{' gpurun_out/r5w/bench.log &&
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 --kind unique rcv1 > gpurun_out/r5w/csr.log 2>&1 && cut -c1-330 gpurun_out/r5w/csr.log | grep '^{'
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --minibatch 10000 > gpurun_out/r5w/e8b10k.log 2>&1 && j gpurun_out/r5w/e8b10k.log "e8 B10k merged"
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > gpurun_out/r5w/b10k.log 2>&1 && j gpurun_out/r5w/b10k.log "B10k"
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5w/b1_$i.log 2>&1 && j gpurun_out/r5w/b1_$i.log "1gpu-20"; done
