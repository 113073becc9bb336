cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5l; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
for p in 2 3 4; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams $p > $O/b10k_p$p.log 2>&1 || exit 3; j $O/b10k_p$p.log "B10k prep=$p"
done
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 --kind ctr unique > $O/csr.log 2>&1 && cut -c1-330 $O/csr.log | grep '^{'
for m in on off; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --minibatch 10000 --exchange-merge $m > $O/e8b10k_$m.log 2>&1 || exit 3; j $O/e8b10k_$m.log "e8 B10k merge=$m"
done
echo rc=$?
