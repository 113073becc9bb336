cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log &&
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 && grep '^{' $O/bench.log | cut -c1-200 &&
timeout -k 10 300 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 --kind unique rcv1 > $O/csr.log 2>&1 && cut -c1-250 $O/csr.log | grep '^{' || exit 5
cd /tmp
for m in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_e8_$m -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 --emulate-peers 8 --exchange-merge $m > $O/seq_e8_$m.log 2>&1 || exit 6
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/seq_b1 -o run -- python $R/bench.py --pipeline 0 --steps 60 --warmup 10 > $O/seq_b1.log 2>&1 || exit 7
echo rc=0
