cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), d['config'].get('collectives_per_step'))"; }
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5e/b1_$i.log 2>&1 || exit 3; j gpurun_out/r5e/b1_$i.log "1gpu-20"
done
for m in on off on off; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 8 --exchange-merge $m > gpurun_out/r5e/e8_$m.log 2>&1 || exit 3; j gpurun_out/r5e/e8_$m.log "e8 merge=$m"
done
for m in on off; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --emulate-peers 2 --exchange-merge $m > gpurun_out/r5e/e2_$m.log 2>&1 || exit 3; j gpurun_out/r5e/e2_$m.log "e2 merge=$m"
done
for cfg in "0 2" "1 2" "1 3" "0 3"; do set -- $cfg
  PSAMD_NATIVE_ITER=$1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams $2 > gpurun_out/r5e/b10k_n$1_p$2.log 2>&1 || exit 4; j gpurun_out/r5e/b10k_n$1_p$2.log "B10k native=$1 prep=$2"
done
timeout -k 10 400 python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200 > gpurun_out/r5e/csr.log 2>&1; echo "csr rc=$?"; cut -c1-330 gpurun_out/r5e/csr.log | grep '^{'
timeout -k 10 400 python benchmarks/bench_app.py --rows 1000000 --files 8 --minibatch 65536 --kind criteo > gpurun_out/r5e/app_criteo.log 2>&1; echo "app rc=$?"; grep '^{' gpurun_out/r5e/app_criteo.log
timeout -k 10 400 python benchmarks/bench_app.py --rows 400000 --files 8 --minibatch 10000 --kind rcv1 > gpurun_out/r5e/app_rcv1.log 2>&1; echo "app rc=$?"; grep '^{' gpurun_out/r5e/app_rcv1.log
