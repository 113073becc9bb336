#!/bin/bash
# round 6: batched sketch atomics (filter tests + tail benches), HIP graph-runtime knobs sweep
# at 8 / 2 emulated peers, cached app at 8 M rows
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_tpf_gpu.py tests/test_gpu_ops.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "tail_filter or countmin" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4))")"; }
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
for pc in 1 0; do for bs in 0 4 16 64; do for g2 in 0 1; do
  if [ $bs = 0 ]; then DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc PSAMD_MX_G2=$g2 run e8_pc${pc}_bs${bs}_g$g2 --steps 100 --warmup 10 --emulate-peers 8
  else DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc DEBUG_HIP_GRAPH_BATCH_SIZE=$bs PSAMD_MX_G2=$g2 run e8_pc${pc}_bs${bs}_g$g2 --steps 100 --warmup 10 --emulate-peers 8; fi
done; done; done
timeout -k 10 400 python -u -m pytest tests/test_train_quality_gpu.py -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "e8asp2m3" > $O/pytest_tq.log 2>&1
echo "pytest tq rc=$?"; grep -E "PASSED|FAILED|SKIPPED|^E " $O/pytest_tq.log | head -10
run c4ftrl --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --fixing-float 1
run c4ftrlm3 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --fixing-float 1 --exchange-merge on --exchange-lag 3
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run e2_pc0 --steps 100 --warmup 10 --emulate-peers 2
run e2_pc1 --steps 100 --warmup 10 --emulate-peers 2
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 > $O/app8m.log 2>&1; echo "app rc=$?"; tail -1 $O/app8m.log
