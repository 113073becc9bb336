#!/bin/bash
# round 6: graph-chain probe, pipeline parity (tail filter, G2), merged asp training, benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python benchmarks/probe_graph_events.py > $O/probe_ge.log 2>&1; echo "probe rc=$?"; tail -2 $O/probe_ge.log
PROBE_SIDE_K=30 timeout -k 10 120 python benchmarks/probe_graph_events.py > $O/probe_ge30.log 2>&1; echo "probe30 rc=$?"; tail -2 $O/probe_ge30.log
timeout -k 10 700 python -u -m pytest tests/test_bench_pipeline_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "kw27 or kw28 or kw29 or tail or rccl" > $O/pytest_pipe.log 2>&1
rc=$?; echo "pytest pipe rc=$rc"; grep -E "PASSED|FAILED" $O/pytest_pipe.log | sed 's/.*:://' | head -20
timeout -k 10 400 python -u -m pytest tests/test_train_quality_gpu.py -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "e8asp2" > $O/pytest_tq.log 2>&1
rc=$?; echo "pytest tq rc=$rc"; grep -E "PASSED|FAILED|^E " $O/pytest_tq.log | head -20
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'), d['config'].get('localize'), d['config'].get('native_iteration'), d['config'].get('consistency')[:30], d['train'].get('loss'))")"; }
run b20 --steps 20 --warmup 5 || exit 1
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
PSAMD_MX_G2=1 run e8g2 --steps 100 --warmup 10 --emulate-peers 8
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
run e8asp --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 || exit 1
run e8aspm2 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --exchange-merge on --exchange-lag 2 || exit 1
run pf5e8 --steps 200 --warmup 10 --prefill 5e8 || exit 1
run pf1e9 --steps 200 --warmup 10 --prefill 1e9 || exit 1
timeout -k 10 400 python benchmarks/bench_app.py --rows 2000000 --files 8 --minibatch 65536 > $O/app2m.log 2>&1; echo "app rc=$?"; tail -2 $O/app2m.log
