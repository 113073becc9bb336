#!/bin/bash
# round 6: 1e10 slowdown (tile / fwd-bwd co-scheduling), tile gate A/B, filter profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
for g in 0 1; do
  for nf in 1e9 1e10; do
    PSAMD_TILE_GATE=$g timeout -k 10 200 python bench.py --steps 300 --warmup 10 --num-features $nf > $O/b_${nf}_g$g.log 2>&1 || exit 3; j $O/b_${nf}_g$g.log "gate=$g nf=$nf 300"
    PSAMD_TILE_GATE=$g timeout -k 10 200 python bench.py --steps 20 --warmup 5 --num-features $nf > $O/b20_${nf}_g$g.log 2>&1 || exit 3; j $O/b20_${nf}_g$g.log "gate=$g nf=$nf 20"
  done
done
cd /tmp
for g in 0 1; do
for nf in 1e9 1e10; do
  PSAMD_TILE_GATE=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_${nf}_g$g -o run -- python $R/bench.py --steps 100 --warmup 10 --num-features $nf > $O/p_${nf}_g$g.log 2>&1 || exit 6
  echo "== gate $g $nf"; python $R/scripts/kbusy_db.py $O/p_${nf}_g$g/run_results.db tp_fwd_bwd 40 100
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_tail -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_tail.log 2>&1 || exit 6
echo "== tail"; python $R/scripts/kbusy_db.py $O/p_tail/run_results.db tp_fwd_bwd 40 100
cd $R
timeout -k 10 600 python -u -m pytest tests/test_bench_pipeline_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "rccl or test_flat_pipeline" > $O/pytest_pipe.log 2>&1
echo "pytest pipe rc=$?"; grep -E "PASSED|FAILED" $O/pytest_pipe.log | sed 's/.*:://' | head -20
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'), d['config'].get('native_iteration'), d['train'].get('loss'))")"; }
run e8 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 run e8pc1 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run e8pc0 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_HIP_GRAPH_BATCH_SIZE=64 run e8bs64 --steps 100 --warmup 10 --emulate-peers 8
HIP_FORCE_DEV_KERNARG=1 run e8kern --steps 100 --warmup 10 --emulate-peers 8
PSAMD_XD=1 run e8aspm2x1 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --exchange-merge on --exchange-lag 2
run e8aspm3 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --exchange-merge on --exchange-lag 3
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 > $O/app8m.log 2>&1; echo "app rc=$?"; tail -1 $O/app8m.log
