#!/bin/bash
# round 6: tail-filter profile (bucket-only ordering), pipeline parity (RCCL loopback G2, flat
# tail), graph-runtime knobs at 8 emulated peers, merged asp lead, cached app at 8 M rows
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4))")"; }
run b20 --steps 20 --warmup 5 || exit 1
run base300 --steps 300 --warmup 10 || exit 1
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run e8tail --steps 100 --warmup 10 --emulate-peers 8 --tail-freq 1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_tail -o run -- python $R/bench.py --steps 100 --warmup 10 --tail-freq 1 > $O/p_tail.log 2>&1 || exit 6
echo "== tail"; python $R/scripts/kbusy_db.py $O/p_tail/run_results.db tp_fwd_bwd 40 100
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_base -o run -- python $R/bench.py --steps 100 --warmup 10 > $O/p_base.log 2>&1 || exit 6
echo "== base"; python $R/scripts/kbusy_db.py $O/p_base/run_results.db tp_fwd_bwd 40 100
cd $R
timeout -k 10 600 python -u -m pytest tests/test_bench_pipeline_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "rccl or test_flat_pipeline" > $O/pytest_pipe.log 2>&1
echo "pytest pipe rc=$?"; grep -E "PASSED|FAILED" $O/pytest_pipe.log | sed 's/.*:://' | head -20
run e8 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 run e8pc1 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run e8pc0 --steps 100 --warmup 10 --emulate-peers 8
DEBUG_HIP_GRAPH_BATCH_SIZE=64 run e8bs64 --steps 100 --warmup 10 --emulate-peers 8
HIP_FORCE_DEV_KERNARG=1 run e8kern --steps 100 --warmup 10 --emulate-peers 8
PSAMD_MX_G2=1 run e8g2 --steps 100 --warmup 10 --emulate-peers 8
PSAMD_XD=1 run e8aspm2x1 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --exchange-merge on --exchange-lag 2
run e8aspm3 --steps 100 --warmup 10 --emulate-peers 8 --consistency asp --algo sgd --fixing-float 2 --exchange-merge on --exchange-lag 3
timeout -k 10 600 python benchmarks/bench_app.py --rows 8000000 --files 8 --minibatch 65536 > $O/app8m.log 2>&1; echo "app rc=$?"; tail -1 $O/app8m.log
